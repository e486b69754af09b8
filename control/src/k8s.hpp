// Kubernetes API client: kubeconfig loading (explicit file, $KUBECONFIG,
// ~/.kube/config, in-cluster service account) and typed REST verbs.
//
// Native C++ equivalent of the reference's L1 "K8s client plumbing"
// (src/k8s/mod.rs:24-37 of isgasho/h2o-kubernetes: from_kubeconfig /
// try_default) plus the kube::Api<T> create/delete/watch calls it used
// (src/k8s/mod.rs:97-100,114-117,134-157,169-179).
#pragma once

#include <functional>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "http.hpp"
#include "json.hpp"

namespace h2ok {

// users[].user.exec: a client.authentication.k8s.io credential plugin (EKS
// `aws eks get-token`, GKE `gke-gcloud-auth-plugin`, AKS `kubelogin`, ...)
struct ExecPlugin {
  std::string api_version = "client.authentication.k8s.io/v1";
  std::string command;
  std::vector<std::string> args;
  std::vector<std::pair<std::string, std::string>> env;
  std::string install_hint;
  bool provide_cluster_info = false;
  std::string base_dir;  // kubeconfig directory: relative command paths resolve here
};

// users[].user.auth-provider (legacy): oidc id-token, gcp access-token / cmd-path
struct AuthProvider {
  std::string name;
  Json config;
  std::string base_dir;
};

struct KubeConfig {
  std::string server;          // https://host:port[/base]
  TlsConfig tls;
  std::string token;           // bearer token
  std::string username, password;
  std::string ns = "default";  // context namespace (kubeconfig default)
  std::string source;          // kubeconfig path ("" = in-cluster)
  std::string context;
  std::optional<ExecPlugin> exec;
  std::optional<AuthProvider> auth_provider;
};

// ExecCredential.status returned by a plugin (PEM strings, RFC 3339 expiry)
struct ExecCredential {
  std::string token, client_cert_pem, client_key_pem;
  long long expires_at = 0;  // unix seconds, 0 = does not expire
};
// Run an exec plugin (fork/exec, KUBERNETES_EXEC_INFO in its environment) and
// parse its ExecCredential; throws KubeConfigError with the plugin's stderr.
ExecCredential run_exec_plugin(const ExecPlugin& p, const KubeConfig& cluster);
// Bearer token of a legacy auth-provider (runs gcp's cmd-path when needed).
std::string auth_provider_token(const AuthProvider& a);

class KubeConfigError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// Load an explicit kubeconfig file (optionally a named context).
KubeConfig load_kubeconfig(const std::string& path, const std::string& context = "");
// Config::infer() order: $KUBECONFIG (first existing entry), ~/.kube/config,
// then the in-cluster service account.  Throws KubeConfigError if none works.
KubeConfig infer_kubeconfig();
KubeConfig in_cluster_config();

struct ResourceKind {
  std::string api;     // "/api/v1" or "/apis/<group>/<version>"
  std::string plural;  // "services"
  std::string kind;    // "Service"
  bool namespaced = true;
};

namespace kinds {
extern const ResourceKind Service;
extern const ResourceKind StatefulSet;
extern const ResourceKind IngressV1;
extern const ResourceKind IngressV1beta1;
extern const ResourceKind Pod;
extern const ResourceKind H2O;       // h2o.ai/v1beta  h2os
extern const ResourceKind TraefikMiddleware;         // traefik.io/v1alpha1 middlewares (Traefik >= 2.10)
extern const ResourceKind TraefikMiddlewareLegacy;   // traefik.containo.us/v1alpha1 (earlier Traefik v2)
extern const ResourceKind CRD;
extern const ResourceKind IngressClass;              // networking.k8s.io/v1 ingressclasses (cluster-scoped)
}  // namespace kinds

class ApiError : public std::runtime_error {
 public:
  ApiError(int status, std::string reason, std::string message, std::string body)
      : std::runtime_error("Kubernetes API error " + std::to_string(status) + " " + reason + ": " + message),
        status(status), reason(std::move(reason)), message(std::move(message)), body(std::move(body)) {}
  int status;
  std::string reason, message, body;
};

struct WatchEvent {
  std::string type;  // ADDED | MODIFIED | DELETED | BOOKMARK | ERROR
  Json object;
};

class KubeClient {
 public:
  explicit KubeClient(KubeConfig cfg);
  const KubeConfig& config() const { return cfg_; }
  const std::string& default_namespace() const { return cfg_.ns; }

  Json create(const ResourceKind& k, const std::string& ns, const Json& body);
  Json get(const ResourceKind& k, const std::string& ns, const std::string& name);
  std::optional<Json> get_opt(const ResourceKind& k, const std::string& ns, const std::string& name);
  Json list(const ResourceKind& k, const std::string& ns, const std::string& label_selector = "",
            const std::string& field_selector = "");
  Json remove(const ResourceKind& k, const std::string& ns, const std::string& name,
              const std::string& propagation = "");
  Json replace(const ResourceKind& k, const std::string& ns, const std::string& name, const Json& body);
  Json merge_patch(const ResourceKind& k, const std::string& ns, const std::string& name, const Json& patch,
                   const std::string& subresource = "");
  // long-poll watch; callback returns false to stop.  Returns HTTP status.
  int watch(const ResourceKind& k, const std::string& ns, const std::string& field_selector,
            const std::string& resource_version, int timeout_s,
            const std::function<bool(const WatchEvent&)>& cb);

  std::string collection_path(const ResourceKind& k, const std::string& ns) const;
  std::string object_path(const ResourceKind& k, const std::string& ns, const std::string& name) const;

 private:
  HttpResponse call(const std::string& method, const std::string& target, const std::string& body = "",
                    const std::string& content_type = "application/json", double timeout_s = 30.0);
  Json checked(const HttpResponse& r);
  void add_auth(HttpRequest& req) const;

  void refresh_credentials(bool force);

  KubeConfig cfg_;
  Url url_;
  long long cred_expires_ = 0;   // exec plugin credential expiry (unix s)
  bool cred_loaded_ = false;
};

// metadata.name of an object ("" if absent)
std::string object_name(const Json& obj);

}  // namespace h2ok
