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

#include "http.hpp"
#include "json.hpp"

namespace h2ok {

struct KubeConfig {
  std::string server;          // https://host:port[/base]
  TlsConfig tls;
  std::string token;           // bearer token
  std::string username, password;
  std::string ns = "default";  // context namespace (kubeconfig default)
  std::string source;          // kubeconfig path ("" = in-cluster)
  std::string context;
};

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
extern const ResourceKind CRD;
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

  KubeConfig cfg_;
  Url url_;
};

// metadata.name of an object ("" if absent)
std::string object_name(const Json& obj);

}  // namespace h2ok
