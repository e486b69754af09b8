// Deployment model, Kubernetes object templates and deploy / undeploy /
// ingress orchestration.
//
// Parity map to isgasho/h2o-kubernetes:
//   DeploymentSpecification / Deployment   src/k8s/mod.rs:39-80
//   h2o_stateful_set / h2o_service / h2o_ingress templates
//                                          src/k8s/templates.rs:1-124
//   deploy_h2o_cluster (+ rollback)        src/k8s/mod.rs:82-127
//   undeploy_h2o                           src/k8s/mod.rs:129-164
//   deploy_ingress (+ 3 s IP watch)        src/k8s/mod.rs:166-199
//   ingress::any_ip / any_path             src/k8s/ingress.rs:1-19
// MI355X-first differences: pods request one `amd.com/gpu` each and run the
// h2omx node runtime (one rank per GPU, RCCL over xGMI), the headless service
// publishes not-ready addresses so peers can rendezvous before the leader is
// Ready, and the StatefulSet's serviceName matches the real service
// (SURVEY.md §7.6 Q2/Q3).
#pragma once
#include <functional>

#include <optional>
#include <string>
#include <vector>

#include "json.hpp"
#include "k8s.hpp"

namespace h2ok {

struct DeploymentSpecification {
  std::string name;
  std::string ns;                 // serialised as "namespace"
  int memory_percentage = 50;
  std::string memory = "1Gi";
  uint32_t num_cpu = 1;
  uint32_t num_h2o_nodes = 1;
  std::optional<std::string> kubeconfig_path;
  // h2omx extensions (optional in descriptors written by the reference)
  std::string image = "h2omx/h2omx-node";
  std::string image_tag = "latest";
  uint32_t gpus_per_node = 1;
  std::string ingress_api = "networking.k8s.io/v1";
  // ingress controller flavour: "" (nginx-style regex path, class left to the
  // cluster default), "nginx" (same, ingressClassName nginx) or "traefik"
  // (Traefik v2 - K3s' default: Prefix path + a StripPrefix Middleware CR)
  std::string ingress_class;
  // set (never persisted) when ingress_class was resolved from the cluster's
  // default IngressClass: the Ingress then names no class (the default applies)
  bool ingress_class_from_cluster = false;

  Json to_json() const;
  static DeploymentSpecification from_json(const Json& j);
};

struct Deployment {
  DeploymentSpecification specification;
  std::vector<Json> ingresses;
  std::vector<Json> stateful_sets;
  std::vector<Json> services;
  std::vector<Json> middlewares;   // Traefik StripPrefix middlewares of the ingress (ingress_class traefik)

  Json to_json() const;
  static Deployment from_json(const Json& j);
};

// ---- templates --------------------------------------------------------------
Json h2o_service(const DeploymentSpecification& s);
Json h2o_stateful_set(const DeploymentSpecification& s);
Json h2o_ingress(const DeploymentSpecification& s);
// Traefik v2 StripPrefix middleware for /<name> (ingress_class "traefik")
Json h2o_strip_prefix_middleware(const DeploymentSpecification& s, const std::string& api_version);
bool valid_ingress_class(const std::string& c);
// Ingress flavour of the cluster's default IngressClass (annotation
// ingressclass.kubernetes.io/is-default-class "true"): "traefik" for a Traefik
// controller (K3s' bundled one: traefik.io/ingress-controller), "nginx" for
// ingress-nginx, "" when no class is marked default, its controller is another
// one, or the classes cannot be read (403 / 404 / older cluster).
std::string default_ingress_class(KubeClient& client);
// common labels / owner reference helpers used by the operator
Json owner_reference(const Json& owner);

// ---- orchestration ----------------------------------------------------------
struct DeployError : public std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Service first, then StatefulSet; on failure the already-created objects are
// deleted (rollback) and DeployError is thrown.  Rollback failures are
// reported, never fatal.
Deployment deploy_h2o_cluster(KubeClient& client, const DeploymentSpecification& spec);

// Delete ingresses -> services -> stateful sets; returns the list of objects
// that could not be deleted (empty = success).  404s count as deleted.
std::vector<std::string> undeploy_h2o(KubeClient& client, const Deployment& d);

// Create the ingress, then watch it up to watch_timeout_s for a load-balancer
// address; the last-seen object is appended to d.ingresses.
void deploy_ingress(KubeClient& client, Deployment& d, int watch_timeout_s = 3);
// Traefik StripPrefix middleware (traefik.io, falling back to traefik.containo.us);
// `decorate` edits the object before the create (the operator adds its
// ownerReference so the middleware is garbage-collected with the CR)
Json create_strip_prefix_middleware(KubeClient& client, const DeploymentSpecification& spec,
                                    const std::function<void(Json&)>& decorate = {});

std::optional<std::string> any_ip(const Json& ingress);
std::optional<std::string> any_path(const Json& ingress);

// descriptor file I/O
std::string persist_deployment(const Deployment& d, bool overwrite, const std::string& explicit_path = "");
Deployment load_deployment(const std::string& path);

// K8s memory quantity validator (same pattern as the reference,
// src/cli/mod.rs:268)
bool valid_memory_quantity(const std::string& s);
// DNS-1123 label check for cluster names
bool valid_dns_label(const std::string& s);

}  // namespace h2ok
