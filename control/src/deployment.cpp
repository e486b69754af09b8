#include "deployment.hpp"
#include "platform.hpp"


#include <chrono>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <regex>
#include <sstream>

namespace h2ok {

// ---------------------------------------------------------------------------
// model
// ---------------------------------------------------------------------------
Json DeploymentSpecification::to_json() const {
  Json j = Json::object();
  j["name"] = name;
  j["namespace"] = ns;
  j["memory_percentage"] = memory_percentage;
  j["memory"] = memory;
  j["num_cpu"] = (int64_t)num_cpu;
  j["num_h2o_nodes"] = (int64_t)num_h2o_nodes;
  j["kubeconfig_path"] = kubeconfig_path ? Json(*kubeconfig_path) : Json();
  j["image"] = image;
  j["image_tag"] = image_tag;
  j["gpus_per_node"] = (int64_t)gpus_per_node;
  j["ingress_api"] = ingress_api;
  if (!ingress_class.empty()) j["ingress_class"] = ingress_class;
  return j;
}

DeploymentSpecification DeploymentSpecification::from_json(const Json& j) {
  DeploymentSpecification s;
  s.name = j.at("name").as_string();
  s.ns = j.at("namespace").as_string();
  s.memory_percentage = (int)j.get_int("memory_percentage", 50);
  s.memory = j.get_string("memory", "1Gi");
  s.num_cpu = (uint32_t)j.get_int("num_cpu", 1);
  s.num_h2o_nodes = (uint32_t)j.get_int("num_h2o_nodes", 1);
  const Json* kc = j.find("kubeconfig_path");
  if (kc && kc->is_string()) s.kubeconfig_path = kc->as_string();
  s.image = j.get_string("image", s.image);
  s.image_tag = j.get_string("image_tag", s.image_tag);
  s.gpus_per_node = (uint32_t)j.get_int("gpus_per_node", 1);
  // descriptors written by the reference tool used the v1beta1 Ingress API
  s.ingress_api = j.get_string("ingress_api", j.has("image") ? s.ingress_api : "networking.k8s.io/v1beta1");
  s.ingress_class = j.get_string("ingress_class", "");
  return s;
}

Json Deployment::to_json() const {
  Json j = Json::object();
  j["specification"] = specification.to_json();
  j["ingresses"] = Json(JsonArray(ingresses.begin(), ingresses.end()));
  j["stateful_sets"] = Json(JsonArray(stateful_sets.begin(), stateful_sets.end()));
  j["services"] = Json(JsonArray(services.begin(), services.end()));
  if (!middlewares.empty()) j["middlewares"] = Json(JsonArray(middlewares.begin(), middlewares.end()));
  return j;
}

Deployment Deployment::from_json(const Json& j) {
  Deployment d;
  d.specification = DeploymentSpecification::from_json(j.at("specification"));
  auto grab = [&](const char* k, std::vector<Json>& out) {
    if (const Json* a = j.find(k))
      if (a->is_array())
        for (auto& e : a->as_array()) out.push_back(e);
  };
  grab("ingresses", d.ingresses);
  grab("stateful_sets", d.stateful_sets);
  grab("services", d.services);
  grab("middlewares", d.middlewares);
  return d;
}

// ---------------------------------------------------------------------------
// templates (MI355X node pods; SURVEY.md §2.6 env contract kept verbatim)
// ---------------------------------------------------------------------------
namespace {

Json kv(const std::string& k, Json v) {
  Json o = Json::object();
  o[k] = std::move(v);
  return o;
}

Json env_var(const std::string& name, const std::string& value) {
  Json e = Json::object();
  e["name"] = name;
  e["value"] = value;
  return e;
}

Json labels_for(const DeploymentSpecification& s) {
  Json l = Json::object();
  l["app"] = s.name;
  l["app.kubernetes.io/name"] = "h2omx";
  l["app.kubernetes.io/instance"] = s.name;
  l["app.kubernetes.io/managed-by"] = "h2ok";
  return l;
}

}  // namespace

Json h2o_service(const DeploymentSpecification& s) {
  Json svc = Json::object();
  svc["apiVersion"] = "v1";
  svc["kind"] = "Service";
  Json md = Json::object();
  md["name"] = s.name + "-service";
  md["namespace"] = s.ns;
  md["labels"] = labels_for(s);
  svc["metadata"] = md;
  Json spec = Json::object();
  spec["type"] = "ClusterIP";
  spec["clusterIP"] = "None";
  // peers must resolve each other before the leader is Ready (Q3)
  spec["publishNotReadyAddresses"] = true;
  spec["selector"] = kv("app", s.name);
  Json ports = Json::array();
  Json http = Json::object();
  http["name"] = "http";
  http["protocol"] = "TCP";
  http["port"] = 80;
  http["targetPort"] = 54321;
  ports.push_back(http);
  Json rdzv = Json::object();
  rdzv["name"] = "rendezvous";
  rdzv["protocol"] = "TCP";
  rdzv["port"] = 29500;
  rdzv["targetPort"] = 29500;
  ports.push_back(rdzv);
  spec["ports"] = ports;
  svc["spec"] = spec;
  return svc;
}

Json h2o_stateful_set(const DeploymentSpecification& s) {
  const std::string nodes = std::to_string(s.num_h2o_nodes);
  Json sts = Json::object();
  sts["apiVersion"] = "apps/v1";
  sts["kind"] = "StatefulSet";
  Json md = Json::object();
  md["name"] = s.name + "-stateful-set";
  md["namespace"] = s.ns;
  md["labels"] = labels_for(s);
  sts["metadata"] = md;
  Json spec = Json::object();
  spec["serviceName"] = s.name + "-service";  // Q2: matches the real service
  spec["podManagementPolicy"] = "Parallel";
  spec["replicas"] = (int64_t)s.num_h2o_nodes;
  spec["selector"] = kv("matchLabels", kv("app", s.name));
  Json tmpl = Json::object();
  Json tmd = Json::object();
  tmd["labels"] = labels_for(s);
  tmpl["metadata"] = tmd;
  Json pod = Json::object();
  // Topologies (docs/ARCHITECTURE.md "Multi-GPU topology"):
  //  * one pod per node with gpus_per_node GPUs and gpus_per_node ranks
  //    (--cluster_size 1 --gpus_per_node 8): every rank shares the pod's IPC,
  //    /dev/shm and device view, so RCCL uses its P2P transport over xGMI;
  //  * one pod per GPU (--gpus_per_node 1): RCCL's P2P / SHM transports between
  //    pods need the host IPC namespace and the HOST /dev/shm, which hostIPC
  //    mounts into the container.  Nothing may be mounted over /dev/shm (a
  //    per-pod emptyDir would hide the host's and push RCCL onto sockets); the
  //    GPU device plugin must also expose peer devices for xGMI P2P.
  pod["hostIPC"] = true;
  pod["terminationGracePeriodSeconds"] = 10;
  Json c = Json::object();
  c["name"] = s.name;
  c["image"] = s.image + ":" + s.image_tag;
  Json cmd = Json::array();
  cmd.push_back("python3");
  cmd.push_back("-m");
  cmd.push_back("h2omx.runtime.node");
  c["command"] = cmd;
  Json ports = Json::array();
  Json p1 = Json::object();
  p1["name"] = "api";
  p1["containerPort"] = 54321;
  p1["protocol"] = "TCP";
  ports.push_back(p1);
  Json p2 = Json::object();
  p2["name"] = "leader";
  p2["containerPort"] = 8081;
  p2["protocol"] = "TCP";
  ports.push_back(p2);
  Json p3 = Json::object();
  p3["name"] = "rendezvous";
  p3["containerPort"] = 29500;
  p3["protocol"] = "TCP";
  ports.push_back(p3);
  c["ports"] = ports;
  Json probe = Json::object();
  Json hg = Json::object();
  hg["path"] = "/kubernetes/isLeaderNode";
  hg["port"] = 8081;
  probe["httpGet"] = hg;
  probe["initialDelaySeconds"] = 5;
  probe["periodSeconds"] = 5;
  probe["failureThreshold"] = 1;
  c["readinessProbe"] = probe;
  Json res = Json::object();
  Json lim = Json::object();
  lim["cpu"] = std::to_string(s.num_cpu);
  lim["memory"] = s.memory;
  if (s.gpus_per_node > 0) lim["amd.com/gpu"] = std::to_string(s.gpus_per_node);
  res["limits"] = lim;
  res["requests"] = lim.deep_copy();
  c["resources"] = res;
  Json env = Json::array();
  env.push_back(env_var("H2O_KUBERNETES_SERVICE_DNS", s.name + "-service." + s.ns + ".svc.cluster.local"));
  env.push_back(env_var("H2O_NODE_LOOKUP_TIMEOUT", "180"));
  env.push_back(env_var("H2O_NODE_EXPECTED_COUNT", nodes));
  env.push_back(env_var("H2O_KUBERNETES_API_PORT", "8081"));
  env.push_back(env_var("H2OMX_MEMORY_PERCENTAGE", std::to_string(s.memory_percentage)));
  env.push_back(env_var("H2OMX_CLUSTER_NAME", s.name));
  env.push_back(env_var("HSA_ENABLE_IPC_MODE_LEGACY", "0"));
  // ranks per pod: the node entry point forks one rank per GPU before any GPU call
  env.push_back(env_var("H2OMX_GPUS_PER_NODE", std::to_string(s.gpus_per_node > 0 ? s.gpus_per_node : 1)));
  Json pod_name = Json::object();
  pod_name["name"] = "POD_NAME";
  pod_name["valueFrom"] = kv("fieldRef", kv("fieldPath", "metadata.name"));
  env.push_back(pod_name);
  c["env"] = env;
  Json containers = Json::array();
  containers.push_back(c);
  pod["containers"] = containers;
  tmpl["spec"] = pod;
  spec["template"] = tmpl;
  sts["spec"] = spec;
  return sts;
}

Json h2o_ingress(const DeploymentSpecification& s) {
  Json ing = Json::object();
  const bool v1 = s.ingress_api != "networking.k8s.io/v1beta1";
  ing["apiVersion"] = v1 ? "networking.k8s.io/v1" : "networking.k8s.io/v1beta1";
  ing["kind"] = "Ingress";
  Json md = Json::object();
  md["name"] = s.name + "-ingress";
  md["namespace"] = s.ns;
  md["labels"] = labels_for(s);
  Json ann = Json::object();
  const bool traefik = s.ingress_class == "traefik";
  if (traefik) {
    // Traefik v2 (K3s' bundled controller, the reference CI's cluster): a plain
    // Prefix route plus the StripPrefix middleware (h2o_strip_prefix_middleware);
    // v2 ignores v1's frontend annotations and takes a regex path literally
    ann["traefik.ingress.kubernetes.io/router.middlewares"] = s.ns + "-" + s.name + "-stripprefix@kubernetescrd";
  } else {
    // strip the /<name> prefix before forwarding (Q12: capture groups exist)
    ann["nginx.ingress.kubernetes.io/rewrite-target"] = "/$2";
    ann["nginx.ingress.kubernetes.io/use-regex"] = "true";
    ann["traefik.frontend.rule.type"] = "PathPrefixStrip";   // Traefik v1
  }
  md["annotations"] = ann;
  ing["metadata"] = md;
  Json path = Json::object();
  if (v1 && traefik) {
    path["path"] = "/" + s.name;
    path["pathType"] = "Prefix";
    Json svc = Json::object();
    svc["name"] = s.name + "-service";
    svc["port"] = kv("number", 80);
    path["backend"] = kv("service", svc);
  } else if (v1) {
    path["path"] = "/" + s.name + "(/|$)(.*)";
    path["pathType"] = "ImplementationSpecific";
    Json svc = Json::object();
    svc["name"] = s.name + "-service";
    svc["port"] = kv("number", 80);
    path["backend"] = kv("service", svc);
  } else {
    path["path"] = "/" + s.name;
    path["pathType"] = "Prefix";
    Json be = Json::object();
    be["serviceName"] = s.name + "-service";
    be["servicePort"] = 80;
    path["backend"] = be;
  }
  Json paths = Json::array();
  paths.push_back(path);
  Json rule = kv("http", kv("paths", paths));
  Json rules = Json::array();
  rules.push_back(rule);
  Json spec = kv("rules", rules);
  // a class resolved from the cluster default is not named: the default applies
  const bool named = !s.ingress_class.empty() && !s.ingress_class_from_cluster;
  if (v1 && named) spec["ingressClassName"] = s.ingress_class;
  ing["spec"] = spec;
  if (!v1 && named) ing["metadata"]["annotations"]["kubernetes.io/ingress.class"] = s.ingress_class;
  return ing;
}

Json h2o_strip_prefix_middleware(const DeploymentSpecification& s, const std::string& api_version) {
  Json mw = Json::object();
  mw["apiVersion"] = api_version;
  mw["kind"] = "Middleware";
  Json md = Json::object();
  md["name"] = s.name + "-stripprefix";
  md["namespace"] = s.ns;
  md["labels"] = labels_for(s);
  mw["metadata"] = md;
  Json prefixes = Json::array();
  prefixes.push_back("/" + s.name);
  mw["spec"] = kv("stripPrefix", kv("prefixes", prefixes));
  return mw;
}

bool valid_ingress_class(const std::string& c) { return c.empty() || c == "nginx" || c == "traefik"; }

std::string default_ingress_class(KubeClient& client) {
  Json lst;
  try {
    lst = client.list(kinds::IngressClass, "");
  } catch (const std::exception&) {
    return "";   // not readable (RBAC) or not served: keep the class-less nginx-style route
  }
  const Json* items = lst.find("items");
  if (!items || !items->is_array()) return "";
  for (auto& ic : items->as_array()) {
    const Json* ann = ic.path("metadata.annotations");
    // (keys with dots: looked up directly, not as a path)
    const std::string key = "ingressclass.kubernetes.io/is-default-class";
    if (!ann || !ann->is_object() || !ann->has(key) || !ann->at(key).is_string() || ann->at(key).as_string() != "true")
      continue;
    const std::string ctl = ic.get_string("spec.controller");
    if (ctl.find("traefik") != std::string::npos) return "traefik";
    if (ctl.find("nginx") != std::string::npos) return "nginx";
    return "";
  }
  return "";
}

Json owner_reference(const Json& owner) {
  Json o = Json::object();
  o["apiVersion"] = owner.get_string("apiVersion");
  o["kind"] = owner.get_string("kind");
  o["name"] = owner.get_string("metadata.name");
  o["uid"] = owner.get_string("metadata.uid");
  o["controller"] = true;
  o["blockOwnerDeletion"] = true;
  return o;
}

// ---------------------------------------------------------------------------
// orchestration
// ---------------------------------------------------------------------------
namespace {

const ResourceKind& ingress_kind(const DeploymentSpecification& s) {
  return s.ingress_api == "networking.k8s.io/v1beta1" ? kinds::IngressV1beta1 : kinds::IngressV1;
}

void rollback(KubeClient& client, const Deployment& d, const std::string& what, const std::string& reason) {
  std::cerr << "Unable to deploy " << what << " for '" << d.specification.name
            << "' deployment. Rewinding existing deployment. Reason:\n" << reason << std::endl;
  auto failed = undeploy_h2o(client, d);
  for (auto& f : failed) std::cerr << "Rollback: unable to undeploy '" << f << "'." << std::endl;
}

}  // namespace

Deployment deploy_h2o_cluster(KubeClient& client, const DeploymentSpecification& spec) {
  Deployment d;
  d.specification = spec;
  try {
    d.services.push_back(client.create(kinds::Service, spec.ns, h2o_service(spec)));
  } catch (const std::exception& e) {
    rollback(client, d, "service", e.what());
    throw DeployError(e.what());
  }
  try {
    d.stateful_sets.push_back(client.create(kinds::StatefulSet, spec.ns, h2o_stateful_set(spec)));
  } catch (const std::exception& e) {
    rollback(client, d, "statefulset", e.what());
    throw DeployError(e.what());
  }
  return d;
}

std::vector<std::string> undeploy_h2o(KubeClient& client, const Deployment& d) {
  std::vector<std::string> failed;
  const std::string& ns = d.specification.ns;
  auto del = [&](const ResourceKind& k, const Json& obj) {
    std::string name = object_name(obj);
    std::string objns = obj.get_string("metadata.namespace", ns);
    try {
      client.remove(k, objns, name, k.kind == "StatefulSet" ? "Background" : "");
    } catch (const ApiError& e) {
      if (e.status != 404) failed.push_back(name);
    } catch (const std::exception&) {
      failed.push_back(name);
    }
  };
  for (auto& i : d.ingresses) {
    const bool beta = i.get_string("apiVersion") == "networking.k8s.io/v1beta1";
    del(beta ? kinds::IngressV1beta1 : kinds::IngressV1, i);
  }
  for (auto& m : d.middlewares) {
    const bool legacy = m.get_string("apiVersion") == "traefik.containo.us/v1alpha1";
    del(legacy ? kinds::TraefikMiddlewareLegacy : kinds::TraefikMiddleware, m);
  }
  for (auto& s : d.services) del(kinds::Service, s);
  for (auto& s : d.stateful_sets) del(kinds::StatefulSet, s);
  return failed;
}

std::optional<std::string> any_ip(const Json& ingress) {
  const Json* lb = ingress.path("status.loadBalancer.ingress");
  if (!lb || !lb->is_array() || lb->size() == 0) return std::nullopt;
  const Json& last = (*lb)[lb->size() - 1];
  std::string ip = last.get_string("ip");
  if (ip.empty()) ip = last.get_string("hostname");
  if (ip.empty()) return std::nullopt;
  return ip;
}

std::optional<std::string> any_path(const Json& ingress) {
  const Json* rules = ingress.path("spec.rules");
  if (!rules || !rules->is_array() || rules->size() == 0) return std::nullopt;
  const Json* paths = (*rules)[rules->size() - 1].path("http.paths");
  if (!paths || !paths->is_array() || paths->size() == 0) return std::nullopt;
  std::string p = (*paths)[paths->size() - 1].get_string("path");
  if (p.empty()) return std::nullopt;
  // strip the regex suffix of the v1 template: "/name(/|$)(.*)" -> "/name"
  size_t paren = p.find('(');
  if (paren != std::string::npos) p = p.substr(0, paren);
  return p;
}

Json create_strip_prefix_middleware(KubeClient& client, const DeploymentSpecification& spec,
                                    const std::function<void(Json&)>& decorate) {
  // traefik.io/v1alpha1 (Traefik >= 2.10); clusters with an earlier v2 only
  // serve the traefik.containo.us group (404 / 405 on the new one)
  auto build = [&](const char* api) {
    Json mw = h2o_strip_prefix_middleware(spec, api);
    if (decorate) decorate(mw);
    return mw;
  };
  try {
    return client.create(kinds::TraefikMiddleware, spec.ns, build("traefik.io/v1alpha1"));
  } catch (const ApiError& e) {
    if (e.status != 404 && e.status != 405) throw;
  }
  return client.create(kinds::TraefikMiddlewareLegacy, spec.ns, build("traefik.containo.us/v1alpha1"));
}

void deploy_ingress(KubeClient& client, Deployment& d, int watch_timeout_s) {
  // no --ingress_class at deploy time: follow the cluster's default IngressClass
  // (K3s, the reference CI's cluster, defaults to Traefik v2, which needs the
  // Prefix + StripPrefix pair; reference templates.rs:104-106 annotated for both)
  DeploymentSpecification spec = d.specification;
  if (spec.ingress_class.empty()) {
    spec.ingress_class = default_ingress_class(client);
    spec.ingress_class_from_cluster = !spec.ingress_class.empty();
  }
  const ResourceKind& k = ingress_kind(spec);
  if (spec.ingress_class == "traefik") d.middlewares.push_back(create_strip_prefix_middleware(client, spec));
  Json created;
  try {
    created = client.create(k, spec.ns, h2o_ingress(spec));
  } catch (...) {
    // Q13: no half-made ingress - the middleware created above goes again
    if (spec.ingress_class == "traefik") {
      Deployment part;
      part.specification = spec;
      part.middlewares.push_back(d.middlewares.back());
      d.middlewares.pop_back();
      undeploy_h2o(client, part);
    }
    throw;
  }
  std::string name = object_name(created);
  Json latest = created;
  if (!any_ip(latest) && watch_timeout_s > 0) {
    try {
      client.watch(k, spec.ns, "metadata.name=" + name, created.get_string("metadata.resourceVersion"),
                   watch_timeout_s, [&](const WatchEvent& ev) {
                     if (ev.type == "MODIFIED" || ev.type == "ADDED") {
                       latest = ev.object;
                       if (any_ip(latest)) return false;
                     }
                     return true;
                   });
    } catch (const std::exception& e) {
      std::cerr << "Warning: watching ingress '" << name << "' failed: " << e.what() << std::endl;
    }
  }
  d.ingresses.push_back(latest);
}

// ---------------------------------------------------------------------------
// descriptor files
// ---------------------------------------------------------------------------
namespace {
bool path_exists(const std::string& p) { return plat::path_exists(p); }
}  // namespace

std::string persist_deployment(const Deployment& d, bool overwrite, const std::string& explicit_path) {
  std::string file_name = explicit_path.empty() ? d.specification.name + ".h2ok" : explicit_path;
  if (path_exists(file_name)) {
    if (overwrite) {
      if (std::remove(file_name.c_str()) != 0)
        throw std::runtime_error("Unable to remove existing deployment file '" + file_name + "'");
    } else {
      int k = 0;
      while (path_exists(file_name)) {
        std::cerr << "Writing file" << std::endl;  // Q5: diagnostics on stderr
        ++k;
        file_name = d.specification.name + "(" + std::to_string(k) + ").h2ok";
      }
    }
  }
  std::ofstream out(file_name, std::ios::binary | std::ios::trunc);
  if (!out) {
    std::cerr << "Unable to write deployment file '" << file_name << "' - skipping." << std::endl;
    throw std::runtime_error("cannot write " + file_name);
  }
  out << d.to_json().dump();
  return file_name;
}

Deployment load_deployment(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("cannot open deployment descriptor '" + path + "'");
  std::ostringstream os;
  os << in.rdbuf();
  return Deployment::from_json(Json::parse(os.str()));
}

bool valid_memory_quantity(const std::string& s) {
  static const std::regex re("^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$");
  return std::regex_match(s, re);
}

bool valid_dns_label(const std::string& s) {
  static const std::regex re("^[a-z0-9]([-a-z0-9]*[a-z0-9])?$");
  return s.size() <= 52 && std::regex_match(s, re);
}

}  // namespace h2ok
