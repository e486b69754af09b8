#include "k8s.hpp"

#include <sys/stat.h>

#include <cstdlib>
#include <fstream>
#include <sstream>

#include "yaml.hpp"

namespace h2ok {

namespace kinds {
const ResourceKind Service{"/api/v1", "services", "Service", true};
const ResourceKind StatefulSet{"/apis/apps/v1", "statefulsets", "StatefulSet", true};
const ResourceKind IngressV1{"/apis/networking.k8s.io/v1", "ingresses", "Ingress", true};
const ResourceKind IngressV1beta1{"/apis/networking.k8s.io/v1beta1", "ingresses", "Ingress", true};
const ResourceKind Pod{"/api/v1", "pods", "Pod", true};
const ResourceKind H2O{"/apis/h2o.ai/v1beta", "h2os", "H2O", true};
const ResourceKind CRD{"/apis/apiextensions.k8s.io/v1", "customresourcedefinitions", "CustomResourceDefinition",
                       false};
}  // namespace kinds

namespace {

bool file_exists(const std::string& p) {
  struct stat st{};
  return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

std::string read_file(const std::string& p) {
  std::ifstream in(p, std::ios::binary);
  if (!in) throw KubeConfigError("cannot read " + p);
  std::ostringstream os;
  os << in.rdbuf();
  return os.str();
}

std::string dir_of(const std::string& p) {
  size_t s = p.rfind('/');
  return s == std::string::npos ? "." : p.substr(0, s);
}

std::string resolve(const std::string& base_dir, const std::string& p) {
  if (p.empty() || p[0] == '/') return p;
  return base_dir + "/" + p;
}

const Json* named(const Json& list, const std::string& name) {
  if (!list.is_array()) return nullptr;
  for (auto& e : list.as_array())
    if (e.get_string("name") == name) return &e;
  return nullptr;
}

// "<x>-data" (base64 inline) or "<x>" (file path)
std::string data_or_file(const Json& obj, const std::string& key, const std::string& base_dir) {
  std::string inline_data = obj.get_string(key + "-data");
  if (!inline_data.empty()) return base64_decode(inline_data);
  std::string file = obj.get_string(key);
  if (!file.empty()) return read_file(resolve(base_dir, file));
  return "";
}

}  // namespace

KubeConfig load_kubeconfig(const std::string& path, const std::string& context) {
  Json doc;
  try {
    doc = yaml_parse(read_file(path));
  } catch (const KubeConfigError&) {
    throw;
  } catch (const std::exception& e) {
    throw KubeConfigError("cannot parse kubeconfig " + path + ": " + e.what());
  }
  if (!doc.is_object()) throw KubeConfigError("kubeconfig " + path + " is not a mapping");
  const std::string base = dir_of(path);
  std::string ctx_name = context.empty() ? doc.get_string("current-context") : context;
  const Json* contexts = doc.find("contexts");
  const Json* ctx = contexts ? named(*contexts, ctx_name) : nullptr;
  if (!ctx && contexts && contexts->is_array() && contexts->size() > 0 && ctx_name.empty()) ctx = &(*contexts)[0];
  if (!ctx) throw KubeConfigError("context '" + ctx_name + "' not found in " + path);
  const Json* c = ctx->find("context");
  if (!c) throw KubeConfigError("context '" + ctx_name + "' has no body");
  KubeConfig kc;
  kc.source = path;
  kc.context = ctx->get_string("name");
  std::string ns = c->get_string("namespace");
  kc.ns = ns.empty() ? "default" : ns;
  const Json* clusters = doc.find("clusters");
  const Json* cl = clusters ? named(*clusters, c->get_string("cluster")) : nullptr;
  if (!cl || !cl->find("cluster")) throw KubeConfigError("cluster '" + c->get_string("cluster") + "' not found");
  const Json& cb = cl->at("cluster");
  kc.server = cb.get_string("server");
  if (kc.server.empty()) throw KubeConfigError("cluster has no server url");
  kc.tls.ca_pem = data_or_file(cb, "certificate-authority", base);
  const Json* insecure = cb.find("insecure-skip-tls-verify");
  kc.tls.insecure = insecure && ((insecure->is_bool() && insecure->as_bool()) ||
                                 (insecure->is_string() && insecure->as_string() == "true"));
  kc.tls.server_name = cb.get_string("tls-server-name");
  const Json* users = doc.find("users");
  std::string uname = c->get_string("user");
  const Json* u = users ? named(*users, uname) : nullptr;
  if (u && u->find("user")) {
    const Json& ub = u->at("user");
    kc.token = ub.get_string("token");
    std::string tf = ub.get_string("tokenFile");
    if (kc.token.empty() && !tf.empty()) kc.token = read_file(resolve(base, tf));
    while (!kc.token.empty() && (kc.token.back() == '\n' || kc.token.back() == '\r')) kc.token.pop_back();
    kc.tls.client_cert_pem = data_or_file(ub, "client-certificate", base);
    kc.tls.client_key_pem = data_or_file(ub, "client-key", base);
    kc.username = ub.get_string("username");
    kc.password = ub.get_string("password");
    if (ub.find("exec") || ub.find("auth-provider"))
      if (kc.token.empty() && kc.tls.client_cert_pem.empty())
        throw KubeConfigError("user '" + uname + "' uses an exec/auth-provider plugin, which h2ok does not run");
  }
  return kc;
}

KubeConfig in_cluster_config() {
  const char* host = std::getenv("KUBERNETES_SERVICE_HOST");
  const char* port = std::getenv("KUBERNETES_SERVICE_PORT");
  const std::string sa = "/var/run/secrets/kubernetes.io/serviceaccount";
  if (!host || !port || !file_exists(sa + "/token")) throw KubeConfigError("not running inside a cluster");
  KubeConfig kc;
  std::string h = host;
  if (h.find(':') != std::string::npos) h = "[" + h + "]";
  kc.server = "https://" + h + ":" + port;
  kc.token = read_file(sa + "/token");
  while (!kc.token.empty() && (kc.token.back() == '\n' || kc.token.back() == '\r')) kc.token.pop_back();
  if (file_exists(sa + "/ca.crt")) kc.tls.ca_pem = read_file(sa + "/ca.crt");
  if (file_exists(sa + "/namespace")) {
    kc.ns = read_file(sa + "/namespace");
    while (!kc.ns.empty() && std::isspace((unsigned char)kc.ns.back())) kc.ns.pop_back();
  }
  kc.source = "";
  return kc;
}

KubeConfig infer_kubeconfig() {
  if (const char* env = std::getenv("KUBECONFIG")) {
    std::stringstream ss(env);
    std::string item;
    while (std::getline(ss, item, ':'))
      if (!item.empty() && file_exists(item)) return load_kubeconfig(item);
  }
  if (const char* home = std::getenv("HOME")) {
    std::string p = std::string(home) + "/.kube/config";
    if (file_exists(p)) return load_kubeconfig(p);
  }
  return in_cluster_config();
}

KubeClient::KubeClient(KubeConfig cfg) : cfg_(std::move(cfg)), url_(parse_url(cfg_.server)) {}

void KubeClient::add_auth(HttpRequest& req) const {
  if (!cfg_.token.empty()) req.headers.emplace_back("Authorization", "Bearer " + cfg_.token);
  else if (!cfg_.username.empty())
    req.headers.emplace_back("Authorization", "Basic " + base64_encode(cfg_.username + ":" + cfg_.password));
}

HttpResponse KubeClient::call(const std::string& method, const std::string& target, const std::string& body,
                              const std::string& content_type, double timeout_s) {
  HttpRequest req;
  req.method = method;
  req.target = url_.path + target;
  req.body = body;
  req.timeout_s = timeout_s;
  if (!body.empty() || method == "POST" || method == "PUT" || method == "PATCH")
    req.headers.emplace_back("Content-Type", content_type);
  add_auth(req);
  return http_request(url_, req, cfg_.tls);
}

Json KubeClient::checked(const HttpResponse& r) {
  if (r.status >= 200 && r.status < 300) return r.body.empty() ? Json::object() : Json::parse(r.body);
  std::string reason, message;
  try {
    Json s = Json::parse(r.body);
    reason = s.get_string("reason");
    message = s.get_string("message");
  } catch (...) {
    message = r.body;
  }
  throw ApiError(r.status, reason, message, r.body);
}

std::string KubeClient::collection_path(const ResourceKind& k, const std::string& ns) const {
  if (!k.namespaced || ns.empty()) return k.api + "/" + k.plural;
  return k.api + "/namespaces/" + ns + "/" + k.plural;
}

std::string KubeClient::object_path(const ResourceKind& k, const std::string& ns, const std::string& name) const {
  return collection_path(k, ns) + "/" + name;
}

Json KubeClient::create(const ResourceKind& k, const std::string& ns, const Json& body) {
  return checked(call("POST", collection_path(k, ns), body.dump()));
}

Json KubeClient::get(const ResourceKind& k, const std::string& ns, const std::string& name) {
  return checked(call("GET", object_path(k, ns, name)));
}

std::optional<Json> KubeClient::get_opt(const ResourceKind& k, const std::string& ns, const std::string& name) {
  auto r = call("GET", object_path(k, ns, name));
  if (r.status == 404) return std::nullopt;
  return checked(r);
}

Json KubeClient::list(const ResourceKind& k, const std::string& ns, const std::string& label_selector,
                      const std::string& field_selector) {
  std::string q;
  if (!label_selector.empty()) q += (q.empty() ? "?" : "&") + std::string("labelSelector=") + url_encode(label_selector);
  if (!field_selector.empty()) q += (q.empty() ? "?" : "&") + std::string("fieldSelector=") + url_encode(field_selector);
  return checked(call("GET", collection_path(k, ns) + q));
}

Json KubeClient::remove(const ResourceKind& k, const std::string& ns, const std::string& name,
                        const std::string& propagation) {
  std::string body;
  if (!propagation.empty()) {
    Json opts = Json::object();
    opts["apiVersion"] = "v1";
    opts["kind"] = "DeleteOptions";
    opts["propagationPolicy"] = propagation;
    body = opts.dump();
  }
  return checked(call("DELETE", object_path(k, ns, name), body));
}

Json KubeClient::replace(const ResourceKind& k, const std::string& ns, const std::string& name, const Json& body) {
  return checked(call("PUT", object_path(k, ns, name), body.dump()));
}

Json KubeClient::merge_patch(const ResourceKind& k, const std::string& ns, const std::string& name, const Json& patch,
                             const std::string& subresource) {
  std::string target = object_path(k, ns, name);
  if (!subresource.empty()) target += "/" + subresource;
  return checked(call("PATCH", target, patch.dump(), "application/merge-patch+json"));
}

int KubeClient::watch(const ResourceKind& k, const std::string& ns, const std::string& field_selector,
                      const std::string& resource_version, int timeout_s,
                      const std::function<bool(const WatchEvent&)>& cb) {
  std::string q = "?watch=1";
  if (!field_selector.empty()) q += "&fieldSelector=" + url_encode(field_selector);
  if (!resource_version.empty()) q += "&resourceVersion=" + url_encode(resource_version);
  if (timeout_s > 0) q += "&timeoutSeconds=" + std::to_string(timeout_s);
  HttpRequest req;
  req.method = "GET";
  req.target = url_.path + collection_path(k, ns) + q;
  req.timeout_s = timeout_s > 0 ? timeout_s + 5.0 : 3600.0;
  add_auth(req);
  return http_stream_lines(url_, req, cfg_.tls, [&](const std::string& line) {
    Json ev;
    try {
      ev = Json::parse(line);
    } catch (...) {
      return true;
    }
    WatchEvent we;
    we.type = ev.get_string("type");
    if (const Json* o = ev.find("object")) we.object = *o;
    return cb(we);
  });
}

std::string object_name(const Json& obj) { return obj.get_string("metadata.name"); }

}  // namespace h2ok
