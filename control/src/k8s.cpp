#include "k8s.hpp"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>

#include "platform.hpp"
#include "yaml.hpp"

namespace h2ok {

namespace kinds {
const ResourceKind Service{"/api/v1", "services", "Service", true};
const ResourceKind StatefulSet{"/apis/apps/v1", "statefulsets", "StatefulSet", true};
const ResourceKind IngressV1{"/apis/networking.k8s.io/v1", "ingresses", "Ingress", true};
const ResourceKind IngressV1beta1{"/apis/networking.k8s.io/v1beta1", "ingresses", "Ingress", true};
const ResourceKind Pod{"/api/v1", "pods", "Pod", true};
const ResourceKind H2O{"/apis/h2o.ai/v1beta", "h2os", "H2O", true};
const ResourceKind TraefikMiddleware{"/apis/traefik.io/v1alpha1", "middlewares", "Middleware", true};
const ResourceKind TraefikMiddlewareLegacy{"/apis/traefik.containo.us/v1alpha1", "middlewares", "Middleware", true};
const ResourceKind CRD{"/apis/apiextensions.k8s.io/v1", "customresourcedefinitions", "CustomResourceDefinition",
                       false};
const ResourceKind IngressClass{"/apis/networking.k8s.io/v1", "ingressclasses", "IngressClass", false};
}  // namespace kinds

namespace {

bool file_exists(const std::string& p) { return plat::is_regular_file(p); }

std::string read_file(const std::string& p) {
  std::ifstream in(p, std::ios::binary);
  if (!in) throw KubeConfigError("cannot read " + p);
  std::ostringstream os;
  os << in.rdbuf();
  return os.str();
}

std::string dir_of(const std::string& p) {
  size_t s = p.find_last_of(plat::path_sep() == '/' ? "/" : "/\\");
  return s == std::string::npos ? "." : p.substr(0, s);
}

bool is_absolute(const std::string& p) {
  if (p.empty()) return false;
  if (p[0] == '/' || p[0] == '\\') return true;
  return plat::path_sep() == '\\' && p.size() > 2 && p[1] == ':';   // C:\...
}

std::string resolve(const std::string& base_dir, const std::string& p) {
  if (p.empty() || is_absolute(p)) return p;
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
    if (const Json* ex = ub.find("exec")) {
      ExecPlugin pl;
      pl.api_version = ex->get_string("apiVersion", pl.api_version);
      pl.command = ex->get_string("command");
      if (pl.command.empty()) throw KubeConfigError("user '" + uname + "': exec plugin has no command");
      if (const Json* a = ex->find("args"))
        if (a->is_array())
          for (auto& v : a->as_array()) pl.args.push_back(v.is_string() ? v.as_string() : v.dump());
      if (const Json* e = ex->find("env"))
        if (e->is_array())
          for (auto& v : e->as_array()) pl.env.emplace_back(v.get_string("name"), v.get_string("value"));
      pl.install_hint = ex->get_string("installHint");
      const Json* pci = ex->find("provideClusterInfo");
      pl.provide_cluster_info = pci && pci->is_bool() && pci->as_bool();
      pl.base_dir = base;
      kc.exec = pl;
    } else if (const Json* ap = ub.find("auth-provider")) {
      AuthProvider a;
      a.name = ap->get_string("name");
      const Json* cfg = ap->find("config");
      a.config = cfg ? cfg->deep_copy() : Json::object();
      a.base_dir = base;
      kc.auth_provider = a;
    }
  }
  return kc;
}

namespace {

int run_capture(const std::vector<std::string>& argv, const std::vector<std::pair<std::string, std::string>>& env,
                std::string& out, std::string& err, double timeout_s) {
  return plat::run_capture(argv, env, out, err, timeout_s);
}

long long parse_rfc3339(const std::string& t) { return plat::parse_rfc3339_utc(t); }

std::string resolve_command(const std::string& base_dir, const std::string& cmd) {
  // a path with a separator is relative to the kubeconfig; a bare name is a PATH lookup
  if (cmd.find('/') != std::string::npos) return resolve(base_dir, cmd);
  return cmd;
}

}  // namespace

ExecCredential run_exec_plugin(const ExecPlugin& p, const KubeConfig& cluster) {
  Json info = Json::object();
  info["apiVersion"] = p.api_version;
  info["kind"] = "ExecCredential";
  Json spec = Json::object();
  spec["interactive"] = false;
  if (p.provide_cluster_info) {
    Json c = Json::object();
    c["server"] = cluster.server;
    if (!cluster.tls.ca_pem.empty()) c["certificate-authority-data"] = base64_encode(cluster.tls.ca_pem);
    if (cluster.tls.insecure) c["insecure-skip-tls-verify"] = true;
    if (!cluster.tls.server_name.empty()) c["tls-server-name"] = cluster.tls.server_name;
    spec["cluster"] = c;
  }
  info["spec"] = spec;
  std::vector<std::string> argv{resolve_command(p.base_dir, p.command)};
  argv.insert(argv.end(), p.args.begin(), p.args.end());
  auto env = p.env;
  env.emplace_back("KUBERNETES_EXEC_INFO", info.dump());
  std::string out, err;
  int rc = run_capture(argv, env, out, err, 60.0);
  if (rc != 0) {
    std::string msg = "exec plugin '" + p.command + "' failed (status " + std::to_string(rc) + ")";
    if (!err.empty()) msg += ": " + err.substr(0, 2000);
    if (rc == 127 && !p.install_hint.empty()) msg += "\n" + p.install_hint;
    throw KubeConfigError(msg);
  }
  Json doc;
  try {
    doc = Json::parse(out);
  } catch (const std::exception& e) {
    throw KubeConfigError("exec plugin '" + p.command + "' printed no ExecCredential JSON: " + e.what());
  }
  if (doc.get_string("kind") != "ExecCredential")
    throw KubeConfigError("exec plugin '" + p.command + "': expected kind ExecCredential");
  const Json* st = doc.find("status");
  if (!st) throw KubeConfigError("exec plugin '" + p.command + "': ExecCredential has no status");
  ExecCredential c;
  c.token = st->get_string("token");
  c.client_cert_pem = st->get_string("clientCertificateData");
  c.client_key_pem = st->get_string("clientKeyData");
  c.expires_at = parse_rfc3339(st->get_string("expirationTimestamp"));
  if (c.token.empty() && (c.client_cert_pem.empty() || c.client_key_pem.empty()))
    throw KubeConfigError("exec plugin '" + p.command + "' returned neither a token nor a client certificate");
  return c;
}

std::string auth_provider_token(const AuthProvider& a) {
  if (a.name == "oidc") {
    std::string t = a.config.get_string("id-token");
    if (t.empty()) throw KubeConfigError("auth-provider oidc: no id-token in the kubeconfig (log in with kubelogin)");
    return t;
  }
  if (a.name == "gcp") {
    std::string t = a.config.get_string("access-token");
    long long exp = parse_rfc3339(a.config.get_string("expiry"));
    if (!t.empty() && (exp == 0 || exp > (long long)std::time(nullptr) + 10)) return t;
    std::string cmd = a.config.get_string("cmd-path");
    if (cmd.empty()) throw KubeConfigError("auth-provider gcp: access token expired and no cmd-path to refresh it");
    std::vector<std::string> argv{resolve_command(a.base_dir, cmd)};
    std::istringstream ss(a.config.get_string("cmd-args"));
    for (std::string w; ss >> w;) argv.push_back(w);
    std::string out, err;
    if (run_capture(argv, {}, out, err, 60.0) != 0)
      throw KubeConfigError("auth-provider gcp: '" + cmd + "' failed: " + err.substr(0, 2000));
    Json doc = Json::parse(out);
    // token-key is a JSONPath such as {.credential.access_token}
    std::string key = a.config.get_string("token-key", "{.credential.access_token}");
    if (!key.empty() && key.front() == '{') key = key.substr(1, key.size() - 2);
    if (!key.empty() && key.front() == '.') key = key.substr(1);
    t = doc.get_string(key);
    if (t.empty()) throw KubeConfigError("auth-provider gcp: no token at " + key);
    return t;
  }
  throw KubeConfigError("auth-provider '" + a.name + "' is not supported (use an exec plugin)");
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
    // list separator: ':' (POSIX), ';' (Windows, where ':' follows drive letters)
    while (std::getline(ss, item, plat::path_sep() == '/' ? ':' : ';'))
      if (!item.empty() && file_exists(item)) return load_kubeconfig(item);
  }
  const char* home = std::getenv("HOME");
  if (!home) home = std::getenv("USERPROFILE");   // Windows
  if (home) {
    std::string p = std::string(home) + "/.kube/config";
    if (file_exists(p)) return load_kubeconfig(p);
  }
  return in_cluster_config();
}

KubeClient::KubeClient(KubeConfig cfg) : cfg_(std::move(cfg)), url_(parse_url(cfg_.server)) {}

// Credentials from an exec plugin / auth-provider: fetched on first use,
// cached until their expiry, re-fetched once after a 401.
void KubeClient::refresh_credentials(bool force) {
  const long long now = (long long)std::time(nullptr);
  if (cfg_.exec) {
    if (!force && cred_loaded_ && (cred_expires_ == 0 || cred_expires_ > now + 10)) return;
    ExecCredential c = run_exec_plugin(*cfg_.exec, cfg_);
    cfg_.token = c.token;
    if (!c.client_cert_pem.empty()) {
      cfg_.tls.client_cert_pem = c.client_cert_pem;
      cfg_.tls.client_key_pem = c.client_key_pem;
    }
    cred_expires_ = c.expires_at;
    cred_loaded_ = true;
  } else if (cfg_.auth_provider) {
    if (!force && cred_loaded_) return;
    cfg_.token = auth_provider_token(*cfg_.auth_provider);
    cred_loaded_ = true;
  }
}

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
  const bool plugin = cfg_.exec.has_value() || cfg_.auth_provider.has_value();
  if (plugin) refresh_credentials(false);
  HttpRequest first = req;
  add_auth(first);
  HttpResponse r = http_request(url_, first, cfg_.tls);
  if (r.status == 401 && plugin) {
    refresh_credentials(true);
    add_auth(req);
    r = http_request(url_, req, cfg_.tls);
  }
  return r;
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
  if (cfg_.exec || cfg_.auth_provider) refresh_credentials(false);
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
