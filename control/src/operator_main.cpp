// h2omx-operator: reconciles `H2O` custom resources (h2o.ai/v1beta) into the
// same headless Service + StatefulSet pair `h2ok deploy` creates, one pod per
// MI355X (amd.com/gpu: 1), and reports status (phase, readyNodes, leaderPod).
//
// The reference snapshot has no operator (kube-derive is declared but unused,
// Cargo.toml:10 of isgasho/h2o-kubernetes); the CR schema mirrors its
// DeploymentSpecification (src/k8s/mod.rs:58-74) as designed in SURVEY.md §7.2.
#include <signal.h>

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <iostream>
#include <map>
#include <thread>

#include "deployment.hpp"
#include "http.hpp"
#include "k8s.hpp"

using namespace h2ok;

namespace {

std::atomic<bool> g_stop{false};

void on_signal(int) { g_stop = true; }

struct Options {
  std::optional<std::string> kubeconfig;
  std::string ns;  // "" = all namespaces
  bool once = false;
  int resync_s = 30;
  int requeue_s = 2;
  std::string default_image = "h2omx/h2omx-node";
  std::string default_tag = "latest";
};

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ULL;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ULL;
  }
  return h;
}

std::string hex(uint64_t v) {
  char buf[17];
  std::snprintf(buf, sizeof buf, "%016llx", (unsigned long long)v);
  return buf;
}

std::string quantity_string(const Json* v, const std::string& dflt) {
  if (!v || v->is_null()) return dflt;
  if (v->is_string()) return v->as_string();
  if (v->is_number()) return std::to_string(v->as_int());
  return dflt;
}

DeploymentSpecification spec_from_cr(const Json& cr, const Options& o) {
  DeploymentSpecification s;
  s.name = object_name(cr);
  s.ns = cr.get_string("metadata.namespace", "default");
  const Json* spec = cr.find("spec");
  Json empty = Json::object();
  if (!spec) spec = &empty;
  s.num_h2o_nodes = (uint32_t)std::max<int64_t>(1, spec->get_int("nodes", 1));
  s.num_cpu = (uint32_t)std::max<int64_t>(1, spec->get_int("resources.cpu", 1));
  s.memory = quantity_string(spec->path("resources.memory"), "1Gi");
  s.memory_percentage = (int)spec->get_int("resources.memoryPercentage", 50);
  s.gpus_per_node = (uint32_t)spec->get_int("resources.gpu", 1);
  s.image = o.default_image;
  s.image_tag = o.default_tag;
  std::string version = spec->get_string("version");
  if (!version.empty()) s.image_tag = version;
  if (const Json* ci = spec->find("customImage")) {
    std::string img = ci->get_string("image");
    size_t colon = img.rfind(':');
    if (!img.empty()) {
      if (colon != std::string::npos && img.find('/', colon) == std::string::npos) {
        s.image = img.substr(0, colon);
        s.image_tag = img.substr(colon + 1);
      } else {
        s.image = img;
      }
    }
  }
  if (const Json* im = spec->find("image")) {
    if (im->is_object()) {
      s.image = im->get_string("name", s.image);
      s.image_tag = im->get_string("tag", s.image_tag);
    }
  }
  return s;
}

void adopt(Json& obj, const Json& cr, const std::string& hash) {
  Json& md = obj["metadata"];
  Json refs = Json::array();
  refs.push_back(owner_reference(cr));
  md["ownerReferences"] = refs;
  md["annotations"]["h2o.ai/spec-hash"] = hash;
}

// Desired-vs-actual comparison of the fields of the headless Service that
// someone may edit by hand (ports, selector); clusterIP is immutable.
bool service_drifted(const Json& cur, const Json& want) {
  const Json* cs = cur.find("spec");
  const Json* ws = want.find("spec");
  if (!cs || !ws) return true;
  auto ports = [](const Json* spec) {
    Json out = Json::array();
    if (const Json* ps = spec->find("ports"))
      if (ps->is_array())
        for (auto& p : ps->as_array()) {
          Json q = Json::object();
          q["port"] = p.get_int("port", 0);
          q["targetPort"] = p.find("targetPort") ? p.at("targetPort") : Json(p.get_int("port", 0));
          q["protocol"] = p.get_string("protocol", "TCP");
          out.push_back(q);
        }
    return out;
  };
  const Json* csel = cs->find("selector");
  const Json* wsel = ws->find("selector");
  return ports(cs) != ports(ws) || !csel || !wsel || *csel != *wsel;
}

const std::string* annotation(const Json& obj, const std::string& key) {
  const Json* ann = obj.path("metadata.annotations");
  if (!ann || !ann->is_object() || !ann->has(key)) return nullptr;
  const Json& v = ann->at(key);
  return v.is_string() ? &v.as_string() : nullptr;
}

class Reconciler {
 public:
  Reconciler(KubeClient& c, Options o) : c_(c), o_(std::move(o)) {}

  // Returns true when the CR needs another pass soon (a replaced StatefulSet
  // is still terminating): the main loop then re-lists within seconds.
  bool reconcile(const Json& cr) {
    const std::string name = object_name(cr);
    const std::string ns = cr.get_string("metadata.namespace", "default");
    if (cr.path("metadata.deletionTimestamp")) return false;  // GC via ownerReferences
    DeploymentSpecification s = spec_from_cr(cr, o_);
    Json svc = h2o_service(s);
    Json sts = h2o_stateful_set(s);
    const std::string hash = hex(fnv1a(sts.at("spec").dump() + svc.at("spec").dump()));
    adopt(svc, cr, hash);
    adopt(sts, cr, hash);
    std::string phase, message;
    bool requeue = false;
    IngressState ing;
    // kept if the ingress pass fails: the next pass still knows what to clean up
    ing.middleware = cr.get_string("status.ingressMiddleware", "");
    try {
      reconcile_service(cr, ns, name, s, svc);
      requeue = reconcile_statefulset(ns, name, s, sts, hash, phase, message);
      ing = reconcile_ingress(cr, ns, name, s, hash);
      if (ing.pending) requeue = true;
    } catch (const std::exception& e) {
      phase = "Failed";
      message = e.what();
      log(ns, name, std::string("reconcile failed: ") + e.what());
    }
    update_status(cr, s, phase, message, ing);
    return requeue;
  }

  void cleanup(const Json& cr) {
    const std::string name = object_name(cr);
    const std::string ns = cr.get_string("metadata.namespace", "default");
    const std::string api = cr.get_string("spec.ingress.apiVersion", "networking.k8s.io/v1");
    const ResourceKind& ik = api == "networking.k8s.io/v1beta1" ? kinds::IngressV1beta1 : kinds::IngressV1;
    std::vector<std::pair<const ResourceKind*, std::string>> owned{
        {&ik, name + "-ingress"}, {&kinds::StatefulSet, name + "-stateful-set"}, {&kinds::Service, name + "-service"}};
    const std::string mw = cr.get_string("status.ingressMiddleware", "");
    if (!mw.empty())
      for (const ResourceKind* mk : {&kinds::TraefikMiddleware, &kinds::TraefikMiddlewareLegacy})
        owned.emplace_back(mk, mw);
    for (auto& [k, n] : owned) {
      try {
        c_.remove(*k, ns, n, "Background");
      } catch (const ApiError& e) {
        if (e.status != 404 && e.status != 405) log(ns, name, std::string("cleanup: ") + e.what());
      } catch (const std::exception& e) {
        log(ns, name, std::string("cleanup: ") + e.what());
      }
    }
    log(ns, name, "deleted");
  }

 private:
  struct IngressState {
    bool enabled = false, pending = false;
    std::string ip, path;
    std::string middleware;   // the StripPrefix middleware this CR owns ("" = none)
  };

  void reconcile_service(const Json& cr, const std::string& ns, const std::string& name,
                         const DeploymentSpecification& s, const Json& svc) {
    auto cur = c_.get_opt(kinds::Service, ns, s.name + "-service");
    if (!cur) {
      c_.create(kinds::Service, ns, svc);
      log(ns, name, "created service " + s.name + "-service");
    } else if (service_drifted(*cur, svc)) {
      // merge patch replaces the lists wholesale: ports / selector back to the template
      Json patch = Json::object();
      patch["spec"]["ports"] = svc.at("spec").at("ports");
      patch["spec"]["selector"] = svc.at("spec").at("selector");
      c_.merge_patch(kinds::Service, ns, s.name + "-service", patch);
      log(ns, name, "service drifted from the template: repaired ports / selector");
    }
    (void)cr;
  }

  // An H2O cloud has a fixed size and configuration, so a spec change replaces
  // the StatefulSet: delete with Foreground propagation (pods go first), and
  // create the new one only once the old object is really gone.  A real
  // apiserver keeps a foreground-deleted object (deletionTimestamp set) until
  // its pods are removed and answers 409 AlreadyExists to a create meanwhile.
  bool reconcile_statefulset(const std::string& ns, const std::string& name, const DeploymentSpecification& s,
                             const Json& sts, const std::string& hash, std::string& phase, std::string& message) {
    const std::string sname = s.name + "-stateful-set";
    auto cur = c_.get_opt(kinds::StatefulSet, ns, sname);
    if (cur && cur->path("metadata.deletionTimestamp")) {
      phase = "Replacing";
      message = "waiting for the previous statefulset to terminate";
      return true;
    }
    if (cur) {
      const std::string* have = annotation(*cur, "h2o.ai/spec-hash");
      if (have && *have == hash) return false;
      c_.remove(kinds::StatefulSet, ns, sname, "Foreground");
      log(ns, name, "spec changed: deleting statefulset (foreground)");
      if (c_.get_opt(kinds::StatefulSet, ns, sname)) {
        phase = "Replacing";
        message = "waiting for the previous statefulset to terminate";
        return true;
      }
    }
    try {
      c_.create(kinds::StatefulSet, ns, sts);
    } catch (const ApiError& e) {
      if (e.status != 409) throw;
      phase = "Replacing";
      message = "waiting for the previous statefulset to terminate";
      return true;
    }
    log(ns, name, std::string(cur ? "recreated" : "created") + " statefulset " + sname);
    return false;
  }

  // spec.ingress {enabled, apiVersion}: the operator owns <name>-ingress
  // (h2ok's third verb, reference src/k8s/mod.rs:166-199) and reports the
  // load-balancer address in status (reference any_ip / any_path).
  IngressState reconcile_ingress(const Json& cr, const std::string& ns, const std::string& name,
                                 DeploymentSpecification s, const std::string& hash) {
    IngressState st;
    const Json* spec_ing = cr.path("spec.ingress");
    st.enabled = spec_ing && spec_ing->is_object() && spec_ing->find("enabled") &&
                 spec_ing->at("enabled").is_bool() && spec_ing->at("enabled").as_bool();
    s.ingress_api = cr.get_string("spec.ingress.apiVersion", "networking.k8s.io/v1");
    s.ingress_class = cr.get_string("spec.ingress.className", "");
    if (!valid_ingress_class(s.ingress_class)) s.ingress_class.clear();
    if (st.enabled && s.ingress_class.empty()) {
      // no className: the cluster's default IngressClass decides the route form
      s.ingress_class = default_ingress_class(c_);
      s.ingress_class_from_cluster = !s.ingress_class.empty();
    }
    const ResourceKind& ik = s.ingress_api == "networking.k8s.io/v1beta1" ? kinds::IngressV1beta1 : kinds::IngressV1;
    const ResourceKind& other = &ik == &kinds::IngressV1 ? kinds::IngressV1beta1 : kinds::IngressV1;
    const std::string iname = s.name + "-ingress";
    auto drop = [&](const ResourceKind& k) {
      try {
        c_.remove(k, ns, iname, "Background");
        log(ns, name, "deleted ingress " + iname + " (" + k.api + ")");
      } catch (const ApiError& e) {
        if (e.status != 404 && e.status != 405) throw;
      }
    };
    // Traefik v2 StripPrefix middleware (Traefik mode), owned like the ingress
    // (ownerReference: garbage-collected with the CR).  The operator only ever
    // touches a middleware it created - recorded in status.ingressMiddleware -
    // so a cluster without the Traefik CRDs, or an RBAC role without them,
    // never sees a middleware request from a CR that does not use Traefik.
    const std::string mname = s.name + "-stripprefix";
    const std::string recorded = cr.get_string("status.ingressMiddleware", "");
    auto drop_mw = [&]() {
      if (recorded.empty()) return;
      for (const ResourceKind* mk : {&kinds::TraefikMiddleware, &kinds::TraefikMiddlewareLegacy}) {
        try {
          c_.remove(*mk, ns, recorded, "Background");
          log(ns, name, "deleted middleware " + recorded);
        } catch (const ApiError& e) {
          // 404 / 405: not served or already gone; 403: not ours to touch
          if (e.status != 404 && e.status != 405 && e.status != 403) throw;
        }
      }
    };
    if (!st.enabled) {
      if (c_.get_opt(ik, ns, iname)) drop(ik);
      drop_mw();
      return st;
    }
    if (s.ingress_class == "traefik") {
      // a Traefik-mode CR needs the middleware RBAC (deploy/operator.yaml grants
      // it): a 403 here fails this CR with the apiserver's message
      bool have = false;
      for (const ResourceKind* mk : {&kinds::TraefikMiddleware, &kinds::TraefikMiddlewareLegacy})
        if (!have && c_.get_opt(*mk, ns, mname)) have = true;
      if (!have) {
        try {
          create_strip_prefix_middleware(c_, s, [&](Json& mw) { adopt(mw, cr, hash); });
          log(ns, name, "created middleware " + mname);
        } catch (const ApiError& e) {
          if (e.status != 409) throw;   // created meanwhile
        }
      }
      st.middleware = mname;
    } else {
      drop_mw();
    }
    Json ing = h2o_ingress(s);
    adopt(ing, cr, hash);
    auto cur = c_.get_opt(ik, ns, iname);
    if (!cur) {
      // apiVersion switched: the object under the other API group goes first
      try {
        if (c_.get_opt(other, ns, iname)) drop(other);
      } catch (const ApiError&) {
      }
      cur = c_.create(ik, ns, ing);
      log(ns, name, "created ingress " + iname);
    }
    if (auto ip = any_ip(*cur)) st.ip = *ip;
    if (auto p = any_path(*cur)) st.path = *p;
    st.pending = st.ip.empty();   // poll until the load balancer publishes an address
    return st;
  }

  void update_status(const Json& cr, const DeploymentSpecification& s, std::string phase, const std::string& msg,
                     const IngressState& ing) {
    const std::string ns = s.ns;
    int ready = 0, total = 0;
    std::string leader, leader_ip;
    try {
      Json pods = c_.list(kinds::Pod, ns, "app=" + s.name);
      if (const Json* items = pods.find("items"))
        for (auto& p : items->as_array()) {
          ++total;
          if (const Json* conds = p.path("status.conditions"))
            if (conds->is_array())
              for (auto& c : conds->as_array())
                if (c.get_string("type") == "Ready" && c.get_string("status") == "True") {
                  ++ready;
                  leader = object_name(p);
                  leader_ip = p.get_string("status.podIP");
                }
        }
    } catch (...) {
    }
    if (phase.empty()) phase = (total == 0) ? "Pending" : (ready > 0 ? "Ready" : "Forming");
    Json st = Json::object();
    st["phase"] = phase;
    st["nodes"] = (int64_t)s.num_h2o_nodes;
    st["readyNodes"] = ready;  // leader-only readiness: 1 when the cloud is formed
    st["pods"] = total;
    st["leaderPod"] = leader;
    st["serviceName"] = s.name + "-service";
    st["observedGeneration"] = cr.get_int("metadata.generation", 0);
    if (!msg.empty()) st["message"] = msg;
    const Json* old = cr.find("status");
    if (!leader.empty()) {
      // GPU peer topology + collective transport as the formed cloud reports it
      // (/3/Cloud h2omx_topology): a pod-per-GPU deployment without peer
      // visibility shows up here, not only in the leader's log.  A cloud's
      // topology is fixed once formed, so it is fetched only when the leader or
      // the phase changed (or it is still missing), not on every reconcile.
      const Json* ot = (old && old->is_object()) ? old->find("topology") : nullptr;
      if (ot && !ot->is_null() && old->get_string("leaderPod") == leader && old->get_string("phase") == phase) {
        st["topology"] = ot->deep_copy();
      } else {
        Json topo = leader_topology(leader, leader_ip);
        if (!topo.is_null()) st["topology"] = topo;
      }
    }
    if (!ing.middleware.empty()) st["ingressMiddleware"] = ing.middleware;
    if (ing.enabled) {
      st["ingressIP"] = ing.ip;
      st["ingressPath"] = ing.path;
      if (!ing.ip.empty()) st["connectURL"] = "http://" + ing.ip + ":80/" + s.name;
    }
    if (old && old->is_object()) {
      Json cmp = st.deep_copy();
      if (*old == cmp) return;
    }
    Json patch = Json::object();
    Json pst = st.deep_copy();
    // a merge patch only removes keys that are explicitly null: clear a stale
    // message / ingress address / topology (leader gone) from an earlier pass
    if (old && old->is_object())
      for (const char* k : {"message", "ingressIP", "ingressPath", "connectURL", "topology", "ingressMiddleware"})
        if (old->has(k) && !st.has(k)) pst[k] = Json();
    patch["status"] = pst;
    try {
      c_.merge_patch(kinds::H2O, ns, s.name, patch, "status");
    } catch (const ApiError& e) {
      if (e.status == 404 || e.status == 405) {
        try {
          c_.merge_patch(kinds::H2O, ns, s.name, patch);
        } catch (...) {
        }
      }
    } catch (...) {
    }
  }

  // GET <leader>/3/Cloud and return its h2omx_topology (null when unreachable).
  // The leader serves the H2O REST API on :54321 at its pod IP;
  // H2OMX_OPERATOR_CLOUD_URL ("http://host:port", "{pod}" replaced by the
  // leader pod name) overrides that address (local test clusters).
  Json leader_topology(const std::string& pod, const std::string& ip) {
    std::string base;
    if (const char* o = std::getenv("H2OMX_OPERATOR_CLOUD_URL")) {
      base = o;
      const auto k = base.find("{pod}");
      if (k != std::string::npos) base.replace(k, 5, pod);
    } else if (!ip.empty()) {
      base = "http://" + ip + ":54321";
    } else {
      return Json();
    }
    try {
      HttpRequest req;
      req.target = "/3/Cloud";
      req.timeout_s = 3.0;
      HttpResponse r = http_request(parse_url(base), req, TlsConfig{});
      if (r.status != 200) return Json();
      Json cloud = Json::parse(r.body);
      if (const Json* t = cloud.find("h2omx_topology")) return t->deep_copy();
    } catch (...) {
    }
    return Json();
  }

  void log(const std::string& ns, const std::string& name, const std::string& what) {
    std::cout << "[h2omx-operator] " << ns << "/" << name << ": " << what << std::endl;
  }

  KubeClient& c_;
  Options o_;
};

int usage() {
  std::cerr << "usage: h2omx-operator [--kubeconfig PATH] [--namespace NS] [--once] [--resync SECONDS] [--requeue SECONDS]\n"
               "                      [--image NAME] [--image-tag TAG]\n";
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--kubeconfig" || a == "-k") o.kubeconfig = next();
    else if (a == "--namespace" || a == "-n") o.ns = next();
    else if (a == "--once") o.once = true;
    else if (a == "--resync") o.resync_s = std::max(1, std::atoi(next().c_str()));
    else if (a == "--requeue") o.requeue_s = std::max(1, std::atoi(next().c_str()));
    else if (a == "--image") o.default_image = next();
    else if (a == "--image-tag") o.default_tag = next();
    else if (a == "-h" || a == "--help") return usage(), 0;
    else return usage();
  }
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  std::optional<KubeClient> client;
  try {
    client.emplace(o.kubeconfig ? load_kubeconfig(*o.kubeconfig) : infer_kubeconfig());
  } catch (const std::exception& e) {
    std::cerr << "h2omx-operator: cannot configure Kubernetes client: " << e.what() << std::endl;
    return 1;
  }
  Reconciler rec(*client, o);
  std::cout << "[h2omx-operator] watching h2os.h2o.ai/v1beta in "
            << (o.ns.empty() ? std::string("all namespaces") : "namespace " + o.ns) << std::endl;
  while (!g_stop) {
    std::string rv;
    bool requeue = false;
    try {
      Json lst = client->list(kinds::H2O, o.ns);
      rv = lst.get_string("metadata.resourceVersion");
      for (auto& cr : lst.at("items").as_array()) requeue |= rec.reconcile(cr);
    } catch (const std::exception& e) {
      std::cerr << "[h2omx-operator] list failed: " << e.what() << std::endl;
      if (o.once) return 1;
      std::this_thread::sleep_for(std::chrono::seconds(2));
      continue;
    }
    if (o.once) break;
    try {
      // a pending replacement / ingress address: re-list after a short watch
      client->watch(kinds::H2O, o.ns, "", rv, requeue ? o.requeue_s : o.resync_s, [&](const WatchEvent& ev) {
        if (g_stop) return false;
        // a CR that needs another pass soon ends this watch: the loop re-lists
        // and then watches with the short requeue timeout
        if (ev.type == "ADDED" || ev.type == "MODIFIED") return !rec.reconcile(ev.object);
        else if (ev.type == "DELETED") rec.cleanup(ev.object);
        return true;
      });
    } catch (const std::exception& e) {
      std::cerr << "[h2omx-operator] watch ended: " << e.what() << std::endl;
      std::this_thread::sleep_for(std::chrono::seconds(1));
    }
  }
  return 0;
}
