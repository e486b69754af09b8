// h2omx-operator: reconciles `H2O` custom resources (h2o.ai/v1beta) into the
// same headless Service + StatefulSet pair `h2ok deploy` creates, one pod per
// MI355X (amd.com/gpu: 1), and reports status (phase, readyNodes, leaderPod).
//
// The reference snapshot has no operator (kube-derive is declared but unused,
// Cargo.toml:10 of isgasho/h2o-kubernetes); the CR schema mirrors its
// DeploymentSpecification (src/k8s/mod.rs:58-74) as designed in SURVEY.md §7.2.
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <iostream>
#include <map>
#include <thread>

#include "deployment.hpp"
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

class Reconciler {
 public:
  Reconciler(KubeClient& c, Options o) : c_(c), o_(std::move(o)) {}

  void reconcile(const Json& cr) {
    const std::string name = object_name(cr);
    const std::string ns = cr.get_string("metadata.namespace", "default");
    if (cr.path("metadata.deletionTimestamp")) return;  // GC via ownerReferences
    DeploymentSpecification s = spec_from_cr(cr, o_);
    Json svc = h2o_service(s);
    Json sts = h2o_stateful_set(s);
    const std::string hash = hex(fnv1a(sts.at("spec").dump() + svc.at("spec").dump()));
    adopt(svc, cr, hash);
    adopt(sts, cr, hash);
    std::string phase, message;
    try {
      if (!c_.get_opt(kinds::Service, ns, s.name + "-service")) {
        c_.create(kinds::Service, ns, svc);
        log(ns, name, "created service " + s.name + "-service");
      }
      auto cur = c_.get_opt(kinds::StatefulSet, ns, s.name + "-stateful-set");
      if (!cur) {
        c_.create(kinds::StatefulSet, ns, sts);
        log(ns, name, "created statefulset " + s.name + "-stateful-set");
      } else if (cur->get_string("metadata.annotations.h2o.ai/spec-hash") != hash &&
                 cur->path("metadata.annotations") &&
                 cur->path("metadata.annotations")->find("h2o.ai/spec-hash") &&
                 cur->path("metadata.annotations")->at("h2o.ai/spec-hash").as_string() != hash) {
        // An H2O cloud has a fixed size and configuration: replace it.
        c_.remove(kinds::StatefulSet, ns, s.name + "-stateful-set", "Foreground");
        c_.create(kinds::StatefulSet, ns, sts);
        log(ns, name, "spec changed: recreated statefulset");
      }
    } catch (const std::exception& e) {
      phase = "Failed";
      message = e.what();
      log(ns, name, std::string("reconcile failed: ") + e.what());
    }
    update_status(cr, s, phase, message);
  }

  void cleanup(const Json& cr) {
    const std::string name = object_name(cr);
    const std::string ns = cr.get_string("metadata.namespace", "default");
    for (auto& [k, n] : std::vector<std::pair<const ResourceKind*, std::string>>{
             {&kinds::StatefulSet, name + "-stateful-set"}, {&kinds::Service, name + "-service"}}) {
      try {
        c_.remove(*k, ns, n, "Background");
      } catch (const ApiError& e) {
        if (e.status != 404) log(ns, name, std::string("cleanup: ") + e.what());
      } catch (const std::exception& e) {
        log(ns, name, std::string("cleanup: ") + e.what());
      }
    }
    log(ns, name, "deleted");
  }

 private:
  void update_status(const Json& cr, const DeploymentSpecification& s, std::string phase, const std::string& msg) {
    const std::string ns = s.ns;
    int ready = 0, total = 0;
    std::string leader;
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
    if (old && old->is_object()) {
      Json cmp = st.deep_copy();
      if (*old == cmp) return;
    }
    Json patch = Json::object();
    patch["status"] = st;
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

  void log(const std::string& ns, const std::string& name, const std::string& what) {
    std::cout << "[h2omx-operator] " << ns << "/" << name << ": " << what << std::endl;
  }

  KubeClient& c_;
  Options o_;
};

int usage() {
  std::cerr << "usage: h2omx-operator [--kubeconfig PATH] [--namespace NS] [--once] [--resync SECONDS]\n"
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
    try {
      Json lst = client->list(kinds::H2O, o.ns);
      rv = lst.get_string("metadata.resourceVersion");
      for (auto& cr : lst.at("items").as_array()) rec.reconcile(cr);
    } catch (const std::exception& e) {
      std::cerr << "[h2omx-operator] list failed: " << e.what() << std::endl;
      if (o.once) return 1;
      std::this_thread::sleep_for(std::chrono::seconds(2));
      continue;
    }
    if (o.once) break;
    try {
      client->watch(kinds::H2O, o.ns, "", rv, o.resync_s, [&](const WatchEvent& ev) {
        if (g_stop) return false;
        if (ev.type == "ADDED" || ev.type == "MODIFIED") rec.reconcile(ev.object);
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
