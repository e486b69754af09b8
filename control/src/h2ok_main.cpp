// h2ok: deploy / undeploy / expose an MI355X H2O (h2omx) cluster on
// Kubernetes.  Behavioural parity with src/main.rs of isgasho/h2o-kubernetes
// (command dispatch :18-37, deploy :39-69, persist :71-101, undeploy
// :103-115, ingress :117-141, descriptor load :143-164, TTY switch :166-169);
// deviations are the fixes listed in SURVEY.md §7.6 (Q1, Q4-Q7, Q13).

#include <iostream>

#include "cli.hpp"
#include "deployment.hpp"
#include "platform.hpp"
#include "k8s.hpp"
#include "yaml.hpp"

using namespace h2ok;

namespace {

constexpr int kExitPanic = 101;  // the reference's exit status on a panic

bool running_on_terminal() { return plat::stdout_is_tty(); }

KubeClient client_for(const std::optional<std::string>& kubeconfig) {
  if (kubeconfig) return KubeClient(load_kubeconfig(*kubeconfig));
  return KubeClient(infer_kubeconfig());
}

DeploymentSpecification to_spec(const UserDeploymentSpecification& u, const std::string& kube_ns) {
  DeploymentSpecification s;
  s.name = u.name;
  s.ns = u.ns ? *u.ns : (kube_ns.empty() ? "default" : kube_ns);  // Q1: honour --namespace
  s.memory_percentage = u.memory_percentage;
  s.memory = u.memory;
  s.num_cpu = u.num_cpu;
  s.num_h2o_nodes = u.num_h2o_nodes;
  s.kubeconfig_path = u.kubeconfig_path;
  s.image = u.image;
  s.image_tag = u.image_tag;
  s.gpus_per_node = u.gpus_per_node;
  s.ingress_api = u.ingress_api;
  s.ingress_class = u.ingress_class;
  return s;
}

int cmd_template(const UserDeploymentSpecification& u) {
  std::string ns = u.ns ? *u.ns : "default";
  if (!u.ns) {
    try {
      ns = client_for(u.kubeconfig_path).default_namespace();
    } catch (...) {
    }
  }
  DeploymentSpecification s = to_spec(u, ns);
  std::cout << yaml_dump(h2o_service(s)) << "---\n" << yaml_dump(h2o_stateful_set(s));
  return 0;
}

int cmd_deploy(const UserDeploymentSpecification& u) {
  std::optional<KubeClient> client;
  try {
    client.emplace(client_for(u.kubeconfig_path));
  } catch (const std::exception& e) {
    if (!u.kubeconfig_path)
      std::cerr << "No kubeconfig provided by the user and search in well-known kubeconfig locations failed: "
                << e.what() << std::endl;
    else
      std::cerr << "Unable to load kubeconfig '" << *u.kubeconfig_path << "': " << e.what() << std::endl;
    return kExitPanic;
  }
  DeploymentSpecification spec = to_spec(u, client->default_namespace());
  Deployment d;
  try {
    d = deploy_h2o_cluster(*client, spec);
  } catch (const std::exception& e) {
    std::cerr << "Unable to deploy H2O cluster. Error:\n" << e.what() << std::endl;
    return kExitPanic;
  }
  std::string file;
  try {
    file = persist_deployment(d, false);
  } catch (const std::exception& e) {
    std::cerr << e.what() << std::endl;
    return kExitPanic;
  }
  if (running_on_terminal()) {
    std::cout << "Deployment of '" << spec.name << "' completed successfully." << std::endl;
    std::cout << "To undeploy, use the 'h2ok undeploy -f " << file << "' command." << std::endl;
  } else {
    std::cout << file << std::flush;  // Q4: the file actually written
  }
  return 0;
}

bool load_existing(const std::string& path, Deployment& d, std::optional<KubeClient>& client) {
  try {
    d = load_deployment(path);
  } catch (const std::exception& e) {
    std::cerr << "Unable to read deployment descriptor '" << path << "': " << e.what() << std::endl;
    return false;
  }
  try {
    client.emplace(client_for(d.specification.kubeconfig_path));
  } catch (const std::exception& e) {
    std::cerr << "Unable to create a Kubernetes client for '" << d.specification.name << "': " << e.what()
              << std::endl;
    return false;
  }
  return true;
}

int cmd_undeploy(const std::string& path) {
  Deployment d;
  std::optional<KubeClient> client;
  if (!load_existing(path, d, client)) return kExitPanic;
  auto failed = undeploy_h2o(*client, d);
  for (auto& f : failed) std::cout << "Unable to undeploy '" << f << "' - skipping." << std::endl;
  if (!failed.empty()) {
    // Q7: keep the descriptor so the remaining objects can still be removed
    std::cerr << "Deployment '" << d.specification.name << "' partially removed; descriptor kept at '" << path
              << "'." << std::endl;
    return 2;
  }
  std::cout << "Removed deployment '" << d.specification.name << "'." << std::endl;
  std::remove(path.c_str());
  return 0;
}

int cmd_ingress(const std::string& path) {
  Deployment d;
  std::optional<KubeClient> client;
  if (!load_existing(path, d, client)) return kExitPanic;
  try {
    deploy_ingress(*client, d, 3);
  } catch (const std::exception& e) {
    std::cerr << "Unable to create ingress for " << d.specification.name << " deployment. Reason: \n" << e.what()
              << std::endl;
    return kExitPanic;
  }
  std::string file = persist_deployment(d, true, path);  // Q6: rewrite the descriptor we were given
  if (running_on_terminal()) {
    std::cout << "Ingress '" << d.specification.name << "' deployed successfully." << std::endl;
    auto ip = any_ip(d.ingresses.back());
    auto p = any_path(d.ingresses.back());
    if (ip && p) {
      std::cout << "You may now use 'h2o.connect()' to connect to the H2O cluster:" << std::endl;
      std::cout << "Python: 'h2o.connect(url=\"http://" << *ip << ":80" << *p << "\")'" << std::endl;
      std::cout << "R: 'h2o.connect(ip = \"" << *ip << "\", context_path = \"" << p->substr(1) << "\", port=80)'"
                << std::endl;
    }
  } else {
    std::cout << file << std::flush;
  }
  return 0;
}

int cmd_status(const std::string& path) {
  Deployment d;
  std::optional<KubeClient> client;
  if (!load_existing(path, d, client)) return kExitPanic;
  const auto& s = d.specification;
  try {
    Json pods = client->list(kinds::Pod, s.ns, "app=" + s.name);
    int ready = 0, total = 0;
    std::string leader;
    for (auto& p : pods.at("items").as_array()) {
      ++total;
      bool is_ready = false;
      if (const Json* conds = p.path("status.conditions"))
        if (conds->is_array())
          for (auto& c : conds->as_array())
            if (c.get_string("type") == "Ready" && c.get_string("status") == "True") is_ready = true;
      if (is_ready) {
        ++ready;
        leader = object_name(p);
      }
      std::cout << object_name(p) << "\t" << p.get_string("status.phase", "Unknown") << "\t"
                << (is_ready ? "leader" : "-") << "\n";
    }
    std::cout << "Deployment '" << s.name << "': " << total << "/" << s.num_h2o_nodes << " pods, leader "
              << (leader.empty() ? "<none yet>" : leader) << "\n";
  } catch (const std::exception& e) {
    std::cerr << "Unable to query deployment '" << s.name << "': " << e.what() << std::endl;
    return kExitPanic;
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> args(argv + 1, argv + argc);
  ParseOutcome po = parse_command_line(args);
  if (po.done) return po.exit_code;
  if (po.input_error) {
    std::cerr << "Unable to process user input: " << po.input_error->debug() << std::endl;
    return 1;
  }
  const Command& c = *po.command;
  switch (c.kind) {
    case CommandKind::Deploy: return cmd_deploy(c.deployment);
    case CommandKind::Template: return cmd_template(c.deployment);
    case CommandKind::Undeploy: return cmd_undeploy(c.descriptor_path);
    case CommandKind::Ingress: return cmd_ingress(c.descriptor_path);
    case CommandKind::Status: return cmd_status(c.descriptor_path);
  }
  return kExitPanic;
}
