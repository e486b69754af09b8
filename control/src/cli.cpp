#include "cli.hpp"
#include "platform.hpp"


#include <cstdio>
#include <iostream>
#include <iterator>
#include <random>
#include <sstream>

#include "deployment.hpp"

namespace h2ok {

namespace {

struct ArgSpec {
  std::string id;
  std::string long_name;
  std::string short_name;  // "" = none
  std::string help;
  std::optional<std::string> default_value;
  bool required = false;
  bool flag = false;  // takes no value
  std::vector<std::string> aliases;
  enum Validator { None, Path, IntGtZero, Percentage, Memory, UInt, DnsLabel, IngressApi, IngressClass } validator = None;
};

struct SubSpec {
  std::string name;
  std::string about;
  std::vector<ArgSpec> args;
};

std::vector<SubSpec> build_app() {
  std::vector<SubSpec> subs;
  SubSpec deploy{"deploy",
                 "Deploys an H2O cluster into Kubernetes. Once successfully deployed a deployment descriptor file "
                 "with cluster name is saved.Such a file can be used to undeploy the cluster or built on top of by "
                 "adding additional services.",
                 {}};
  deploy.args.push_back({"cluster_size", "cluster_size", "s", "Number of H2O Nodes in the cluster. Up to 2^32.",
                         std::nullopt, true, false, {"cluster-size"}, ArgSpec::IntGtZero});
  deploy.args.push_back({"kubeconfig", "kubeconfig", "k",
                         "Path to 'kubeconfig' yaml file. If not specified, well-known locations are scanned for "
                         "kubeconfig.",
                         std::nullopt, false, false, {}, ArgSpec::Path});
  deploy.args.push_back({"namespace", "namespace", "n",
                         "Kubernetes cluster namespace to connect to. If not specified, kubeconfig default is used.",
                         std::nullopt, false, false, {}, ArgSpec::DnsLabel});
  deploy.args.push_back({"name", "cluster_name", "c",
                         "Name of the H2O cluster deployment. Used as prefix for K8S entities. Generated if not "
                         "specified.",
                         std::nullopt, false, false, {"cluster-name"}, ArgSpec::DnsLabel});
  deploy.args.push_back({"memory_percentage", "memory_percentage", "p",
                         "Memory percentage allocated by H2O inside the container. <0,100>. Defaults to 50% to make "
                         "space for XGBoost.",
                         std::string("50"), false, false, {"memory-percentage"}, ArgSpec::Percentage});
  deploy.args.push_back({"memory", "memory", "m",
                         "Amount of memory allocated by each H2O node - in a format accepted by K8S, e.g. 4Gi.",
                         std::string("1Gi"), false, false, {}, ArgSpec::Memory});
  deploy.args.push_back({"cpus", "cpus", "", "Number of CPUs allocated for each H2O node.", std::string("1"), false,
                         false, {}, ArgSpec::IntGtZero});
  deploy.args.push_back({"gpus_per_node", "gpus_per_node", "g",
                         "AMD Instinct GPUs (amd.com/gpu) per H2O node; one rank per GPU.", std::string("1"), false,
                         false, {"gpus-per-node"}, ArgSpec::UInt});
  deploy.args.push_back({"image", "image", "", "Node container image name.", std::string("h2omx/h2omx-node"), false,
                         false, {}, ArgSpec::None});
  deploy.args.push_back({"image_tag", "image_tag", "", "Node container image tag.", std::string("latest"), false,
                         false, {"image-tag"}, ArgSpec::None});
  deploy.args.push_back({"ingress_api", "ingress_api", "",
                         "Ingress API version used by later 'ingress' calls: networking.k8s.io/v1 or "
                         "networking.k8s.io/v1beta1.",
                         std::string("networking.k8s.io/v1"), false, false, {"ingress-api"}, ArgSpec::IngressApi});
  deploy.args.push_back({"ingress_class", "ingress_class", "",
                         "Ingress controller of later 'ingress' calls: nginx, traefik (Traefik v2, e.g. K3s: Prefix "
                         "path + StripPrefix middleware) or empty for the cluster default class (nginx-style paths).",
                         std::string(""), false, false, {"ingress-class"}, ArgSpec::IngressClass});
  deploy.args.push_back({"dry_run", "dry_run", "", "Print the Kubernetes manifests as YAML instead of deploying.",
                         std::nullopt, false, true, {"dry-run"}, ArgSpec::None});
  subs.push_back(deploy);

  SubSpec undeploy{"undeploy", "Undeploys an existing H2O cluster from Kubernetes", {}};
  undeploy.args.push_back({"file", "file", "f",
                           "H2O deployment descriptor file path. If not specified, attempt is made to parse "
                           "deployment descriptor path from stdin.",
                           std::nullopt, false, false, {}, ArgSpec::Path});
  subs.push_back(undeploy);

  SubSpec ingress{"ingress", "Creates an ingress pointing to the given H2O K8S deployment", {}};
  ingress.args.push_back(undeploy.args[0]);
  subs.push_back(ingress);

  SubSpec status{"status", "Shows the pods, readiness and leader of an existing H2O deployment", {}};
  status.args.push_back(undeploy.args[0]);
  subs.push_back(status);
  return subs;
}

std::string opt_sig(const ArgSpec& a) {
  std::string sig = a.short_name.empty() ? "    " : "-" + a.short_name + ", ";
  sig += "--" + a.long_name;
  if (!a.flag) sig += " <" + a.id + ">";
  return sig;
}

std::string usage_line(const SubSpec& s) {
  std::string u = "h2ok " + s.name + " [FLAGS] [OPTIONS]";
  for (auto& a : s.args)
    if (a.required) u += " --" + a.long_name + " <" + a.id + ">";
  return u;
}

std::string sub_help(const SubSpec& s) {
  std::ostringstream os;
  os << "h2ok-" << s.name << " \n" << s.about << "\n\nUSAGE:\n    " << usage_line(s) << "\n\nFLAGS:\n";
  std::vector<std::pair<std::string, std::string>> flags = {{"-h, --help", "Prints help information"},
                                                            {"-V, --version", "Prints version information"}};
  for (auto& a : s.args)
    if (a.flag) flags.push_back({"    --" + a.long_name, a.help});
  size_t w = 0;
  for (auto& f : flags) w = std::max(w, f.first.size());
  for (auto& f : flags) os << "    " << f.first << std::string(w - f.first.size() + 4, ' ') << f.second << "\n";
  std::vector<std::pair<std::string, std::string>> opts;
  for (auto& a : s.args) {
    if (a.flag) continue;
    std::string h = a.help;
    if (a.default_value) h += " [default: " + *a.default_value + "]";
    opts.push_back({opt_sig(a), h});
  }
  if (!opts.empty()) {
    os << "\nOPTIONS:\n";
    w = 0;
    for (auto& o : opts) w = std::max(w, o.first.size());
    for (auto& o : opts) os << "    " << o.first << std::string(w - o.first.size() + 4, ' ') << o.second << "\n";
  }
  return os.str();
}

std::string general_help(const std::vector<SubSpec>& subs) {
  std::ostringstream os;
  os << kAppName << " " << kAppVersion << "\n\nUSAGE:\n    h2ok <SUBCOMMAND>\n\nFLAGS:\n"
     << "    -h, --help       Prints help information\n"
     << "    -V, --version    Prints version information\n\nSUBCOMMANDS:\n";
  std::vector<std::pair<std::string, std::string>> rows;
  for (auto& s : subs) rows.push_back({s.name, s.about});
  rows.push_back({"help", "Prints this message or the help of the given subcommand(s)"});
  std::sort(rows.begin(), rows.end());
  for (auto& r : rows) os << "    " << r.first << std::string(12 - std::min<size_t>(r.first.size(), 11), ' ') << r.second << "\n";
  return os.str();
}

bool is_file(const std::string& p) { return plat::is_regular_file(p); }

std::optional<std::string> validate(const ArgSpec& a, const std::string& v) {
  auto parse_int = [&](long long& out) -> bool {
    try {
      size_t used = 0;
      out = std::stoll(v, &used);
      return used == v.size();
    } catch (...) {
      return false;
    }
  };
  long long n = 0;
  switch (a.validator) {
    case ArgSpec::Path:
      if (!is_file(v)) return "Invalid file path: '" + v + "'";
      return std::nullopt;
    case ArgSpec::IntGtZero:
      if (!parse_int(n)) return "Error: '" + v + "' is not an integer.";
      if (n < 1) return std::string("Error: The number provided must be greater than zero.");
      if (n > 4294967295LL) return std::string("Error: The number must be at most 2^32-1.");
      return std::nullopt;
    case ArgSpec::UInt:
      if (!parse_int(n) || n < 0 || n > 64) return "Error: '" + v + "' must be an integer in <0,64>.";
      return std::nullopt;
    case ArgSpec::Percentage:
      if (!parse_int(n)) return "Error: '" + v + "' is not an integer.";
      if (n < 0 || n > 100) return std::string("Error: The number must be withing range <0,100>.");
      return std::nullopt;
    case ArgSpec::Memory:
      if (!valid_memory_quantity(v))
        return std::string(
            "Memory requirement must match the following pattern: ^([+-]?[0-9.]+)([eEinumkKMGTP]*[-+]?[0-9]*)$. "
            "For example 1Gi or 1024Mi.");
      return std::nullopt;
    case ArgSpec::DnsLabel:
      if (!valid_dns_label(v))
        return "Error: '" + v + "' must be a lowercase DNS-1123 label (a-z, 0-9, '-'; at most 52 characters).";
      return std::nullopt;
    case ArgSpec::IngressClass:
      if (!valid_ingress_class(v)) return "Error: unsupported ingress class '" + v + "' (nginx or traefik).";
      return std::nullopt;
    case ArgSpec::IngressApi:
      if (v != "networking.k8s.io/v1" && v != "networking.k8s.io/v1beta1")
        return "Error: unsupported ingress API '" + v + "'.";
      return std::nullopt;
    default:
      return std::nullopt;
  }
}

std::string trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n");
  if (b == std::string::npos) return "";
  size_t e = s.find_last_not_of(" \t\r\n");
  return s.substr(b, e - b + 1);
}

}  // namespace

std::string UserInputError::debug() const {
  return std::string("UserInputError { kind: ") +
         (kind == CommandErrorKind::MissingDeploymentDescriptor ? "MissingDeploymentDescriptor"
                                                                 : "UnreachableDeploymentDescriptor") +
         " }";
}

std::string generate_cluster_name() {
  static const char* adj[] = {"agile", "bold", "brisk", "calm", "clever", "cosmic", "crisp", "daring", "eager",
                              "fast", "fierce", "gentle", "glowing", "grand", "happy", "keen", "lively", "lucid",
                              "mighty", "nimble", "noble", "polar", "quick", "quiet", "rapid", "sharp", "silent",
                              "solar", "steady", "swift", "tidy", "vivid", "witty", "zesty"};
  static const char* noun[] = {"falcon", "otter", "comet", "photon", "quasar", "raven", "tiger", "maple", "river",
                               "summit", "aurora", "cobalt", "ember", "harbor", "lynx", "nebula", "orbit", "pine",
                               "prism", "spark", "vertex", "willow", "zephyr", "meteor", "canyon", "glacier"};
  std::random_device rd;
  std::mt19937 g(rd());
  return std::string("h2o-") + adj[g() % (sizeof adj / sizeof *adj)] + "-" + noun[g() % (sizeof noun / sizeof *noun)];
}

ParseOutcome parse_command_line(const std::vector<std::string>& args, const std::string& stdin_override,
                                bool use_stdin_override) {
  ParseOutcome out;
  const auto subs = build_app();
  if (args.empty()) {  // ArgRequiredElseHelp
    std::cerr << general_help(subs);
    out.done = true;
    out.exit_code = 1;
    return out;
  }
  const std::string& first = args[0];
  if (first == "-h" || first == "--help" || first == "help") {
    if (first == "help" && args.size() > 1) {
      for (auto& s : subs)
        if (s.name == args[1]) {
          std::cout << sub_help(s);
          out.done = true;
          return out;
        }
    }
    std::cout << general_help(subs);
    out.done = true;
    return out;
  }
  if (first == "-V" || first == "--version") {
    std::cout << kAppName << " " << kAppVersion << "\n";
    out.done = true;
    return out;
  }
  const SubSpec* sub = nullptr;
  for (auto& s : subs)
    if (s.name == first) sub = &s;
  if (!sub) {
    std::cerr << "error: Found argument '" << first << "' which wasn't expected, or isn't valid in this context\n\n"
              << "USAGE:\n    h2ok <SUBCOMMAND>\n\nFor more information try --help\n";
    out.done = true;
    out.exit_code = 1;
    return out;
  }
  std::map<std::string, std::string> vals;
  for (size_t i = 1; i < args.size(); ++i) {
    std::string a = args[i];
    if (a == "-h" || a == "--help") {
      std::cout << sub_help(*sub);
      out.done = true;
      return out;
    }
    if (a == "-V" || a == "--version") {
      std::cout << "h2ok-" << sub->name << " \n";
      out.done = true;
      return out;
    }
    std::string inline_val;
    bool has_inline = false;
    if (a.rfind("--", 0) == 0) {
      size_t eq = a.find('=');
      if (eq != std::string::npos) {
        inline_val = a.substr(eq + 1);
        a = a.substr(0, eq);
        has_inline = true;
      }
    }
    const ArgSpec* spec = nullptr;
    for (auto& s : sub->args) {
      if (a == "--" + s.long_name || (!s.short_name.empty() && a == "-" + s.short_name)) spec = &s;
      for (auto& al : s.aliases)
        if (a == "--" + al) spec = &s;
    }
    if (!spec) {
      std::cerr << "error: Found argument '" << args[i] << "' which wasn't expected, or isn't valid in this context\n\n"
                << "USAGE:\n    " << usage_line(*sub) << "\n\nFor more information try --help\n";
      out.done = true;
      out.exit_code = 1;
      return out;
    }
    if (spec->flag) {
      vals[spec->id] = "true";
      continue;
    }
    std::string v;
    if (has_inline) {
      v = inline_val;
    } else if (i + 1 < args.size()) {
      v = args[++i];
    } else {
      std::cerr << "error: The argument '" << opt_sig(*spec).substr(4)
                << "' requires a value but none was supplied\n\nUSAGE:\n    " << usage_line(*sub)
                << "\n\nFor more information try --help\n";
      out.done = true;
      out.exit_code = 1;
      return out;
    }
    if (auto err = validate(*spec, v)) {
      std::cerr << "error: Invalid value for '--" << spec->long_name << " <" << spec->id << ">': " << *err << "\n";
      out.done = true;
      out.exit_code = 1;
      return out;
    }
    vals[spec->id] = v;
  }
  std::vector<const ArgSpec*> missing;
  for (auto& s : sub->args)
    if (s.required && !vals.count(s.id)) missing.push_back(&s);
  if (!missing.empty()) {
    std::cerr << "error: The following required arguments were not provided:\n";
    for (auto* m : missing) std::cerr << "    --" << m->long_name << " <" << m->id << ">\n";
    std::cerr << "\nUSAGE:\n    " << usage_line(*sub) << "\n\nFor more information try --help\n";
    out.done = true;
    out.exit_code = 1;
    return out;
  }
  for (auto& s : sub->args)
    if (!vals.count(s.id) && s.default_value) vals[s.id] = *s.default_value;

  Command cmd;
  if (sub->name == "deploy") {
    cmd.kind = CommandKind::Deploy;
    auto& d = cmd.deployment;
    d.name = vals.count("name") ? vals["name"] : generate_cluster_name();
    if (vals.count("namespace")) d.ns = vals["namespace"];
    d.memory_percentage = std::stoi(vals["memory_percentage"]);
    d.memory = vals["memory"];
    d.num_cpu = (uint32_t)std::stoul(vals["cpus"]);
    d.num_h2o_nodes = (uint32_t)std::stoul(vals["cluster_size"]);
    if (vals.count("kubeconfig")) d.kubeconfig_path = vals["kubeconfig"];
    d.gpus_per_node = (uint32_t)std::stoul(vals["gpus_per_node"]);
    d.image = vals["image"];
    d.image_tag = vals["image_tag"];
    d.ingress_api = vals["ingress_api"];
    d.ingress_class = vals["ingress_class"];
    d.dry_run = vals.count("dry_run") > 0;
    if (d.dry_run) cmd.kind = CommandKind::Template;
    out.command = cmd;
    return out;
  }
  // undeploy / ingress / status: -f, else the path is read from stdin (Q8, Q9)
  cmd.kind = sub->name == "undeploy" ? CommandKind::Undeploy
                                     : (sub->name == "ingress" ? CommandKind::Ingress : CommandKind::Status);
  if (vals.count("file")) {
    cmd.descriptor_path = vals["file"];
    out.command = cmd;
    return out;
  }
  std::string in;
  if (use_stdin_override) {
    in = stdin_override;
  } else {
    std::ostringstream os;
    os << std::cin.rdbuf();
    in = os.str();
  }
  std::string path = trim(in);
  if (path.empty()) {
    out.input_error = UserInputError{CommandErrorKind::MissingDeploymentDescriptor};
    return out;
  }
  if (is_file(path)) {
    cmd.descriptor_path = path;
  } else {
    std::string rel = plat::current_dir() + "/" + path;
    if (!is_file(rel)) {
      out.input_error = UserInputError{CommandErrorKind::UnreachableDeploymentDescriptor};
      return out;
    }
    cmd.descriptor_path = rel;
  }
  out.command = cmd;
  return out;
}

}  // namespace h2ok
