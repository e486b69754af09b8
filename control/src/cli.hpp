// h2ok command-line parsing: same subcommands, flags, defaults, validators,
// help titles and exit codes as the reference's clap app
// (src/cli/mod.rs:160-279 of isgasho/h2o-kubernetes), with the input bugs
// listed in SURVEY.md §7.6 fixed (Q8 trimming, Q9 ingress stdin, Q10 proper
// numeric errors, Q15 --cluster-size alias).
#pragma once

#include <map>
#include <optional>
#include <string>
#include <vector>

namespace h2ok {

constexpr const char* kAppName = "H2O Kubernetes CLI";
constexpr const char* kAppVersion = "0.1.0";

enum class CommandKind { Deploy, Undeploy, Ingress, Status, Template };

struct UserDeploymentSpecification {
  std::string name;
  std::optional<std::string> ns;
  int memory_percentage = 50;
  std::string memory = "1Gi";
  uint32_t num_cpu = 1;
  uint32_t num_h2o_nodes = 1;
  std::optional<std::string> kubeconfig_path;
  std::string image = "h2omx/h2omx-node";
  std::string image_tag = "latest";
  uint32_t gpus_per_node = 1;
  std::string ingress_api = "networking.k8s.io/v1";
  std::string ingress_class;
  bool dry_run = false;
};

enum class CommandErrorKind { MissingDeploymentDescriptor, UnreachableDeploymentDescriptor };

struct UserInputError {
  CommandErrorKind kind;
  std::string debug() const;  // "UserInputError { kind: ... }"
};

struct Command {
  CommandKind kind;
  UserDeploymentSpecification deployment;  // Deploy / Template
  std::string descriptor_path;             // Undeploy / Ingress / Status
};

// Result of parsing: either a command, a user-input error (exit 1 with the
// reference's message), or a terminal outcome already printed (help,
// version, validation error) with its exit code.
struct ParseOutcome {
  std::optional<Command> command;
  std::optional<UserInputError> input_error;
  int exit_code = 0;
  bool done = false;  // help/version/clap-style error already printed
};

ParseOutcome parse_command_line(const std::vector<std::string>& args, const std::string& stdin_override = "",
                                bool use_stdin_override = false);

std::string generate_cluster_name();

}  // namespace h2ok
