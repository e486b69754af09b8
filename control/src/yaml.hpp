// YAML subset reader/writer for kubeconfig files and manifests.
//
// Supports block mappings and sequences (including "- key: value" compact
// items and sequences indented at their parent key's level), flow
// collections, single/double quoted scalars, literal/folded block scalars,
// comments and "---" document markers: everything kubeconfig files written by
// kubectl, k3s, kind and cloud CLIs use.  YAML documents are converted to the
// same Json value type the rest of the control plane uses.
#pragma once

#include <string>
#include <vector>

#include "json.hpp"

namespace h2ok {

class YamlError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// Parse the first document.
Json yaml_parse(const std::string& text);
// Parse every document of a multi-document stream.
std::vector<Json> yaml_parse_all(const std::string& text);
// Serialise a Json value as block-style YAML.
std::string yaml_dump(const Json& v);

}  // namespace h2ok
