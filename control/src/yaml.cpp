#include "yaml.hpp"

#include <cctype>
#include <sstream>

namespace h2ok {

namespace {

struct Line {
  int indent;
  std::string text;  // content without indentation / trailing comment
  int lineno;
};

std::string rstrip(const std::string& s) {
  size_t e = s.size();
  while (e > 0 && std::isspace((unsigned char)s[e - 1])) --e;
  return s.substr(0, e);
}

std::string strip(const std::string& s) {
  size_t b = 0;
  while (b < s.size() && std::isspace((unsigned char)s[b])) ++b;
  return rstrip(s.substr(b));
}

// remove a trailing "# comment" that is outside quotes
std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || std::isspace((unsigned char)s[i - 1]))) return rstrip(s.substr(0, i));
  }
  return rstrip(s);
}

Json scalar(const std::string& raw) {
  std::string s = strip(raw);
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Json();
  if (s.size() >= 2 && s.front() == '"' && s.back() == '"') {
    try {
      return Json::parse(s);  // JSON string escapes are a subset of YAML's
    } catch (...) {
      return Json(s.substr(1, s.size() - 2));
    }
  }
  if (s.size() >= 2 && s.front() == '\'' && s.back() == '\'') {
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') {
        out += '\'';
        ++i;
      } else {
        out += s[i];
      }
    }
    return Json(out);
  }
  if (s == "true" || s == "True" || s == "TRUE") return Json(true);
  if (s == "false" || s == "False" || s == "FALSE") return Json(false);
  bool intlike = !s.empty();
  for (size_t i = 0; i < s.size(); ++i) {
    if (!(std::isdigit((unsigned char)s[i]) || (i == 0 && (s[i] == '-' || s[i] == '+')))) intlike = false;
  }
  if (intlike && s != "-" && s != "+" && s.size() < 18) {
    if (!(s.size() > 1 && s[0] == '0')) return Json((int64_t)std::stoll(s));
  }
  bool floatlike = !s.empty() && s.find_first_not_of("0123456789.eE+-") == std::string::npos &&
                   s.find('.') != std::string::npos && s.find_first_of("0123456789") != std::string::npos;
  if (floatlike) {
    try {
      size_t used = 0;
      double d = std::stod(s, &used);
      if (used == s.size()) return Json(d);
    } catch (...) {
    }
  }
  return Json(s);
}

// flow collections: {a: b, c: [1, 2]}
class FlowParser {
 public:
  explicit FlowParser(const std::string& s) : s_(s) {}
  Json parse() {
    Json v = value();
    ws();
    if (i_ != s_.size()) throw YamlError("trailing characters in flow collection: " + s_);
    return v;
  }

 private:
  void ws() {
    while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) ++i_;
  }
  Json value() {
    ws();
    if (i_ >= s_.size()) return Json();
    if (s_[i_] == '{') return obj();
    if (s_[i_] == '[') return arr();
    return scalar(token(false));
  }
  std::string token(bool key) {
    ws();
    size_t st = i_;
    if (i_ < s_.size() && (s_[i_] == '"' || s_[i_] == '\'')) {
      char q = s_[i_++];
      while (i_ < s_.size() && !(s_[i_] == q && s_[i_ - 1] != '\\')) ++i_;
      ++i_;
      return s_.substr(st, i_ - st);
    }
    while (i_ < s_.size() && s_[i_] != ',' && s_[i_] != '}' && s_[i_] != ']' && !(key && s_[i_] == ':')) ++i_;
    return strip(s_.substr(st, i_ - st));
  }
  Json obj() {
    ++i_;
    Json o = Json::object();
    ws();
    if (i_ < s_.size() && s_[i_] == '}') {
      ++i_;
      return o;
    }
    while (i_ < s_.size()) {
      Json k = scalar(token(true));
      ws();
      Json v;
      if (i_ < s_.size() && s_[i_] == ':') {
        ++i_;
        v = value();
      }
      o[k.is_string() ? k.as_string() : k.dump()] = v;
      ws();
      if (i_ < s_.size() && s_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < s_.size() && s_[i_] == '}') {
        ++i_;
        return o;
      }
      break;
    }
    throw YamlError("bad flow mapping: " + s_);
  }
  Json arr() {
    ++i_;
    Json a = Json::array();
    ws();
    if (i_ < s_.size() && s_[i_] == ']') {
      ++i_;
      return a;
    }
    while (i_ < s_.size()) {
      a.push_back(value());
      ws();
      if (i_ < s_.size() && s_[i_] == ',') {
        ++i_;
        continue;
      }
      if (i_ < s_.size() && s_[i_] == ']') {
        ++i_;
        return a;
      }
      break;
    }
    throw YamlError("bad flow sequence: " + s_);
  }
  const std::string& s_;
  size_t i_ = 0;
};

Json value_of(const std::string& raw) {
  std::string s = strip(raw);
  if (!s.empty() && (s[0] == '{' || s[0] == '[')) return FlowParser(s).parse();
  return scalar(s);
}

// find "key: value" separator outside quotes; returns npos if not a mapping entry
size_t map_sep(const std::string& s) {
  bool sq = false, dq = false;
  int depth = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
    else if (!sq && !dq) {
      if (c == '{' || c == '[') ++depth;
      else if (c == '}' || c == ']') --depth;
      else if (c == ':' && depth == 0 && (i + 1 == s.size() || s[i + 1] == ' ' || s[i + 1] == '\t')) return i;
    }
  }
  return std::string::npos;
}

bool is_seq_item(const std::string& t) { return t == "-" || (t.size() >= 2 && t[0] == '-' && t[1] == ' '); }

class BlockParser {
 public:
  BlockParser(std::vector<Line> lines, std::vector<std::string> raw) : L_(std::move(lines)), raw_(std::move(raw)) {}

  Json parse() {
    if (L_.empty()) return Json();
    return block(L_[0].indent);
  }

 private:
  Json block(int indent) {
    if (pos_ >= L_.size()) return Json();
    if (is_seq_item(L_[pos_].text)) return seq(L_[pos_].indent);
    if (map_sep(L_[pos_].text) != std::string::npos) return map(L_[pos_].indent);
    // bare scalar (possibly multi-line plain scalar)
    std::string acc = L_[pos_++].text;
    while (pos_ < L_.size() && L_[pos_].indent >= indent && map_sep(L_[pos_].text) == std::string::npos &&
           !is_seq_item(L_[pos_].text))
      acc += " " + L_[pos_++].text;
    return value_of(acc);
  }

  Json nested_after_key(int ind) {
    if (pos_ >= L_.size()) return Json();
    const Line& nx = L_[pos_];
    if (nx.indent > ind) return block(nx.indent);
    if (nx.indent == ind && is_seq_item(nx.text)) return seq(ind);
    return Json();
  }

  std::string block_scalar(int ind, char style) {
    std::vector<std::string> parts;
    int content_indent = -1;
    while (pos_ < L_.size() && L_[pos_].indent > ind) {
      const Line& ln = L_[pos_];
      if (content_indent < 0) content_indent = ln.indent;
      // use the raw line so inner indentation / '#' survive
      std::string r = raw_[ln.lineno];
      parts.push_back(r.size() > (size_t)content_indent ? r.substr(content_indent) : strip(r));
      ++pos_;
    }
    std::string out;
    for (size_t i = 0; i < parts.size(); ++i) {
      out += parts[i];
      if (i + 1 < parts.size()) out += (style == '|') ? "\n" : " ";
    }
    if (!parts.empty()) out += "\n";
    return out;
  }

  Json map(int ind) {
    Json o = Json::object();
    while (pos_ < L_.size() && L_[pos_].indent == ind && !is_seq_item(L_[pos_].text)) {
      std::string t = L_[pos_].text;
      size_t sep = map_sep(t);
      if (sep == std::string::npos) throw YamlError("expected 'key: value' at line " + std::to_string(L_[pos_].lineno + 1));
      Json k = scalar(t.substr(0, sep));
      std::string key = k.is_string() ? k.as_string() : k.dump();
      std::string rest = strip(t.substr(sep + 1));
      ++pos_;
      if (rest.empty()) {
        o[key] = nested_after_key(ind);
      } else if (rest == "|" || rest == ">" || rest == "|-" || rest == ">-" || rest == "|+" || rest == ">+") {
        std::string s = block_scalar(ind, rest[0]);
        if (rest.size() > 1 && rest[1] == '-') {
          while (!s.empty() && s.back() == '\n') s.pop_back();
        }
        o[key] = Json(s);
      } else {
        o[key] = value_of(rest);
      }
    }
    return o;
  }

  Json seq(int ind) {
    Json a = Json::array();
    while (pos_ < L_.size() && L_[pos_].indent == ind && is_seq_item(L_[pos_].text)) {
      std::string t = L_[pos_].text;
      std::string rest = t.size() > 1 ? t.substr(2) : "";
      size_t lead = 0;
      while (lead < rest.size() && rest[lead] == ' ') ++lead;
      rest = rest.substr(lead);
      if (rest.empty()) {
        ++pos_;
        a.push_back(pos_ < L_.size() && L_[pos_].indent > ind ? block(L_[pos_].indent) : Json());
      } else if (is_seq_item(rest) || (map_sep(rest) != std::string::npos && rest[0] != '{' && rest[0] != '[')) {
        // compact nested collection: re-interpret this line at the item's column
        L_[pos_].indent = ind + 2 + (int)lead;
        L_[pos_].text = rest;
        a.push_back(block(L_[pos_].indent));
      } else {
        ++pos_;
        a.push_back(value_of(rest));
      }
    }
    return a;
  }

  std::vector<Line> L_;
  std::vector<std::string> raw_;
  size_t pos_ = 0;
};

std::vector<std::vector<std::string>> split_docs(const std::string& text) {
  std::vector<std::vector<std::string>> docs(1);
  std::istringstream in(text);
  std::string ln;
  while (std::getline(in, ln)) {
    if (!ln.empty() && ln.back() == '\r') ln.pop_back();
    if (ln.rfind("---", 0) == 0 && strip(ln.substr(3)).empty()) {
      if (!docs.back().empty()) docs.emplace_back();
      continue;
    }
    if (ln.rfind("...", 0) == 0 && strip(ln.substr(3)).empty()) continue;
    docs.back().push_back(ln);
  }
  return docs;
}

Json parse_doc(const std::vector<std::string>& raw) {
  std::vector<Line> lines;
  for (size_t i = 0; i < raw.size(); ++i) {
    const std::string& r = raw[i];
    int ind = 0;
    while (ind < (int)r.size() && r[ind] == ' ') ++ind;
    std::string t = strip_comment(r.substr(ind));
    if (t.empty()) continue;
    lines.push_back({ind, t, (int)i});
  }
  if (lines.size() == 1 && (lines[0].text[0] == '{' || lines[0].text[0] == '[')) return value_of(lines[0].text);
  return BlockParser(std::move(lines), raw).parse();
}

bool needs_quotes(const std::string& s) {
  if (s.empty()) return true;
  if (s == "true" || s == "false" || s == "null" || s == "~" || s == "yes" || s == "no") return true;
  if (std::isspace((unsigned char)s.front()) || std::isspace((unsigned char)s.back())) return true;
  if (s.find_first_of(":#{}[],&*!|>'\"%@`\n") != std::string::npos) return true;
  if (s[0] == '-' || s[0] == '?') return true;
  bool num = s.find_first_not_of("0123456789.eE+-") == std::string::npos;
  return num;
}

void dump_yaml(const Json& v, std::string& out, int indent, bool inline_first) {
  auto pad = [&](int n) { out.append((size_t)n, ' '); };
  switch (v.type()) {
    case Json::Type::Object: {
      if (v.size() == 0) {
        out += "{}\n";
        return;
      }
      bool first = true;
      for (auto& kv : v.as_object()) {
        if (!(first && inline_first)) pad(indent);
        first = false;
        out += needs_quotes(kv.first) ? Json(kv.first).dump() : kv.first;
        out += ":";
        const Json& c = kv.second;
        if ((c.is_object() || c.is_array()) && c.size() > 0) {
          out += "\n";
          dump_yaml(c, out, c.is_array() ? indent : indent + 2, false);
        } else {
          out += " ";
          dump_yaml(c, out, indent + 2, true);
        }
      }
      return;
    }
    case Json::Type::Array: {
      if (v.size() == 0) {
        out += "[]\n";
        return;
      }
      for (auto& e : v.as_array()) {
        pad(indent);
        out += "- ";
        if ((e.is_object() || e.is_array()) && e.size() > 0) {
          dump_yaml(e, out, indent + 2, true);
        } else {
          dump_yaml(e, out, indent + 2, true);
        }
      }
      return;
    }
    case Json::Type::String:
      out += needs_quotes(v.as_string()) ? v.dump() : v.as_string();
      out += "\n";
      return;
    default:
      out += v.dump();
      out += "\n";
  }
}

}  // namespace

Json yaml_parse(const std::string& text) {
  auto docs = split_docs(text);
  for (auto& d : docs) {
    Json j = parse_doc(d);
    if (!j.is_null()) return j;
  }
  return Json();
}

std::vector<Json> yaml_parse_all(const std::string& text) {
  std::vector<Json> out;
  for (auto& d : split_docs(text)) {
    Json j = parse_doc(d);
    if (!j.is_null()) out.push_back(j);
  }
  return out;
}

std::string yaml_dump(const Json& v) {
  std::string out;
  dump_yaml(v, out, 0, false);
  return out;
}

}  // namespace h2ok
