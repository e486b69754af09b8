#include "json.hpp"

#include <cstdio>
#include <cstring>
#include <sstream>

namespace h2ok {

namespace {

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}

  Json parse_document() {
    skip_ws();
    Json v = parse_value(0);
    skip_ws();
    if (i_ != s_.size()) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const std::string& msg) {
    throw JsonError("JSON parse error at offset " + std::to_string(i_) + ": " + msg);
  }
  void skip_ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
  }
  char peek() {
    if (i_ >= s_.size()) fail("unexpected end");
    return s_[i_];
  }
  void expect(char c) {
    if (peek() != c) fail(std::string("expected '") + c + "'");
    ++i_;
  }
  Json parse_value(int depth) {
    if (depth > 256) fail("nesting too deep");
    skip_ws();
    char c = peek();
    if (c == '{') return parse_object(depth);
    if (c == '[') return parse_array(depth);
    if (c == '"') return Json(parse_string());
    if (c == 't') return literal("true", Json(true));
    if (c == 'f') return literal("false", Json(false));
    if (c == 'n') return literal("null", Json());
    return parse_number();
  }
  Json literal(const char* w, Json v) {
    size_t n = std::strlen(w);
    if (s_.compare(i_, n, w) != 0) fail("bad literal");
    i_ += n;
    return v;
  }
  Json parse_number() {
    size_t st = i_;
    bool is_float = false;
    if (i_ < s_.size() && (s_[i_] == '-' || s_[i_] == '+')) ++i_;
    while (i_ < s_.size()) {
      char c = s_[i_];
      if (c >= '0' && c <= '9') {
        ++i_;
      } else if (c == '.' || c == 'e' || c == 'E' || c == '-' || c == '+') {
        is_float = true;
        ++i_;
      } else {
        break;
      }
    }
    if (st == i_) fail("bad value");
    std::string tok = s_.substr(st, i_ - st);
    try {
      if (!is_float) return Json((int64_t)std::stoll(tok));
      return Json(std::stod(tok));
    } catch (...) {
      fail("bad number '" + tok + "'");
    }
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i_ + 4 > s_.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string parse_string() {
    expect('"');
    std::string out;
    while (true) {
      if (i_ >= s_.size()) fail("unterminated string");
      char c = s_[i_++];
      if (c == '"') break;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (i_ >= s_.size()) fail("bad escape");
      char e = s_[i_++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
            i_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Json parse_array(int depth) {
    expect('[');
    JsonArray a;
    skip_ws();
    if (peek() == ']') {
      ++i_;
      return Json(std::move(a));
    }
    while (true) {
      a.push_back(parse_value(depth + 1));
      skip_ws();
      char c = peek();
      ++i_;
      if (c == ']') break;
      if (c != ',') fail("expected ',' or ']'");
    }
    return Json(std::move(a));
  }
  Json parse_object(int depth) {
    expect('{');
    JsonObject o;
    skip_ws();
    if (peek() == '}') {
      ++i_;
      return Json(std::move(o));
    }
    while (true) {
      skip_ws();
      std::string k = parse_string();
      skip_ws();
      expect(':');
      Json v = parse_value(depth + 1);
      bool replaced = false;
      for (auto& kv : o)
        if (kv.first == k) {
          kv.second = v;
          replaced = true;
        }
      if (!replaced) o.emplace_back(std::move(k), std::move(v));
      skip_ws();
      char c = peek();
      ++i_;
      if (c == '}') break;
      if (c != ',') fail("expected ',' or '}'");
    }
    return Json(std::move(o));
  }

  const std::string& s_;
  size_t i_ = 0;
};

}  // namespace

Json Json::parse(const std::string& text) { return Parser(text).parse_document(); }

const Json* Json::path(const std::string& dotted) const {
  const Json* cur = this;
  size_t st = 0;
  while (cur && st <= dotted.size()) {
    size_t dot = dotted.find('.', st);
    std::string key = dotted.substr(st, dot == std::string::npos ? std::string::npos : dot - st);
    if (cur->is_array()) {
      try {
        size_t idx = std::stoul(key);
        if (idx >= cur->size()) return nullptr;
        cur = &(*cur->arr_)[idx];
      } catch (...) {
        return nullptr;
      }
    } else {
      cur = cur->find(key);
    }
    if (dot == std::string::npos) break;
    st = dot + 1;
  }
  return cur;
}

Json Json::deep_copy() const {
  switch (type_) {
    case Type::Array: {
      JsonArray a;
      for (auto& v : *arr_) a.push_back(v.deep_copy());
      return Json(std::move(a));
    }
    case Type::Object: {
      JsonObject o;
      for (auto& kv : *obj_) o.emplace_back(kv.first, kv.second.deep_copy());
      return Json(std::move(o));
    }
    default:
      return *this;
  }
}

bool Json::operator==(const Json& o) const {
  if (type_ != o.type_) return false;
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::Number: return num_ == o.num_;
    case Type::String: return str_ == o.str_;
    case Type::Array: return *arr_ == *o.arr_;
    case Type::Object: {
      if (obj_->size() != o.obj_->size()) return false;
      for (auto& kv : *obj_) {
        const Json* v = o.find(kv.first);
        if (!v || !(*v == kv.second)) return false;
      }
      return true;
    }
  }
  return false;
}

std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  return out;
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent <= 0) return;
    out += '\n';
    out.append((size_t)(indent * d), ' ');
  };
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Number: {
      if (is_int_) {
        out += std::to_string(int_);
      } else if (std::isfinite(num_) && num_ == std::floor(num_) && std::fabs(num_) < 1e15) {
        char buf[64];
        std::snprintf(buf, sizeof buf, "%.1f", num_);
        out += buf;
      } else if (std::isfinite(num_)) {
        char buf[64];
        std::snprintf(buf, sizeof buf, "%.17g", num_);
        out += buf;
      } else {
        out += "null";
      }
      break;
    }
    case Type::String:
      out += '"';
      out += json_escape(str_);
      out += '"';
      break;
    case Type::Array: {
      out += '[';
      bool first = true;
      for (auto& v : *arr_) {
        if (!first) out += ',';
        first = false;
        nl(depth + 1);
        v.dump_to(out, indent, depth + 1);
      }
      if (!arr_->empty()) nl(depth);
      out += ']';
      break;
    }
    case Type::Object: {
      out += '{';
      bool first = true;
      for (auto& kv : *obj_) {
        if (!first) out += ',';
        first = false;
        nl(depth + 1);
        out += '"';
        out += json_escape(kv.first);
        out += indent > 0 ? "\": " : "\":";
        kv.second.dump_to(out, indent, depth + 1);
      }
      if (!obj_->empty()) nl(depth);
      out += '}';
      break;
    }
  }
}

std::string Json::dump() const {
  std::string out;
  dump_to(out, 0, 0);
  return out;
}

std::string Json::dump_pretty(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

}  // namespace h2ok
