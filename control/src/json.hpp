// Minimal ordered JSON value, parser and compact serializer for the h2ok
// control plane (descriptor files, Kubernetes API bodies, watch events).
//
// Objects keep insertion order so the descriptor layout matches the
// reference's serde_json output field order (src/k8s/mod.rs:41-74 of
// isgasho/h2o-kubernetes): specification, ingresses, stateful_sets, services.
#pragma once

#include <cmath>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace h2ok {

class Json;
using JsonObject = std::vector<std::pair<std::string, Json>>;
using JsonArray = std::vector<Json>;

class JsonError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Json {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };

  Json() : type_(Type::Null) {}
  Json(std::nullptr_t) : type_(Type::Null) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Number), num_(v), is_int_(true), int_(v) {}
  Json(int64_t v) : type_(Type::Number), num_((double)v), is_int_(true), int_(v) {}
  Json(uint32_t v) : type_(Type::Number), num_(v), is_int_(true), int_(v) {}
  Json(double v) : type_(Type::Number), num_(v), is_int_(false), int_((int64_t)v) {}
  Json(const char* s) : type_(Type::String), str_(s) {}
  Json(std::string s) : type_(Type::String), str_(std::move(s)) {}
  Json(JsonArray a) : type_(Type::Array), arr_(std::make_shared<JsonArray>(std::move(a))) {}
  Json(JsonObject o) : type_(Type::Object), obj_(std::make_shared<JsonObject>(std::move(o))) {}

  static Json object() { return Json(JsonObject{}); }
  static Json array() { return Json(JsonArray{}); }
  static Json parse(const std::string& text);

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Number; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const {
    if (!is_bool()) throw JsonError("not a bool");
    return b_;
  }
  double as_double() const {
    if (!is_number()) throw JsonError("not a number");
    return num_;
  }
  int64_t as_int() const {
    if (!is_number()) throw JsonError("not a number");
    return is_int_ ? int_ : (int64_t)num_;
  }
  const std::string& as_string() const {
    if (!is_string()) throw JsonError("not a string");
    return str_;
  }
  JsonArray& as_array() {
    if (!is_array()) throw JsonError("not an array");
    return *arr_;
  }
  const JsonArray& as_array() const {
    if (!is_array()) throw JsonError("not an array");
    return *arr_;
  }
  JsonObject& as_object() {
    if (!is_object()) throw JsonError("not an object");
    return *obj_;
  }
  const JsonObject& as_object() const {
    if (!is_object()) throw JsonError("not an object");
    return *obj_;
  }

  // object access
  bool has(const std::string& k) const {
    if (!is_object()) return false;
    for (auto& kv : *obj_)
      if (kv.first == k) return true;
    return false;
  }
  const Json* find(const std::string& k) const {
    if (!is_object()) return nullptr;
    for (auto& kv : *obj_)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  Json* find(const std::string& k) {
    if (!is_object()) return nullptr;
    for (auto& kv : *obj_)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  Json& operator[](const std::string& k) {
    if (is_null()) *this = object();
    for (auto& kv : as_object())
      if (kv.first == k) return kv.second;
    obj_->emplace_back(k, Json());
    return obj_->back().second;
  }
  const Json& at(const std::string& k) const {
    const Json* v = find(k);
    if (!v) throw JsonError("missing key: " + k);
    return *v;
  }
  // path lookup "a.b.c"; returns nullptr when any hop is missing
  const Json* path(const std::string& dotted) const;
  std::string get_string(const std::string& dotted, const std::string& dflt = "") const {
    const Json* v = path(dotted);
    return (v && v->is_string()) ? v->as_string() : dflt;
  }
  int64_t get_int(const std::string& dotted, int64_t dflt = 0) const {
    const Json* v = path(dotted);
    if (!v) return dflt;
    if (v->is_number()) return v->as_int();
    if (v->is_string()) {
      try {
        return std::stoll(v->as_string());
      } catch (...) {
        return dflt;
      }
    }
    return dflt;
  }
  void erase(const std::string& k) {
    if (!is_object()) return;
    auto& o = *obj_;
    for (auto it = o.begin(); it != o.end(); ++it)
      if (it->first == k) {
        o.erase(it);
        return;
      }
  }

  // array access
  void push_back(Json v) {
    if (is_null()) *this = array();
    as_array().push_back(std::move(v));
  }
  size_t size() const {
    if (is_array()) return arr_->size();
    if (is_object()) return obj_->size();
    return 0;
  }
  Json& operator[](size_t i) { return as_array().at(i); }
  const Json& operator[](size_t i) const { return as_array().at(i); }

  Json deep_copy() const;
  std::string dump() const;  // compact
  std::string dump_pretty(int indent = 2) const;
  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  void dump_to(std::string& out, int indent, int depth) const;
  Type type_;
  bool b_ = false;
  double num_ = 0;
  bool is_int_ = false;
  int64_t int_ = 0;
  std::string str_;
  std::shared_ptr<JsonArray> arr_;
  std::shared_ptr<JsonObject> obj_;
};

std::string json_escape(const std::string& s);

}  // namespace h2ok
