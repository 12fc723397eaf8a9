// Minimal JSON value, parser and serializer for the kgwe control-plane core.
//
// Used for the amd-smi fixture HAL, topology snapshots, the scheduler-extender
// wire format (ExtenderArgs / ExtenderFilterResult / HostPriorityList /
// ExtenderBindingArgs) and cost-journal records, so the hot scheduling path
// never round-trips through Python objects.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace kgwe {

class Json {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::map<std::string, Json>;

  Json() : type_(Type::Null) {}
  Json(std::nullptr_t) : type_(Type::Null) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Number), n_(v) {}
  Json(int64_t v) : type_(Type::Number), n_(static_cast<double>(v)) {}
  Json(uint64_t v) : type_(Type::Number), n_(static_cast<double>(v)) {}
  Json(double v) : type_(Type::Number), n_(v) {}
  Json(const char* s) : type_(Type::String), s_(std::make_shared<std::string>(s)) {}
  Json(std::string s) : type_(Type::String), s_(std::make_shared<std::string>(std::move(s))) {}
  Json(Array a) : type_(Type::Array), a_(std::make_shared<Array>(std::move(a))) {}
  Json(Object o) : type_(Type::Object), o_(std::make_shared<Object>(std::move(o))) {}

  static Json array() { return Json(Array{}); }
  static Json object() { return Json(Object{}); }
  static Json parse(const std::string& text);

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Number; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool(bool dflt = false) const { return is_bool() ? b_ : dflt; }
  double as_number(double dflt = 0.0) const { return is_number() ? n_ : dflt; }
  int64_t as_int(int64_t dflt = 0) const {
    return is_number() ? static_cast<int64_t>(n_) : dflt;
  }
  const std::string& as_string() const;
  std::string str(const std::string& dflt = "") const { return is_string() ? *s_ : dflt; }

  const Array& items() const;
  Array& items();
  const Object& fields() const;
  Object& fields();

  // Object access: get() returns a shared null for a missing key.
  const Json& get(const std::string& key) const;
  bool has(const std::string& key) const;
  Json& operator[](const std::string& key);  // creates (converts null to object)
  const Json& at(size_t i) const { return items().at(i); }
  size_t size() const;
  void push_back(Json v);

  std::string dump() const;
  void dump_to(std::string& out) const;

 private:
  void own();  // copy-on-write before mutation
  Type type_;
  bool b_ = false;
  double n_ = 0.0;
  std::shared_ptr<std::string> s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
};

std::string json_escape(const std::string& s);

}  // namespace kgwe
