// json.h — small JSON DOM for the scene / camera / settings files (the reference uses
// nlohmann::json, Serialize.cpp; that library is not part of this image). Objects keep key order
// of the file; lookups follow nlohmann's value(key, default) rules used by the loader.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace rt2 {

class Json {
 public:
  enum class Type { kNull, kBool, kNumber, kString, kArray, kObject };

  Json() = default;
  static Json number(double v) {
    Json j;
    j.type_ = Type::kNumber;
    j.num_ = v;
    return j;
  }
  static Json string(std::string s) {
    Json j;
    j.type_ = Type::kString;
    j.str_ = std::move(s);
    return j;
  }
  static Json array() {
    Json j;
    j.type_ = Type::kArray;
    return j;
  }
  static Json object() {
    Json j;
    j.type_ = Type::kObject;
    return j;
  }

  // Parses `text`; on failure returns false and sets `err` to "line L col C: message".
  static bool Parse(const std::string& text, Json& out, std::string& err);
  // Reads and parses a file; a missing file is an error (the reference returns null json and
  // throws later, Util.cpp:21-32).
  static bool ParseFile(const std::string& path, Json& out, std::string& err);

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::kNull; }
  bool is_number() const { return type_ == Type::kNumber; }
  bool is_string() const { return type_ == Type::kString; }
  bool is_array() const { return type_ == Type::kArray; }
  bool is_object() const { return type_ == Type::kObject; }
  bool is_bool() const { return type_ == Type::kBool; }

  double as_number() const { return type_ == Type::kBool ? (bool_ ? 1.0 : 0.0) : num_; }
  bool as_bool() const { return type_ == Type::kBool ? bool_ : num_ != 0.0; }
  const std::string& as_string() const { return str_; }
  const std::vector<Json>& items() const { return arr_; }
  const std::vector<std::pair<std::string, Json>>& members() const { return obj_; }

  const Json* find(const std::string& key) const;
  bool contains(const std::string& key) const { return find(key) != nullptr; }

  void push_back(Json v) { arr_.push_back(std::move(v)); }
  void set(const std::string& key, Json v);

  // nlohmann-style dump(indent) with keys sorted (nlohmann::json is std::map based) and floats
  // printed as the shortest round-trip decimal of the double, "x.0" for integral values.
  std::string Dump(int indent) const;

 private:
  void DumpTo(std::string& out, int indent, int level) const;
  Type type_ = Type::kNull;
  double num_ = 0;
  bool bool_ = false;
  bool integral_ = false;  // number written without fraction/exponent in the source
  std::string str_;
  std::vector<Json> arr_;
  std::vector<std::pair<std::string, Json>> obj_;
  friend class JsonParser;

 public:
  static Json integer(int64_t v) {
    Json j = number((double)v);
    j.integral_ = true;
    return j;
  }
  static Json boolean(bool b) {
    Json j;
    j.type_ = Type::kBool;
    j.bool_ = b;
    return j;
  }
};

}  // namespace rt2
