// Minimal JSON DOM for the KServe-v2 REST codec (no rapidjson / TritonJson on
// the box).  Objects keep insertion order so request bodies are emitted in
// the same field order as the reference (src/c++/library/http_client.cc:411-578).
// Parsing accepts NaN/Infinity like the reference's json_utils
// (src/c++/library/json_utils.cc:33-45).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace triton { namespace client { namespace json {

class Value {
 public:
  enum class Type { Null, Bool, Int, UInt, Double, String, Array, Object };

  Value() : type_(Type::Null) {}
  explicit Value(bool b) : type_(Type::Bool), b_(b) {}
  explicit Value(int v) : type_(Type::Int), i_(v) {}
  explicit Value(int64_t v) : type_(Type::Int), i_(v) {}
  explicit Value(uint64_t v) : type_(Type::UInt), u_(v) {}
  explicit Value(double v) : type_(Type::Double), d_(v) {}
  explicit Value(const char* s) : type_(Type::String), s_(s) {}
  explicit Value(const std::string& s) : type_(Type::String), s_(s) {}
  static Value Array() { Value v; v.type_ = Type::Array; return v; }
  static Value Object() { Value v; v.type_ = Type::Object; return v; }

  Type type() const { return type_; }
  bool IsNull() const { return type_ == Type::Null; }
  bool IsBool() const { return type_ == Type::Bool; }
  bool IsNumber() const { return type_ == Type::Int || type_ == Type::UInt || type_ == Type::Double; }
  bool IsInt() const { return type_ == Type::Int || type_ == Type::UInt; }
  bool IsString() const { return type_ == Type::String; }
  bool IsArray() const { return type_ == Type::Array; }
  bool IsObject() const { return type_ == Type::Object; }

  bool AsBool() const { return type_ == Type::Bool ? b_ : (IsNumber() ? AsDouble() != 0 : false); }
  int64_t AsInt() const
  {
    return type_ == Type::Int ? i_ : type_ == Type::UInt ? static_cast<int64_t>(u_)
           : type_ == Type::Double ? static_cast<int64_t>(d_) : type_ == Type::Bool ? (b_ ? 1 : 0) : 0;
  }
  uint64_t AsUInt() const
  {
    return type_ == Type::UInt ? u_ : type_ == Type::Int ? static_cast<uint64_t>(i_)
           : type_ == Type::Double ? static_cast<uint64_t>(d_) : 0;
  }
  double AsDouble() const
  {
    return type_ == Type::Double ? d_ : type_ == Type::Int ? static_cast<double>(i_)
           : type_ == Type::UInt ? static_cast<double>(u_) : 0.0;
  }
  const std::string& AsString() const { return s_; }

  // array
  size_t Size() const { return type_ == Type::Array ? arr_.size() : type_ == Type::Object ? obj_.size() : 0; }
  const Value& operator[](size_t i) const { return arr_[i]; }
  Value& operator[](size_t i) { return arr_[i]; }
  Value& Append(Value v) { arr_.push_back(std::move(v)); return arr_.back(); }
  const std::vector<Value>& Elements() const { return arr_; }

  // object
  const Value* Find(const std::string& key) const
  {
    for (const auto& kv : obj_)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
  Value* Find(const std::string& key)
  {
    for (auto& kv : obj_)
      if (kv.first == key) return &kv.second;
    return nullptr;
  }
  /// Set (or replace) key; returns the stored value.
  Value& Set(const std::string& key, Value v)
  {
    for (auto& kv : obj_)
      if (kv.first == key) { kv.second = std::move(v); return kv.second; }
    obj_.emplace_back(key, std::move(v));
    return obj_.back().second;
  }
  const std::vector<std::pair<std::string, Value>>& Members() const { return obj_; }

  std::string Serialize() const;
  void Write(std::string* out) const;

 private:
  Type type_;
  bool b_ = false;
  int64_t i_ = 0;
  uint64_t u_ = 0;
  double d_ = 0;
  std::string s_;
  std::vector<Value> arr_;
  std::vector<std::pair<std::string, Value>> obj_;
};

/// Parse `len` bytes; returns false and sets *err on malformed input.
bool Parse(const char* data, size_t len, Value* out, std::string* err);
inline bool Parse(const std::string& s, Value* out, std::string* err) { return Parse(s.data(), s.size(), out, err); }

void AppendEscapedString(std::string* out, const std::string& s);

}}}  // namespace triton::client::json
