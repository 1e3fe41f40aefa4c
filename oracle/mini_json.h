// mini_json.h — tiny JSON reader/writer used by the CPU oracle for its I/O.
//
// TEST INFRASTRUCTURE ONLY (see oracle/README.md).  Supports the subset the
// fixtures use: objects, arrays, strings (with \uXXXX escapes), integers
// (int64), booleans and null.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ojson {

struct Value {
  enum Kind { Null, Bool, Int, Str, Arr, Obj } kind = Null;
  bool b = false;
  int64_t i = 0;
  std::string s;
  std::vector<Value> a;
  std::vector<std::pair<std::string, Value>> o;  // insertion order kept

  bool is_null() const { return kind == Null; }
  const Value* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Value& at(const std::string& k) const {
    static Value null_v;
    const Value* v = get(k);
    return v ? *v : null_v;
  }
  int64_t as_int(int64_t def = 0) const { return kind == Int ? i : (kind == Bool ? (b ? 1 : 0) : def); }
  std::string as_str(const std::string& def = "") const { return kind == Str ? s : def; }
  bool as_bool(bool def = false) const { return kind == Bool ? b : def; }
};

class Parser {
 public:
  explicit Parser(const char* p) : p_(p) {}
  Value parse() {
    Value v = value();
    ws();
    if (*p_) throw std::runtime_error("trailing characters in JSON");
    return v;
  }

 private:
  const char* p_;
  void ws() {
    while (*p_ == ' ' || *p_ == '\n' || *p_ == '\t' || *p_ == '\r') ++p_;
  }
  Value value() {
    ws();
    Value v;
    char c = *p_;
    if (c == '{') {
      ++p_;
      v.kind = Value::Obj;
      ws();
      if (*p_ == '}') { ++p_; return v; }
      for (;;) {
        ws();
        std::string k = str();
        ws();
        if (*p_++ != ':') throw std::runtime_error("expected ':'");
        v.o.emplace_back(std::move(k), value());
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == '}') { ++p_; return v; }
        throw std::runtime_error("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p_;
      v.kind = Value::Arr;
      ws();
      if (*p_ == ']') { ++p_; return v; }
      for (;;) {
        v.a.push_back(value());
        ws();
        if (*p_ == ',') { ++p_; continue; }
        if (*p_ == ']') { ++p_; return v; }
        throw std::runtime_error("expected ',' or ']'");
      }
    }
    if (c == '"') { v.kind = Value::Str; v.s = str(); return v; }
    if (c == 't' && std::string(p_, 4) == "true") { p_ += 4; v.kind = Value::Bool; v.b = true; return v; }
    if (c == 'f' && std::string(p_, 5) == "false") { p_ += 5; v.kind = Value::Bool; v.b = false; return v; }
    if (c == 'n' && std::string(p_, 4) == "null") { p_ += 4; return v; }
    if (c == '-' || (c >= '0' && c <= '9')) {
      bool neg = false;
      if (*p_ == '-') { neg = true; ++p_; }
      uint64_t u = 0;
      while (*p_ >= '0' && *p_ <= '9') u = u * 10 + uint64_t(*p_++ - '0');
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') throw std::runtime_error("non-integer number");
      v.kind = Value::Int;
      v.i = neg ? int64_t(0 - u) : int64_t(u);
      return v;
    }
    throw std::runtime_error(std::string("bad JSON at: ") + std::string(p_, 20));
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += char(cp);
    else if (cp < 0x800) { out += char(0xC0 | (cp >> 6)); out += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { out += char(0xE0 | (cp >> 12)); out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F)); }
    else { out += char(0xF0 | (cp >> 18)); out += char(0x80 | ((cp >> 12) & 0x3F)); out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F)); }
  }
  std::string str() {
    if (*p_++ != '"') throw std::runtime_error("expected string");
    std::string out;
    while (*p_ && *p_ != '"') {
      if (*p_ == '\\') {
        ++p_;
        char e = *p_++;
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            uint32_t cp = std::stoul(std::string(p_, 4), nullptr, 16);
            p_ += 4;
            if (cp >= 0xD800 && cp < 0xDC00 && p_[0] == '\\' && p_[1] == 'u') {
              uint32_t lo = std::stoul(std::string(p_ + 2, 4), nullptr, 16);
              p_ += 6;
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(out, cp);
            break;
          }
          default: out += e;
        }
      } else {
        out += *p_++;
      }
    }
    if (*p_++ != '"') throw std::runtime_error("unterminated string");
    return out;
  }
};

inline Value parse(const char* s) { return Parser(s).parse(); }

inline void quote(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\t': out += "\\t"; break;
      case '\r': out += "\\r"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += char(c);
        }
    }
  }
  out += '"';
}

}  // namespace ojson
