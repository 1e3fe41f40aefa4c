// json_reader.h — minimal JSON DOM for the host layer's JSON entry points
// (objects, arrays, strings, int64, bool, null).
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace kjson {

struct Node {
  enum Type { kNull, kBool, kInt, kString, kArray, kObject };
  Type type = kNull;
  bool boolean = false;
  int64_t integer = 0;
  std::string str;
  std::vector<Node> items;
  std::vector<std::pair<std::string, Node>> fields;

  const Node* find(const char* key) const {
    if (type != kObject) return nullptr;
    for (const auto& f : fields)
      if (f.first == key) return &f.second;
    return nullptr;
  }
  const Node& operator[](const char* key) const {
    static const Node kNullNode;
    const Node* n = find(key);
    return n ? *n : kNullNode;
  }
  bool null() const { return type == kNull; }
  int64_t i64(int64_t def = 0) const { return type == kInt ? integer : def; }
  bool b(bool def = false) const { return type == kBool ? boolean : def; }
  const std::string& s() const {
    static const std::string kEmpty;
    return type == kString ? str : kEmpty;
  }
};

class Reader {
 public:
  explicit Reader(const char* text) : p_(text) {}
  Node read() {
    Node n = value();
    skip();
    if (*p_) throw std::runtime_error("json: trailing data");
    return n;
  }

 private:
  const char* p_;
  void skip() {
    while (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r') ++p_;
  }
  bool lit(const char* w) {
    size_t n = 0;
    while (w[n]) n++;
    for (size_t i = 0; i < n; i++)
      if (p_[i] != w[i]) return false;
    p_ += n;
    return true;
  }
  static void utf8(std::string& o, uint32_t c) {
    if (c < 0x80) {
      o += char(c);
    } else if (c < 0x800) {
      o += char(0xC0 | (c >> 6));
      o += char(0x80 | (c & 63));
    } else if (c < 0x10000) {
      o += char(0xE0 | (c >> 12));
      o += char(0x80 | ((c >> 6) & 63));
      o += char(0x80 | (c & 63));
    } else {
      o += char(0xF0 | (c >> 18));
      o += char(0x80 | ((c >> 12) & 63));
      o += char(0x80 | ((c >> 6) & 63));
      o += char(0x80 | (c & 63));
    }
  }
  uint32_t hex4() {
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
      char ch = *p_++;
      v <<= 4;
      if (ch >= '0' && ch <= '9') v |= uint32_t(ch - '0');
      else if (ch >= 'a' && ch <= 'f') v |= uint32_t(ch - 'a' + 10);
      else if (ch >= 'A' && ch <= 'F') v |= uint32_t(ch - 'A' + 10);
      else throw std::runtime_error("json: bad \\u escape");
    }
    return v;
  }
  std::string string() {
    if (*p_ != '"') throw std::runtime_error("json: expected string");
    ++p_;
    std::string o;
    for (;;) {
      char ch = *p_++;
      if (ch == '\0') throw std::runtime_error("json: unterminated string");
      if (ch == '"') break;
      if (ch != '\\') {
        o += ch;
        continue;
      }
      char e = *p_++;
      switch (e) {
        case 'n': o += '\n'; break;
        case 't': o += '\t'; break;
        case 'r': o += '\r'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'u': {
          uint32_t c = hex4();
          if (c >= 0xD800 && c < 0xDC00 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            c = 0x10000 + ((c - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(o, c);
          break;
        }
        default: o += e;
      }
    }
    return o;
  }
  Node value() {
    skip();
    Node n;
    if (*p_ == '{') {
      ++p_;
      n.type = Node::kObject;
      skip();
      if (*p_ == '}') {
        ++p_;
        return n;
      }
      for (;;) {
        skip();
        std::string k = string();
        skip();
        if (*p_++ != ':') throw std::runtime_error("json: expected ':'");
        n.fields.emplace_back(std::move(k), value());
        skip();
        char ch = *p_++;
        if (ch == ',') continue;
        if (ch == '}') return n;
        throw std::runtime_error("json: expected ',' or '}'");
      }
    }
    if (*p_ == '[') {
      ++p_;
      n.type = Node::kArray;
      skip();
      if (*p_ == ']') {
        ++p_;
        return n;
      }
      for (;;) {
        n.items.push_back(value());
        skip();
        char ch = *p_++;
        if (ch == ',') continue;
        if (ch == ']') return n;
        throw std::runtime_error("json: expected ',' or ']'");
      }
    }
    if (*p_ == '"') {
      n.type = Node::kString;
      n.str = string();
      return n;
    }
    if (lit("true")) {
      n.type = Node::kBool;
      n.boolean = true;
      return n;
    }
    if (lit("false")) {
      n.type = Node::kBool;
      return n;
    }
    if (lit("null")) return n;
    if (*p_ == '-' || (*p_ >= '0' && *p_ <= '9')) {
      bool neg = *p_ == '-';
      if (neg) ++p_;
      uint64_t u = 0;
      while (*p_ >= '0' && *p_ <= '9') u = u * 10 + uint64_t(*p_++ - '0');
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') throw std::runtime_error("json: non-integer number");
      n.type = Node::kInt;
      n.integer = neg ? int64_t(0 - u) : int64_t(u);
      return n;
    }
    throw std::runtime_error("json: unexpected character");
  }
};

inline Node parse(const char* text) { return Reader(text).read(); }

inline void write_string(std::string& out, std::string_view s) {
  out += '"';
  size_t run = 0;  // start of the pending run of characters that need no escape
  for (size_t i = 0; i < s.size(); i++) {
    const unsigned char ch = static_cast<unsigned char>(s[i]);
    if (ch >= 0x20 && ch != '"' && ch != '\\') continue;
    out.append(s.data() + run, i - run);
    run = i + 1;
    if (ch == '"') out += "\\\"";
    else if (ch == '\\') out += "\\\\";
    else if (ch == '\n') out += "\\n";
    else if (ch == '\t') out += "\\t";
    else if (ch == '\r') out += "\\r";
    else {
      char buf[8];
      snprintf(buf, sizeof buf, "\\u%04x", ch);
      out += buf;
    }
  }
  out.append(s.data() + run, s.size() - run);
  out += '"';
}

}  // namespace kjson
