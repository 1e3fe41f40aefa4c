// label_selectors.h — host-side validation and failure text for the two
// label predicates findTopologyAssignment builds before fillInCounts
// (reference /root/reference/pkg/cache/scheduler/tas_flavor_snapshot.go):
//
//   nodeSelector  labels.ValidatedSelectorFromSet            :879-887
//                 -> "invalid node selectors: %s, reason: %s"
//   affinity      nodeaffinity.NewNodeSelector(required...)  :889-897
//                 -> "invalid affinity node selectors: %s, reason: %s"
//
// The text follows the vendored helpers: labels.NewRequirement
// (vendor/k8s.io/apimachinery/pkg/labels/selector.go:185-225),
// content.IsLabelKey / IsLabelValue / IsDNS1123Subdomain
// (vendor/.../api/validate/content/kube.go:43-94, dns.go:64-101), field.Error
// and field.Path rendering (vendor/.../util/validation/field/errors.go:63-117,
// path.go:92-117), ErrorList.ToAggregate and aggregate.Error with Flatten
// (field/errors.go:353-368, util/errors/errors.go:70-96, :182-200),
// nodeSelectorRequirementsAsSelector / AsFieldSelector
// (vendor/k8s.io/component-helpers/scheduling/corev1/nodeaffinity/
// nodeaffinity.go:214-293) and (*v1.NodeSelector).String
// (vendor/k8s.io/api/core/v1/generated.pb.go:22060-22107).
//
// Matching itself is not done here: the host compiles affinity to per-column
// value-id sets that the fill kernels test (tas_host.cpp compile_affinity).
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <string_view>
#include <vector>

namespace kueue_tas {
namespace labelsel {

struct Expr {  // v1.NodeSelectorRequirement
  std::string key, op;
  std::optional<std::vector<std::string>> values;  // nullopt: JSON null / absent (Go nil slice)
};
struct Term {  // v1.NodeSelectorTerm
  std::vector<Expr> exprs, fields;
  bool empty() const { return exprs.empty() && fields.empty(); }  // isEmptyNodeSelectorTerm
};
using RequiredAffinity = std::vector<Term>;  // v1.NodeSelector.NodeSelectorTerms

// strconv.Quote (ASCII escapes; well-formed multi-byte UTF-8 kept)
inline std::string quote(const std::string& s) {
  std::string o = "\"";
  for (size_t i = 0; i < s.size(); i++) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    switch (c) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\a': o += "\\a"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\v': o += "\\v"; continue;
      default: break;
    }
    if (c >= 0x20 && c < 0x7f) {
      o += char(c);
      continue;
    }
    const int n = c >= 0xf0 && c < 0xf8 ? 4 : c >= 0xe0 ? (c < 0xf0 ? 3 : 0) : c >= 0xc0 ? 2 : 0;
    bool good = n > 0 && i + size_t(n) <= s.size();
    for (int k = 1; good && k < n; k++) good = (static_cast<unsigned char>(s[i + size_t(k)]) & 0xc0) == 0x80;
    if (good) {
      o.append(s, i, size_t(n));
      i += size_t(n) - 1;
    } else {
      char b[8];
      snprintf(b, sizeof b, "\\x%02x", c);
      o += b;
    }
  }
  return o + "\"";
}

// encoding/json string escaping (HTML-safe, as json.Marshal does)
inline void json_escape(std::string& o, const std::string& s) {
  o += '"';
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += char(c);
    } else if (c == '\n') o += "\\n";
    else if (c == '\r') o += "\\r";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else o += char(c);
  }
  o += '"';
}
inline std::string json_list(const std::optional<std::vector<std::string>>& v) {
  if (!v) return "null";
  std::string o = "[";
  for (size_t i = 0; i < v->size(); i++) {
    if (i) o += ',';
    json_escape(o, (*v)[i]);
  }
  return o + "]";
}

// strconv.ParseInt(s, 10, 64)
inline bool parse_int(const std::string& s, int64_t* out) {
  size_t i = (!s.empty() && (s[0] == '+' || s[0] == '-')) ? 1 : 0;
  if (i == s.size()) return false;
  const bool neg = i && s[0] == '-';
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + unsigned(s[i] - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v == ((unsigned __int128)1 << 63)) return false;
  if (out) *out = neg ? int64_t(0 - uint64_t(v)) : int64_t(uint64_t(v));
  return true;
}

// ---- content validators ------------------------------------------------------
inline std::string regex_msg(std::string msg, const char* re, std::initializer_list<const char*> ex) {
  msg += " (e.g. ";
  bool first = true;
  for (const char* e : ex) {
    if (!first) msg += " or ";
    first = false;
    msg += std::string("'") + e + "', ";
  }
  return msg + "regex used for validation is '" + re + "')";
}
inline bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
// ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]
inline bool qualified_name_ok(std::string_view s) {
  if (s.empty() || !alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}
// [a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*
inline bool dns_subdomain_ok(std::string_view s) {
  auto lc = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
  size_t b = 0;
  for (;;) {
    const size_t e = s.find('.', b);
    const size_t len = (e == std::string_view::npos ? s.size() : e) - b;
    if (len == 0 || !lc(s[b]) || !lc(s[b + len - 1])) return false;
    for (size_t k = b; k < b + len; k++)
      if (!lc(s[k]) && s[k] != '-') return false;
    if (e == std::string_view::npos) return true;
    b = e + 1;
  }
}
constexpr const char* kKeyMsg =
    "must consist of alphanumeric characters, '-', '_' or '.', and must start and end with an alphanumeric character";
constexpr const char* kKeyRe = "([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]";

// content.IsLabelKey, messages joined with "; " ("" when valid)
inline std::string label_key_problems(const std::string& k) {
  std::vector<std::string> errs;
  const size_t slash = k.find('/');
  std::string name = k;
  if (slash != std::string::npos) {
    if (k.find('/', slash + 1) != std::string::npos)
      return "a valid label key " + regex_msg(kKeyMsg, kKeyRe, {"MyName", "my.name", "123-abc"}) +
             " with an optional DNS subdomain prefix and '/' (e.g. 'example.com/MyName')";
    const std::string prefix = k.substr(0, slash);
    name = k.substr(slash + 1);
    if (prefix.empty()) {
      errs.push_back("prefix part must be non-empty");
    } else {
      if (prefix.size() > 253) errs.push_back("prefix part must be no more than 253 bytes");
      if (!dns_subdomain_ok(prefix))
        errs.push_back("prefix part " + regex_msg("a lowercase RFC 1123 subdomain must consist of lower case "
                                                  "alphanumeric characters, '-' or '.', and must start and end with an "
                                                  "alphanumeric character",
                                                  "[a-z0-9]([-a-z0-9]*[a-z0-9])?(\\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*",
                                                  {"example.com"}));
    }
  }
  if (name.empty()) errs.push_back("name part must be non-empty");
  else if (name.size() > 63) errs.push_back("name part must be no more than 63 bytes");
  if (!qualified_name_ok(name)) errs.push_back("name part " + regex_msg(kKeyMsg, kKeyRe, {"MyName", "my.name", "123-abc"}));
  std::string o;
  for (size_t i = 0; i < errs.size(); i++) o += (i ? "; " : "") + errs[i];
  return o;
}
// content.IsLabelValue ("" when valid)
inline std::string label_value_problems(const std::string& v) {
  std::string o;
  if (v.size() > 63) o = "must be no more than 63 bytes";
  if (!v.empty() && !qualified_name_ok(v)) {
    if (!o.empty()) o += "; ";
    o += regex_msg("a valid label must be an empty string or consist of alphanumeric characters, '-', '_' or '.', and "
                   "must start and end with an alphanumeric character",
                   "(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?", {"MyValue", "my_value", "12345"});
  }
  return o;
}

// Allocation-free equivalents of label_key_problems(k).empty() and
// label_value_problems(v).empty(): the common (valid) case of every compile.
inline bool label_key_ok(std::string_view k) {
  std::string_view name = k;
  const size_t slash = k.find('/');
  if (slash != std::string_view::npos) {
    if (k.find('/', slash + 1) != std::string_view::npos) return false;
    const std::string_view prefix = k.substr(0, slash);
    if (prefix.empty() || prefix.size() > 253 || !dns_subdomain_ok(prefix)) return false;
    name = k.substr(slash + 1);
  }
  return !name.empty() && name.size() <= 63 && qualified_name_ok(name);
}
inline bool label_value_ok(std::string_view v) { return v.size() <= 63 && (v.empty() || qualified_name_ok(v)); }
// labels.NewRequirement succeeds (requirement_errors would add nothing)
inline bool requirement_ok(const std::string& key, const std::string& op, const std::optional<std::vector<std::string>>& vals) {
  if (!label_key_ok(key)) return false;
  const size_t n = vals ? vals->size() : 0;
  if (op == "In" || op == "NotIn") {
    if (n == 0) return false;
  } else if (op == "=") {
    if (n != 1) return false;
  } else if (op == "Exists" || op == "DoesNotExist") {
    if (n != 0) return false;
  } else {
    if (n != 1 || !parse_int((*vals)[0], nullptr)) return false;
  }
  for (size_t i = 0; i < n; i++)
    if (!label_value_ok((*vals)[i])) return false;
  return true;
}

// ---- error collection --------------------------------------------------------
// field.Error text: "<path>: <Type>: <value>[: <detail>]"
inline std::string field_error(const std::string& path, const char* type, const std::string& value,
                               const std::string& detail) {
  std::string m = path + ": " + type + ": " + value;
  if (!detail.empty()) m += ": " + detail;
  return m;
}
// messages of one labels.NewRequirement (path prefix p: "" or "...matchExpressions[j]"),
// after ErrorList.ToAggregate's de-duplication
inline void requirement_errors(const std::string& p, const std::string& key, const std::string& op,
                               const std::optional<std::vector<std::string>>& vals, std::vector<std::string>* out) {
  auto sub = [&](const std::string& c) { return p.empty() ? c : p + "." + c; };
  std::vector<std::string> errs;
  const std::string kp = label_key_problems(key);
  if (!kp.empty()) errs.push_back(field_error(sub("key"), "Invalid value", quote(key), kp));
  const size_t n = vals ? vals->size() : 0;
  const std::string vp = sub("values");
  if (op == "In" || op == "NotIn") {
    if (n == 0) errs.push_back(field_error(vp, "Invalid value", json_list(vals), "for 'in', 'notin' operators, values set can't be empty"));
  } else if (op == "=") {
    if (n != 1) errs.push_back(field_error(vp, "Invalid value", json_list(vals), "exact-match compatibility requires one single value"));
  } else if (op == "Exists" || op == "DoesNotExist") {
    if (n != 0) errs.push_back(field_error(vp, "Invalid value", json_list(vals), "values set must be empty for exists and does not exist"));
  } else {  // Gt, Lt
    if (n != 1) errs.push_back(field_error(vp, "Invalid value", json_list(vals), "for 'Gt', 'Lt' operators, exactly one value is required"));
    for (size_t i = 0; i < n; i++)
      if (!parse_int((*vals)[i], nullptr))
        errs.push_back(field_error(vp + "[" + std::to_string(i) + "]", "Invalid value", quote((*vals)[i]),
                                   "for 'Gt', 'Lt' operators, the value must be an integer"));
  }
  for (size_t i = 0; i < n; i++) {
    const std::string pv = label_value_problems((*vals)[i]);
    if (!pv.empty())
      errs.push_back(field_error(vp + "[" + std::to_string(i) + "][" + key + "]", "Invalid value", quote((*vals)[i]), pv));
  }
  std::set<std::string> seen;
  for (auto& e : errs)
    if (seen.insert(e).second) out->push_back(e);
}
// aggregate.Error (de-duplicated, bracketed when more than one message)
inline std::string aggregate(const std::vector<std::string>& msgs) {
  if (msgs.size() == 1) return msgs[0];
  std::set<std::string> seen;
  std::string r;
  for (auto& m : msgs)
    if (seen.insert(m).second) r += (seen.size() > 1 ? ", " : "") + m;
  return seen.size() == 1 ? r : "[" + r + "]";
}

// "invalid node selectors: ..." reason, or "" when the selector is valid.
// Go ranges over the map (random order) and reports the first invalid entry;
// here the smallest invalid key is reported (deterministic).
inline std::string node_selector_failure(const std::map<std::string, std::string>& sel) {
  for (auto& kv : sel) {
    if (label_key_ok(kv.first) && label_value_ok(kv.second)) continue;
    std::vector<std::string> errs;
    requirement_errors("", kv.first, "=", std::vector<std::string>{kv.second}, &errs);
    if (errs.empty()) continue;
    std::string m = "invalid node selectors: map[";
    bool first = true;
    for (auto& x : sel) {
      m += (first ? "" : " ") + x.first + ":" + x.second;
      first = false;
    }
    return m + "], reason: " + aggregate(errs);
  }
  return "";
}

// (*v1.NodeSelector).String
inline std::string node_selector_string(const RequiredAffinity& terms) {
  auto reqs = [](const std::vector<Expr>& v) {
    std::string o = "[]NodeSelectorRequirement{";
    for (auto& r : v) {
      o += "NodeSelectorRequirement{Key:" + r.key + ",Operator:" + r.op + ",Values:[";
      if (r.values)
        for (size_t i = 0; i < r.values->size(); i++) o += (i ? " " : "") + (*r.values)[i];
      o += "],},";
    }
    return o + "}";
  };
  std::string o = "&NodeSelector{NodeSelectorTerms:[]NodeSelectorTerm{";
  for (auto& t : terms) o += "NodeSelectorTerm{MatchExpressions:" + reqs(t.exprs) + ",MatchFields:" + reqs(t.fields) + ",},";
  return o + "},}";
}

// "invalid affinity node selectors: ..." reason, or "" when every non-empty
// term parses (nodeaffinity.NewNodeSelector).
inline bool affinity_ok(const RequiredAffinity& terms) {
  for (const Term& t : terms) {
    for (const Expr& e : t.exprs) {
      const bool known = e.op == "In" || e.op == "NotIn" || e.op == "Exists" || e.op == "DoesNotExist" ||
                         e.op == "Gt" || e.op == "Lt";
      if (!known || !requirement_ok(e.key, e.op, e.values)) return false;
    }
    for (const Expr& e : t.fields)
      if (!(e.op == "In" || e.op == "NotIn") || !e.values || e.values->size() != 1) return false;
  }
  return true;
}
inline std::string affinity_failure(const RequiredAffinity& terms) {
  if (affinity_ok(terms)) return "";
  std::vector<std::string> errs;
  for (size_t i = 0; i < terms.size(); i++) {
    const Term& t = terms[i];
    if (t.empty()) continue;
    const std::string tp = "nodeSelectorTerms[" + std::to_string(i) + "]";
    for (size_t j = 0; j < t.exprs.size(); j++) {
      const Expr& e = t.exprs[j];
      const std::string p = tp + ".matchExpressions[" + std::to_string(j) + "]";
      if (e.op == "In" || e.op == "NotIn" || e.op == "Exists" || e.op == "DoesNotExist" || e.op == "Gt" || e.op == "Lt") {
        requirement_errors(p, e.key, e.op, e.values, &errs);
      } else {
        std::string v;
        json_escape(v, e.op);
        errs.push_back(field_error(p + ".operator", "Unsupported value", v,
                                   "supported values: \"In\", \"NotIn\", \"Exists\", \"DoesNotExist\", \"Gt\", \"Lt\""));
      }
    }
    for (size_t j = 0; j < t.fields.size(); j++) {
      const Expr& e = t.fields[j];
      const std::string p = tp + ".matchFields[" + std::to_string(j) + "]";
      if (e.op == "In" || e.op == "NotIn") {
        if (!e.values || e.values->size() != 1)
          errs.push_back(field_error(p + ".values", "Invalid value", json_list(e.values), "must have one element"));
      } else {
        std::string v;
        json_escape(v, e.op);
        errs.push_back(field_error(p + ".operator", "Unsupported value", v, "supported values: \"In\", \"NotIn\""));
      }
    }
  }
  if (errs.empty()) return "";
  return "invalid affinity node selectors: " + node_selector_string(terms) + ", reason: " + aggregate(errs);
}

}  // namespace labelsel
}  // namespace kueue_tas
