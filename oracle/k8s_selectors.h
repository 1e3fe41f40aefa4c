// k8s_selectors.h — TEST INFRASTRUCTURE ONLY (part of the parity oracle).
//
// CPU restatement of the vendored Kubernetes helpers findTopologyAssignment
// uses to filter leaves (reference /root/reference/pkg/cache/scheduler/
// tas_flavor_snapshot.go:879-897, :1599-1610), written in the shape of the Go
// code (Path, field.Error, aggregate) so the failure strings come out the same:
//
//   labels.ValidatedSelectorFromSet / NewRequirement / Requirement.Matches
//       vendor/k8s.io/apimachinery/pkg/labels/selector.go:185-294, :954-968
//   content.IsLabelKey / IsLabelValue / IsDNS1123Subdomain
//       vendor/k8s.io/apimachinery/pkg/api/validate/content/kube.go:43-94, dns.go:64-101
//   field.Path / field.Error / ErrorList.ToAggregate
//       vendor/k8s.io/apimachinery/pkg/util/validation/field/path.go:40-117, errors.go:63-117, :353-368
//   errors.NewAggregate / Flatten / aggregate.Error
//       vendor/k8s.io/apimachinery/pkg/util/errors/errors.go:47-96, :182-200
//   nodeaffinity.NewNodeSelector / NodeSelector.Match
//       vendor/k8s.io/component-helpers/scheduling/corev1/nodeaffinity/nodeaffinity.go:40-292
//   (*v1.NodeSelector).String  vendor/k8s.io/api/core/v1/generated.pb.go:22060-22107
//
// Deterministic choice where Go is not: ValidatedSelectorFromSet ranges over
// a Go map (random order) and returns the first invalid entry's error; this
// restatement visits the keys in sorted order.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <string>
#include <vector>

namespace oracle {
namespace k8s {

// ---- strconv ---------------------------------------------------------------
// strconv.Quote for the byte strings that occur here (ASCII escapes; other
// bytes of valid UTF-8 are kept, invalid bytes become \x..).
inline std::string go_quote(const std::string& s) {
  std::string out = "\"";
  for (size_t i = 0; i < s.size(); i++) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c == '"' || c == '\\') {
      out += '\\';
      out += char(c);
    } else if (c == '\a') out += "\\a";
    else if (c == '\b') out += "\\b";
    else if (c == '\f') out += "\\f";
    else if (c == '\n') out += "\\n";
    else if (c == '\r') out += "\\r";
    else if (c == '\t') out += "\\t";
    else if (c == '\v') out += "\\v";
    else if (c < 0x20 || c == 0x7f) {
      char b[8];
      snprintf(b, sizeof b, "\\x%02x", c);
      out += b;
    } else if (c < 0x80) {
      out += char(c);
    } else {  // multi-byte UTF-8: keep when well formed
      int len = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
      bool ok = len > 0 && i + size_t(len) <= s.size();
      for (int k = 1; ok && k < len; k++) ok = (static_cast<unsigned char>(s[i + k]) >> 6) == 2;
      if (ok) {
        out.append(s, i, size_t(len));
        i += size_t(len) - 1;
      } else {
        char b[8];
        snprintf(b, sizeof b, "\\x%02x", c);
        out += b;
      }
    }
  }
  return out + "\"";
}

// strconv.ParseInt(s, 10, 64) == nil
inline bool parse_int64(const std::string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  unsigned __int128 acc = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    acc = acc * 10 + unsigned(s[i] - '0');
    if (acc > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && acc == ((unsigned __int128)1 << 63)) return false;
  if (out) *out = neg ? int64_t(uint64_t(0) - uint64_t(acc)) : int64_t(acc);
  return true;
}

// encoding/json.Marshal of a []string (HTML-safe escaping; nil -> null)
inline std::string json_strings(const std::optional<std::vector<std::string>>& v) {
  if (!v) return "null";
  std::string out = "[";
  for (size_t i = 0; i < v->size(); i++) {
    if (i) out += ",";
    out += "\"";
    for (unsigned char c : (*v)[i]) {
      if (c == '"') out += "\\\"";
      else if (c == '\\') out += "\\\\";
      else if (c == '\n') out += "\\n";
      else if (c == '\r') out += "\\r";
      else if (c == '\t') out += "\\t";
      else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
        char b[8];
        snprintf(b, sizeof b, "\\u%04x", c);
        out += b;
      } else out += char(c);
    }
    out += "\"";
  }
  return out + "]";
}
inline std::string json_string(const std::string& s) {
  std::string j = json_strings(std::vector<std::string>{s});
  return j.substr(1, j.size() - 2);
}

// ---- field.Path --------------------------------------------------------------
struct Path {
  std::string name;   // "" for a subscript
  std::string index;
  std::shared_ptr<const Path> parent;
};
using PathP = std::shared_ptr<const Path>;
inline PathP child(const PathP& p, const std::string& name) { return std::make_shared<Path>(Path{name, "", p}); }
inline PathP index(const PathP& p, int i) { return std::make_shared<Path>(Path{"", std::to_string(i), p}); }
inline PathP key(const PathP& p, const std::string& k) { return std::make_shared<Path>(Path{"", k, p}); }
inline std::string path_string(const PathP& p) {  // path.go:92-117
  if (!p) return "<nil>";
  std::vector<const Path*> elems;
  for (const Path* q = p.get(); q; q = q->parent.get()) elems.push_back(q);
  std::string buf;
  for (size_t i = elems.size(); i-- > 0;) {
    const Path* q = elems[i];
    if (q->parent && !q->name.empty()) buf += ".";
    if (!q->name.empty()) buf += q->name;
    else buf += "[" + q->index + "]";
  }
  return buf;
}

// ---- field.Error (errors.go:63-117) -------------------------------------------
// BadValue kinds that occur on this path: a Go string (%q), a []string and a
// named string type (both rendered with json.Marshal).
struct FieldError {
  std::string type;    // "Invalid value" / "Unsupported value"
  std::string field;
  std::string value;   // already rendered
  std::string detail;
  std::string error() const {
    std::string s = type + ": " + value;
    if (!detail.empty()) s += ": " + detail;
    return field + ": " + s;
  }
};
inline FieldError invalid_str(const PathP& p, const std::string& v, const std::string& detail) {
  return {"Invalid value", path_string(p), go_quote(v), detail};
}
inline FieldError invalid_list(const PathP& p, const std::optional<std::vector<std::string>>& v, const std::string& detail) {
  return {"Invalid value", path_string(p), json_strings(v), detail};
}
inline FieldError not_supported(const PathP& p, const std::string& v, const std::vector<std::string>& valid) {
  std::string detail;
  if (!valid.empty()) {
    detail = "supported values: ";
    for (size_t i = 0; i < valid.size(); i++) detail += (i ? ", " : "") + go_quote(valid[i]);
  }
  return {"Unsupported value", path_string(p), json_string(v), detail};
}
// ErrorList.ToAggregate drops repeated messages; the aggregate's Error()
// also de-duplicates and brackets more than one distinct message.
inline std::vector<std::string> to_aggregate(const std::vector<FieldError>& list) {
  std::vector<std::string> msgs;
  std::set<std::string> seen;
  for (auto& e : list) {
    std::string m = e.error();
    if (seen.insert(m).second) msgs.push_back(m);
  }
  return msgs;
}
inline std::string aggregate_error(const std::vector<std::string>& msgs) {  // errors.go:70-96
  if (msgs.empty()) return "";
  if (msgs.size() == 1) return msgs[0];
  std::set<std::string> seen;
  std::string result;
  for (auto& m : msgs) {
    if (!seen.insert(m).second) continue;
    if (seen.size() > 1) result += ", ";
    result += m;
  }
  if (seen.size() == 1) return result;
  return "[" + result + "]";
}

// ---- content validators (kube.go, dns.go, errors.go) ---------------------------
inline std::string regex_error(const std::string& msg, const std::string& re, const std::vector<std::string>& examples) {
  if (examples.empty()) return msg + " (regex used for validation is '" + re + "')";
  std::string m = msg + " (e.g. ";
  for (size_t i = 0; i < examples.size(); i++) {
    if (i > 0) m += " or ";
    m += "'" + examples[i] + "', ";
  }
  return m + "regex used for validation is '" + re + "')";
}
inline bool is_alnum(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
// ^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$
inline bool match_label_key_name(const std::string& s) {
  if (s.empty() || !is_alnum(s.front()) || !is_alnum(s.back())) return false;
  for (unsigned char c : s)
    if (!(is_alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
// ^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$
inline bool match_dns1123_subdomain(const std::string& s) {
  auto lo = [](unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
  size_t start = 0;
  while (true) {
    size_t end = s.find('.', start);
    std::string part = s.substr(start, end == std::string::npos ? std::string::npos : end - start);
    if (part.empty() || !lo(part.front()) || !lo(part.back())) return false;
    for (unsigned char c : part)
      if (!(lo(c) || c == '-')) return false;
    if (end == std::string::npos) return true;
    start = end + 1;
  }
}
static const char* kLabelKeyFmt = "([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]";
static const char* kLabelKeyErrMsg =
    "must consist of alphanumeric characters, '-', '_' or '.', and must start and end with an alphanumeric character";
inline std::vector<std::string> is_dns1123_subdomain(const std::string& v) {
  std::vector<std::string> errs;
  if (v.size() > 253) errs.push_back("must be no more than 253 bytes");
  if (!match_dns1123_subdomain(v))
    errs.push_back(regex_error(
        "a lowercase RFC 1123 subdomain must consist of lower case alphanumeric characters, '-' or '.', and must start "
        "and end with an alphanumeric character",
        "[a-z0-9]([-a-z0-9]*[a-z0-9])?(\\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*", {"example.com"}));
  return errs;
}
inline std::vector<std::string> is_label_key(const std::string& v) {  // kube.go:43-72
  std::vector<std::string> errs;
  std::vector<std::string> parts;
  size_t start = 0;
  while (true) {
    size_t e = v.find('/', start);
    parts.push_back(v.substr(start, e == std::string::npos ? std::string::npos : e - start));
    if (e == std::string::npos) break;
    start = e + 1;
  }
  std::string name;
  if (parts.size() == 1) {
    name = parts[0];
  } else if (parts.size() == 2) {
    const std::string& prefix = parts[0];
    name = parts[1];
    if (prefix.empty()) errs.push_back("prefix part must be non-empty");
    else
      for (auto& m : is_dns1123_subdomain(prefix)) errs.push_back("prefix part " + m);
  } else {
    errs.push_back("a valid label key " + regex_error(kLabelKeyErrMsg, kLabelKeyFmt, {"MyName", "my.name", "123-abc"}) +
                   " with an optional DNS subdomain prefix and '/' (e.g. 'example.com/MyName')");
    return errs;
  }
  if (name.empty()) errs.push_back("name part must be non-empty");
  else if (name.size() > 63) errs.push_back("name part must be no more than 63 bytes");
  if (!match_label_key_name(name))
    errs.push_back("name part " + regex_error(kLabelKeyErrMsg, kLabelKeyFmt, {"MyName", "my.name", "123-abc"}));
  return errs;
}
inline std::vector<std::string> is_label_value(const std::string& v) {  // kube.go:85-94
  std::vector<std::string> errs;
  if (v.size() > 63) errs.push_back("must be no more than 63 bytes");
  if (!v.empty() && !match_label_key_name(v))
    errs.push_back(regex_error(
        "a valid label must be an empty string or consist of alphanumeric characters, '-', '_' or '.', and must start "
        "and end with an alphanumeric character",
        "(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?", {"MyValue", "my_value", "12345"}));
  return errs;
}
inline std::string join(const std::vector<std::string>& v, const std::string& sep) {
  std::string o;
  for (size_t i = 0; i < v.size(); i++) o += (i ? sep : "") + v[i];
  return o;
}

// ---- labels.Requirement (selector.go:160-294) ------------------------------------
enum class Op { In, NotIn, Equals, Exists, DoesNotExist, Gt, Lt };
struct Requirement {
  std::string key;
  Op op;
  std::vector<std::string> values;
  bool matches(const std::map<std::string, std::string>& ls) const {
    auto it = ls.find(key);
    switch (op) {
      case Op::In:
      case Op::Equals:
        if (it == ls.end()) return false;
        for (auto& v : values)
          if (v == it->second) return true;
        return false;
      case Op::NotIn:
        if (it == ls.end()) return true;
        for (auto& v : values)
          if (v == it->second) return false;
        return true;
      case Op::Exists: return it != ls.end();
      case Op::DoesNotExist: return it == ls.end();
      case Op::Gt:
      case Op::Lt: {
        if (it == ls.end()) return false;
        int64_t lv, rv;
        if (!parse_int64(it->second, &lv)) return false;
        if (values.size() != 1) return false;
        if (!parse_int64(values[0], &rv)) return false;
        return (op == Op::Gt && lv > rv) || (op == Op::Lt && lv < rv);
      }
    }
    return false;
  }
};
// NewRequirement: the field errors of one requirement (before ToAggregate)
inline std::vector<FieldError> new_requirement(const std::string& k, Op op,
                                               const std::optional<std::vector<std::string>>& vals, const PathP& path) {
  std::vector<FieldError> errs;
  auto kerr = is_label_key(k);
  if (!kerr.empty()) errs.push_back(invalid_str(child(path, "key"), k, join(kerr, "; ")));
  PathP vp = child(path, "values");
  const size_t n = vals ? vals->size() : 0;
  switch (op) {
    case Op::In:
    case Op::NotIn:
      if (n == 0) errs.push_back(invalid_list(vp, vals, "for 'in', 'notin' operators, values set can't be empty"));
      break;
    case Op::Equals:
      if (n != 1) errs.push_back(invalid_list(vp, vals, "exact-match compatibility requires one single value"));
      break;
    case Op::Exists:
    case Op::DoesNotExist:
      if (n != 0) errs.push_back(invalid_list(vp, vals, "values set must be empty for exists and does not exist"));
      break;
    case Op::Gt:
    case Op::Lt:
      if (n != 1) errs.push_back(invalid_list(vp, vals, "for 'Gt', 'Lt' operators, exactly one value is required"));
      for (size_t i = 0; i < n; i++)
        if (!parse_int64((*vals)[i], nullptr))
          errs.push_back(invalid_str(index(vp, int(i)), (*vals)[i], "for 'Gt', 'Lt' operators, the value must be an integer"));
      break;
  }
  for (size_t i = 0; i < n; i++) {
    auto verr = is_label_value((*vals)[i]);
    if (!verr.empty()) errs.push_back(invalid_str(key(index(vp, int(i)), k), (*vals)[i], join(verr, "; ")));
  }
  return errs;
}

// labels.ValidatedSelectorFromSet (selector.go:954-968): "" on success, else
// the first failing requirement's aggregated error (sorted key order).
inline std::string validated_selector_from_set(const std::map<std::string, std::string>& set) {
  for (auto& kv : set) {
    auto errs = new_requirement(kv.first, Op::Equals, std::vector<std::string>{kv.second}, nullptr);
    if (!errs.empty()) return aggregate_error(to_aggregate(errs));
  }
  return "";
}
// fmt %s of a map[string]string: "map[k1:v1 k2:v2]" in sorted key order
inline std::string go_map_string(const std::map<std::string, std::string>& m) {
  std::string o = "map[";
  bool first = true;
  for (auto& kv : m) {
    if (!first) o += " ";
    first = false;
    o += kv.first + ":" + kv.second;
  }
  return o + "]";
}

// ---- v1.NodeSelector and nodeaffinity --------------------------------------------
struct NodeSelectorRequirement {
  std::string key, op;
  std::optional<std::vector<std::string>> values;
};
struct NodeSelectorTerm {
  std::vector<NodeSelectorRequirement> matchExpressions, matchFields;
};
struct NodeSelector {
  std::vector<NodeSelectorTerm> terms;
};

// (*v1.NodeSelector).String (generated.pb.go:22060-22107)
inline std::string requirement_string(const NodeSelectorRequirement& r) {
  std::string vals = "[";
  if (r.values)
    for (size_t i = 0; i < r.values->size(); i++) vals += (i ? " " : "") + (*r.values)[i];
  vals += "]";
  return "&NodeSelectorRequirement{Key:" + r.key + ",Operator:" + r.op + ",Values:" + vals + ",}";
}
inline std::string strip_first_amp(std::string s) {
  size_t p = s.find('&');
  if (p != std::string::npos) s.erase(p, 1);
  return s;
}
inline std::string node_selector_string(const NodeSelector& ns) {
  std::string terms = "[]NodeSelectorTerm{";
  for (auto& t : ns.terms) {
    std::string me = "[]NodeSelectorRequirement{";
    for (auto& r : t.matchExpressions) me += strip_first_amp(requirement_string(r)) + ",";
    me += "}";
    std::string mf = "[]NodeSelectorRequirement{";
    for (auto& r : t.matchFields) mf += strip_first_amp(requirement_string(r)) + ",";
    mf += "}";
    terms += strip_first_amp("&NodeSelectorTerm{MatchExpressions:" + me + ",MatchFields:" + mf + ",}") + ",";
  }
  terms += "}";
  return "&NodeSelector{NodeSelectorTerms:" + terms + ",}";
}

struct FieldTerm {  // fields.hasTerm / notHasTerm
  std::string field, value;
  bool equal;
};
struct ParsedTerm {  // nodeaffinity.nodeSelectorTerm (nodeaffinity.go:164-201)
  bool hasLabels = false;
  std::vector<Requirement> labels;  // empty with hasLabels: labels.Nothing()
  bool hasFields = false;
  std::vector<FieldTerm> fields;     // empty with hasFields: fields.Nothing()
  bool match(const std::map<std::string, std::string>& nodeLabels, const std::string& nodeName) const {
    if (hasLabels) {
      if (labels.empty()) return false;  // labels.Nothing()
      for (auto& r : labels)
        if (!r.matches(nodeLabels)) return false;
    }
    if (hasFields && !nodeName.empty()) {  // nodeFields = {"metadata.name": name} when the name is set
      if (fields.empty()) return false;   // fields.Nothing()
      for (auto& f : fields) {
        const std::string got = f.field == "metadata.name" ? nodeName : std::string();
        if ((got == f.value) != f.equal) return false;
      }
    }
    return true;
  }
};
struct ParsedNodeSelector {
  std::vector<ParsedTerm> terms;
  bool match(const std::map<std::string, std::string>& nodeLabels, const std::string& nodeName) const {
    for (auto& t : terms)
      if (t.match(nodeLabels, nodeName)) return true;
    return false;
  }
};

// nodeaffinity.NewNodeSelector: "" and *out on success, else the flattened
// aggregate error message.
inline std::string new_node_selector(const NodeSelector& ns, ParsedNodeSelector* out) {
  out->terms.clear();
  std::vector<std::string> errs;  // flattened messages of every term's parse errors
  PathP path = child(nullptr, "nodeSelectorTerms");
  for (size_t i = 0; i < ns.terms.size(); i++) {
    const NodeSelectorTerm& term = ns.terms[i];
    if (term.matchExpressions.empty() && term.matchFields.empty()) continue;  // isEmptyNodeSelectorTerm
    PathP p = index(path, int(i));
    ParsedTerm pt;
    std::vector<std::string> terrs;
    if (!term.matchExpressions.empty()) {  // nodeSelectorRequirementsAsSelector (:214-251)
      pt.hasLabels = true;
      PathP ep = child(p, "matchExpressions");
      std::vector<std::string> rerrs;
      for (size_t j = 0; j < term.matchExpressions.size(); j++) {
        const auto& expr = term.matchExpressions[j];
        PathP rp = index(ep, int(j));
        Op op;
        if (expr.op == "In") op = Op::In;
        else if (expr.op == "NotIn") op = Op::NotIn;
        else if (expr.op == "Exists") op = Op::Exists;
        else if (expr.op == "DoesNotExist") op = Op::DoesNotExist;
        else if (expr.op == "Gt") op = Op::Gt;
        else if (expr.op == "Lt") op = Op::Lt;
        else {
          rerrs.push_back(not_supported(child(rp, "operator"), expr.op, {"In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"})
                              .error());
          continue;
        }
        auto ferrs = new_requirement(expr.key, op, expr.values, rp);
        if (!ferrs.empty()) {
          for (auto& m : to_aggregate(ferrs)) rerrs.push_back(m);  // Flatten of the requirement's aggregate
        } else {
          pt.labels.push_back({expr.key, op, expr.values ? *expr.values : std::vector<std::string>{}});
        }
      }
      if (!rerrs.empty()) {
        terrs.insert(terrs.end(), rerrs.begin(), rerrs.end());
        pt.labels.clear();
      }
    }
    if (!term.matchFields.empty()) {  // nodeSelectorRequirementsAsFieldSelector (:260-293)
      pt.hasFields = true;
      PathP fp = child(p, "matchFields");
      std::vector<std::string> ferrs;
      for (size_t j = 0; j < term.matchFields.size(); j++) {
        const auto& expr = term.matchFields[j];
        PathP rp = index(fp, int(j));
        if (expr.op == "In" || expr.op == "NotIn") {
          const size_t n = expr.values ? expr.values->size() : 0;
          if (n != 1) ferrs.push_back(invalid_list(child(rp, "values"), expr.values, "must have one element").error());
          else pt.fields.push_back({expr.key, (*expr.values)[0], expr.op == "In"});
        } else {
          ferrs.push_back(not_supported(child(rp, "operator"), expr.op, {"In", "NotIn"}).error());
        }
      }
      if (!ferrs.empty()) {
        terrs.insert(terrs.end(), ferrs.begin(), ferrs.end());
        pt.fields.clear();
      }
    }
    errs.insert(errs.end(), terrs.begin(), terrs.end());
    out->terms.push_back(std::move(pt));
  }
  if (!errs.empty()) {
    out->terms.clear();
    return aggregate_error(errs);
  }
  return "";
}

}  // namespace k8s
}  // namespace oracle
