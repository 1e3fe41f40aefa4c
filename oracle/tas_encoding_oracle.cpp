// tas_encoding_oracle.cpp — CPU restatement of the v1beta2 TopologyAssignment
// wire encoding (reference pkg/util/tas/tas_assignment.go).
//
// TEST INFRASTRUCTURE ONLY (the checker, see tas_oracle.cpp's header): loaded
// by tests/ alone.  Pinned by the reference's own vectors,
// tests/golden/tas_v1beta2_encoding.json (tools/extract_encoding_goldens.py
// from tas_assignment_test.go bothWaysTestCases / oneWayTestCases).
//
// JSON shapes (same as the fixture):
//   internal: {"levels": [...], "domains": [{"values": [...], "count": n}]}
//   v1beta2:  {"levels": [...], "slices": [{"domainCount": n,
//              "podCounts": {"universal": c} | {"individual": [...]},
//              "valuesPerLevel": [{"universal": s} |
//                                 {"individual": {"prefix"?, "suffix"?, "roots": [...]}}]}]}
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "mini_json.h"

namespace encoding_oracle {

struct LevelValues {  // kueue.TopologyAssignmentSliceLevelValues
  bool universal = false;
  std::string value;  // Universal
  bool has_prefix = false, has_suffix = false;
  std::string prefix, suffix;
  std::vector<std::string> roots;
};

// fillSingleCompactSliceValues (tas_assignment.go:135-197), sequentially as written.
static LevelValues fill_single_compact_slice_values(const std::vector<std::string>& in) {
  std::string prefix, suffix;
  size_t maxLen = 0, minLen = 0, count = 0;
  for (const std::string& s : in) {
    count++;
    if (count == 1) {
      prefix = s;
      suffix = s;
      maxLen = minLen = s.size();
      continue;
    }
    const size_t n = s.size();
    minLen = std::min(minLen, n);
    maxLen = std::max(maxLen, n);
    if (n < prefix.size()) prefix = prefix.substr(0, n);
    if (n < suffix.size()) suffix = suffix.substr(suffix.size() - n);
    for (size_t i = 0; i < prefix.size(); i++)
      if (s[i] != prefix[i]) {
        prefix = prefix.substr(0, i);
        break;
      }
    for (size_t i = 0; i < suffix.size(); i++)
      if (s[s.size() - 1 - i] != suffix[suffix.size() - 1 - i]) {
        suffix = suffix.substr(suffix.size() - i);
        break;
      }
  }
  LevelValues v;
  if (prefix.size() == maxLen) {  // all strings equal (:174-178)
    v.universal = true;
    v.value = prefix;
    return v;
  }
  if (prefix.size() + suffix.size() > minLen) prefix = prefix.substr(0, minLen - suffix.size());  // :180-184
  v.has_prefix = !prefix.empty();
  v.has_suffix = !suffix.empty();
  v.prefix = prefix;
  v.suffix = suffix;
  for (const std::string& s : in) v.roots.push_back(s.substr(prefix.size(), s.size() - prefix.size() - suffix.size()));
  return v;
}

static void quote(std::string& out, const std::string& s) { ojson::quote(out, s); }

// singleCompactSliceEncoding (:199-249) / V1Beta2From (:251-259).
static std::string v1beta2_from(const ojson::Value& ta) {
  std::string out = "{\"levels\":[";
  const auto& levels = ta.at("levels").a;
  for (size_t i = 0; i < levels.size(); i++) {
    if (i) out += ",";
    quote(out, levels[i].as_str());
  }
  out += "],\"slices\":[";
  const auto& doms = ta.at("domains").a;
  const size_t n = doms.size();
  if (n == 0) return out + "]}";
  out += "{\"domainCount\":" + std::to_string(n) + ",\"podCounts\":";
  bool same = true;
  for (size_t i = 1; i < n; i++)
    if (doms[i].at("count").as_int() != doms[i - 1].at("count").as_int()) same = false;
  if (same) {
    out += "{\"universal\":" + std::to_string(doms[0].at("count").as_int()) + "}";
  } else {
    out += "{\"individual\":[";
    for (size_t i = 0; i < n; i++) out += (i ? "," : "") + std::to_string(doms[i].at("count").as_int());
    out += "]}";
  }
  out += ",\"valuesPerLevel\":[";
  for (size_t l = 0; l < levels.size(); l++) {
    std::vector<std::string> vals;
    for (auto& d : doms) vals.push_back(d.at("values").a.at(l).as_str());
    LevelValues v = fill_single_compact_slice_values(vals);
    if (l) out += ",";
    if (v.universal) {
      out += "{\"universal\":";
      quote(out, v.value);
      out += "}";
      continue;
    }
    out += "{\"individual\":{";
    if (v.has_prefix) {
      out += "\"prefix\":";
      quote(out, v.prefix);
      out += ",";
    }
    if (v.has_suffix) {
      out += "\"suffix\":";
      quote(out, v.suffix);
      out += ",";
    }
    out += "\"roots\":[";
    for (size_t i = 0; i < v.roots.size(); i++) {
      if (i) out += ",";
      quote(out, v.roots[i]);
    }
    out += "]}}";
  }
  return out + "]}]}";
}

// InternalFrom / InternalSeqFrom (:103-133) with valueAtIndex / countAtIndex (:40-55).
static std::string internal_from(const ojson::Value& ta) {
  std::string out = "{\"levels\":[";
  const auto& levels = ta.at("levels").a;
  for (size_t i = 0; i < levels.size(); i++) {
    if (i) out += ",";
    quote(out, levels[i].as_str());
  }
  out += "],\"domains\":[";
  bool first = true;
  for (auto& sl : ta.at("slices").a) {
    const int64_t dc = sl.at("domainCount").as_int();
    const ojson::Value& pc = sl.at("podCounts");
    for (int64_t i = 0; i < dc; i++) {
      if (!first) out += ",";
      first = false;
      out += "{\"values\":[";
      for (size_t l = 0; l < levels.size(); l++) {
        const ojson::Value& v = sl.at("valuesPerLevel").a.at(l);
        std::string s;
        if (auto u = v.get("universal")) {
          s = u->as_str();
        } else {
          const ojson::Value& ind = v.at("individual");
          auto p = ind.get("prefix");
          auto x = ind.get("suffix");
          s = (p ? p->as_str() : "") + ind.at("roots").a.at(size_t(i)).as_str() + (x ? x->as_str() : "");
        }
        if (l) out += ",";
        quote(out, s);
      }
      int64_t c = pc.get("universal") ? pc.get("universal")->as_int() : pc.at("individual").a.at(size_t(i)).as_int();
      out += "],\"count\":" + std::to_string(c) + "}";
    }
  }
  return out + "]}";
}

static char* dup_out(const std::string& s) {
  char* p = static_cast<char*>(malloc(s.size() + 1));
  memcpy(p, s.data(), s.size() + 1);
  return p;
}

}  // namespace encoding_oracle

extern "C" {

// direction 0: internal -> v1beta2 (V1Beta2From); 1: v1beta2 -> internal (InternalFrom).
int tas_oracle_encoding(const char* json, int direction, char** out_json) {
  using namespace encoding_oracle;
  try {
    ojson::Value v = ojson::parse(json);
    *out_json = dup_out(direction == 0 ? v1beta2_from(v) : internal_from(v));
    return 0;
  } catch (const std::exception& e) {
    std::string out = "{\"error\":";
    ojson::quote(out, e.what());
    *out_json = dup_out(out + "}");
    return -1;
  }
}

}  // extern "C"
