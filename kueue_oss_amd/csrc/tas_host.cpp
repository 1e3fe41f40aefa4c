// tas_host.cpp — host layer of libkueue_tas.so: the C++ mirror of the Go API
// of Kueue's TAS evaluation path on top of the device layer.
//
// Mirrors (reference /root/reference/pkg/cache/scheduler/):
//   TASFlavorCache.snapshot + caches       tas_flavor.go:118-171, tas_nodes_cache.go:38-72,
//                                          tas_non_tas_pod_cache.go:46-120
//   TASFlavorSnapshot.addNode/initialize   tas_flavor_snapshot.go:160-241
//   FindTopologyAssignmentsForFlavor       :519-594 (groups, leader/workers :596-609,
//                                          assumedUsage :658-666, stop at first failure)
//   findTopologyAssignment prelude         :804-897 (requests + pods:1, slice size/levels,
//                                          validation reasons, tolerations, nodeSelector,
//                                          required node affinity compiled to label-id sets)
//   notFitMessage / multiLayerNotFitMessage / ExclusionStats.formatReasons
//                                          :1721-1793, :480-499
// Everything between the prelude and buildAssignment runs on the GPU
// (tas_kernels.hip).  This layer never evaluates a placement on the CPU: if the
// device library or a GPU is unavailable, creation fails loudly.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <deque>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/kueue_tas_debug.h"
#include "json_reader.h"
#include "label_selectors.h"
#include "tas_balanced.h"
#include "tas_pool.h"

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

namespace kueue_tas {

using Requests = std::map<std::string, int64_t>;

// fn(a, b) over [0, n) cut into contiguous ranges of at least `grain`
// items, on up to 8 threads (the host mirror's O(N) passes).
template <class F>
static void parallel_ranges(size_t n, size_t grain, F fn) {
  const size_t t = std::min<size_t>({8, std::max<unsigned>(1, std::thread::hardware_concurrency()), n / grain + 1});
  if (t <= 1) {
    fn(size_t(0), n);
    return;
  }
  std::vector<std::thread> pool;
  for (size_t k = 1; k < t; k++) pool.emplace_back(fn, n * k / t, n * (k + 1) / t);
  fn(size_t(0), n / t);
  for (auto& th : pool) th.join();
}

// A leaf index by string key (DomainID, node name) through a stable slot per
// key: reordering the leaves (FlavorSnapshot::flush_joins) rewrites one
// contiguous int array, never the hash table.
struct LeafIndex {
  std::unordered_map<std::string, int32_t> slot;
  std::vector<int32_t> leaf;
  int32_t find(const std::string& k) const {
    auto it = slot.find(k);
    return it == slot.end() ? -1 : leaf[size_t(it->second)];
  }
  bool count(const std::string& k) const { return slot.count(k) != 0; }
  int32_t at(const std::string& k) const { return leaf[size_t(slot.at(k))]; }
  void add(const std::string& k, int32_t l) {  // the first leaf of a key stays
    if (slot.emplace(k, int32_t(leaf.size())).second) leaf.push_back(l);
  }
  void set(const std::string& k, int32_t l) {
    auto r = slot.emplace(k, int32_t(leaf.size()));
    if (r.second) leaf.push_back(l);
    else leaf[size_t(r.first->second)] = l;
  }
  void clear() {
    slot.clear();
    leaf.clear();
  }
  void remap(const std::vector<int32_t>& rm) {
    for (auto& l : leaf) l = rm[size_t(l)];
  }
};

// Per-leaf values held by pointer: reordering the leaves moves pointers, not
// the std::map headers (whose tree root points back at its header — a cache
// miss per moved map).
template <class T>
struct LeafVec {
  std::vector<std::unique_ptr<T>> v;
  LeafVec() = default;
  LeafVec(const LeafVec& o) { *this = o; }
  LeafVec(LeafVec&&) noexcept = default;
  LeafVec& operator=(LeafVec&&) noexcept = default;
  LeafVec& operator=(const LeafVec& o) {
    if (this != &o) {
      v.clear();
      v.reserve(o.v.size());
      for (auto& p : o.v) v.push_back(std::make_unique<T>(*p));
    }
    return *this;
  }
  T& operator[](size_t i) { return *v[i]; }
  const T& operator[](size_t i) const { return *v[i]; }
  size_t size() const { return v.size(); }
  void resize(size_t n) {
    const size_t o = v.size();
    v.resize(n);
    for (size_t i = o; i < n; i++) v[i] = std::make_unique<T>();
  }
  struct const_iterator {
    typename std::vector<std::unique_ptr<T>>::const_iterator it;
    const T& operator*() const { return **it; }
    const_iterator& operator++() {
      ++it;
      return *this;
    }
    bool operator!=(const const_iterator& o) const { return it != o.it; }
  };
  const_iterator begin() const { return {v.begin()}; }
  const_iterator end() const { return {v.end()}; }
};
static const char* kHostname = "kubernetes.io/hostname";

static int64_t add64(int64_t a, int64_t b) { return int64_t(uint64_t(a) + uint64_t(b)); }
static int64_t sub64(int64_t a, int64_t b) { return int64_t(uint64_t(a) - uint64_t(b)); }
static int64_t mul64(int64_t a, int64_t b) { return int64_t(uint64_t(a) * uint64_t(b)); }
static void req_add(Requests& r, const Requests& o) {
  for (auto& kv : o) r[kv.first] = add64(r[kv.first], kv.second);
}
static void req_sub(Requests& r, const Requests& o) {
  for (auto& kv : o) r[kv.first] = sub64(r[kv.first], kv.second);
}
static int32_t go_div32(int32_t a, int32_t b) {
  if (b == -1) return int32_t(0u - uint32_t(a));
  return a / b;
}

// Resource names interned process-wide (ids never change): a compiled request
// maps each name to its snapshot column through one array lookup.
static int32_t intern_resource(const std::string& name) {
  static std::mutex mu;
  static std::unordered_map<std::string, int32_t> ids;
  std::lock_guard<std::mutex> lock(mu);
  return ids.emplace(name, int32_t(ids.size())).first->second;
}

struct Taint {
  std::string key, value, effect;
  bool operator==(const Taint& o) const { return key == o.key && value == o.value && effect == o.effect; }
  bool operator<(const Taint& o) const {
    return std::tie(key, value, effect) < std::tie(o.key, o.value, o.effect);
  }
};
struct Toleration {
  std::string key, op, value, effect;
  bool operator<(const Toleration& o) const {
    return std::tie(key, op, value, effect) < std::tie(o.key, o.op, o.value, o.effect);
  }
};

// Taint.ToString (vendor/k8s.io/api/core/v1/taint.go:28-39)
static std::string taint_string(const Taint& t) {
  if (t.effect.empty()) return t.value.empty() ? t.key : t.key + "=" + t.value + ":";
  return t.value.empty() ? t.key + ":" + t.effect : t.key + "=" + t.value + ":" + t.effect;
}

// content.IsDecimalInteger + strconv.ParseInt (validate/content/decimal_int.go:30-62)
static bool decimal_int(const std::string& v, int64_t* out) {
  if (v.empty()) return false;
  size_t i = v[0] == '-' ? 1 : 0;
  if (i == 1 && v.size() == 1) return false;
  if (v[i] == '0') {
    if (v.size() == 1) {
      *out = 0;
      return true;
    }
    return false;
  }
  unsigned __int128 acc = 0;
  for (size_t j = i; j < v.size(); j++) {
    if (v[j] < '0' || v[j] > '9') return false;
    acc = acc * 10 + unsigned(v[j] - '0');
    if (acc > ((unsigned __int128)1 << 63)) return false;
  }
  if (i == 0 && acc == ((unsigned __int128)1 << 63)) return false;
  *out = i ? int64_t(uint64_t(0) - uint64_t(acc)) : int64_t(acc);
  return true;
}

// Toleration.ToleratesTaint with enableComparisonOperators=true
// (vendor/k8s.io/api/core/v1/toleration.go:52-112; tas_flavor_snapshot.go:1586)
static bool tolerates(const Toleration& t, const Taint& x) {
  if (!t.effect.empty() && t.effect != x.effect) return false;
  if (!t.key.empty() && t.key != x.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == x.value;
  if (t.op == "Exists") return true;
  if (t.op == "Lt" || t.op == "Gt") {
    int64_t a, b;
    if (!decimal_int(t.value, &a) || !decimal_int(x.value, &b)) return false;
    return t.op == "Lt" ? b < a : b > a;
  }
  return false;
}

// decimal text of v appended to out (strconv.FormatInt; no locale, no allocation)
static void append_int(std::string& out, int64_t v) {
  char b[24];
  char* e = b + sizeof b;
  char* p = e;
  uint64_t u = v < 0 ? uint64_t(0) - uint64_t(v) : uint64_t(v);
  do {
    *--p = char('0' + u % 10);
    u /= 10;
  } while (u);
  if (v < 0) *--p = '-';
  out.append(p, size_t(e - p));
}

static std::string go_quote(const std::string& s) {  // strconv.Quote for ASCII input
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += char(c);
    } else if (c == '\n') o += "\\n";
    else if (c == '\t') o += "\\t";
    else if (c == '\r') o += "\\r";
    else if (c < 0x20 || c == 0x7f) {
      char b[8];
      snprintf(b, sizeof b, "\\x%02x", c);
      o += b;
    } else o += char(c);
  }
  return o + "\"";
}

// resources.ResourceQuantityString (pkg/resources/requests.go:113-150) as
// resource.Quantity.String renders it (vendor/k8s.io/apimachinery/pkg/api/
// resource/quantity.go:425-467 CanonicalizeBytes, amount.go:257-293,
// suffix.go): cpu is a DecimalSI milli-quantity; memory, ephemeral-storage
// and hugepages-* are newCanonicalQuantity(v, BinarySI) (the BinarySI string
// re-parsed: a value that is no multiple of 1024 prints as DecimalSI);
// anything else is a DecimalSI quantity.  Exact for every int64.
static std::string decimal_si(int64_t v, int exp) {  // AsCanonicalBytes + decimal suffix
  if (v == 0) return "0";
  const bool neg = v < 0;
  unsigned __int128 a = neg ? (unsigned __int128)(uint64_t(0) - uint64_t(v)) : (unsigned __int128)uint64_t(v);
  while (a >= 10 && a % 10 == 0) {
    a /= 10;
    exp++;
  }
  switch (exp % 3) {  // Go's % keeps the dividend's sign, as C++'s does
    case 1: case -2: a *= 10; exp -= 1; break;
    case 2: case -1: a *= 100; exp -= 2; break;
    default: break;
  }
  char b[48];
  char* e = b + sizeof b;
  char* p = e;
  do {
    *--p = char('0' + int(a % 10));
    a /= 10;
  } while (a);
  if (neg) *--p = '-';
  std::string s(p, size_t(e - p));
  switch (exp) {
    case -9: return s + "n";
    case -6: return s + "u";
    case -3: return s + "m";
    case 3: return s + "k";
    case 6: return s + "M";
    case 9: return s + "G";
    case 12: return s + "T";
    case 15: return s + "P";
    case 18: return s + "E";
    default: return s;  // 0 (and no other exponent arises from an int64)
  }
}
static std::string resource_quantity_string(const std::string& name, int64_t v) {
  if (name == "cpu") return decimal_si(v, -3);
  const bool binary = name == "memory" || name == "ephemeral-storage" || name.rfind("hugepages-", 0) == 0;
  if (!binary) return decimal_si(v, 0);
  if (v == 0) return "0";
  if (v > -1024 && v < 1024) return decimal_si(v, 0);
  const bool neg = v < 0;
  uint64_t a = neg ? uint64_t(0) - uint64_t(v) : uint64_t(v);
  int e = 0;
  while (a >= 1024 && a % 1024 == 0) {
    a /= 1024;
    e++;
  }
  if (e == 0) return decimal_si(v, 0);  // no suffix: re-parsed as DecimalSI
  static const char* kBin[] = {"", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  std::string s = std::to_string(a);
  return (neg ? "-" : "") + s + kBin[e];
}

struct NodeInfo {
  std::string name;
  std::map<std::string, std::string> labels;
  std::vector<Taint> taints;
  Requests allocatable;
};

struct SliceConstraint {
  std::string topology;
  int32_t size;
};
struct TopologyRequest {  // kueue.PodSetTopologyRequest (apis/kueue/v1beta2/workload_types.go:165-249)
  std::optional<std::string> required, preferred, sliceRequiredTopology;
  std::optional<bool> unconstrained;
  std::optional<int32_t> sliceSize;
  std::vector<SliceConstraint> constraints;
};
// utiltas.TopologyAssignment with explicit values (the existing assignment of
// an admitted workload comes from its status, not from this snapshot).
struct ExplicitAssignment {
  std::vector<std::string> levels;
  std::vector<std::pair<std::vector<std::string>, int32_t>> domains;  // (values, count)
};
static std::string join_values(const std::vector<std::string>& v) {  // utiltas.DomainID
  std::string id;
  for (size_t k = 0; k < v.size(); k++) {
    if (k) id += ",";
    id += v[k];
  }
  return id;
}
static ExplicitAssignment parse_explicit(const kjson::Node& ta) {
  ExplicitAssignment a;
  for (auto& l : ta["levels"].items) a.levels.push_back(l.s());
  for (auto& d : ta["domains"].items) {
    std::vector<std::string> vals;
    for (auto& x : d["values"].items) vals.push_back(x.s());
    a.domains.emplace_back(std::move(vals), int32_t(d["count"].i64()));
  }
  return a;
}
struct TASPodSetRequests {  // tas_flavor_snapshot.go:356-367
  std::string name;
  std::optional<TopologyRequest> topologyRequest;
  Requests singlePodRequests;
  std::vector<std::pair<int32_t, int64_t>> requestIds;  // singlePodRequests by interned name, same order
  int32_t count = 0;
  bool implied = false;
  std::optional<std::string> podSetGroupName;
  std::vector<Toleration> tolerations;
  std::optional<std::map<std::string, std::string>> nodeSelector;
  // PodSpec affinity.nodeAffinity.requiredDuringSchedulingIgnoredDuringExecution (podset.go:104-144)
  std::optional<labelsel::RequiredAffinity> affinity;
  // PreviousAssignment of an elastic workload slice (:364-366), internal form
  std::optional<ExplicitAssignment> previousAssignment;
};
struct DomainAssignment {
  int32_t leaf;
  int32_t count;
};
// (leaf, count) pairs of one assignment: a view into the device layer's
// packed entries (valid until its next batch) or into `own`.
struct DomainSpan {
  const DomainAssignment* p = nullptr;
  size_t n = 0;
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const DomainAssignment& operator[](size_t i) const { return p[i]; }
  const DomainAssignment* begin() const { return p; }
  const DomainAssignment* end() const { return p + n; }
};
// One domain of utiltas.TopologyAssignment (tas_assignment.go:30-38):
// Values = the leaf's levelValues[levelIdx:] (buildAssignment :1472-1501
// slices the domain's own values, no string copies), Count.
struct DomainValues {
  const std::string* values;
  int32_t n;
  int32_t count;
};
struct PodSetResult {
  std::string name;
  bool has_assignment = false;
  DomainSpan domains;                  // leaf indices (lexicographic order)
  std::vector<DomainAssignment> own;   // storage once the view is materialized
  // with KUEUE_TAS_RUN_VALUES, the TopologyAssignment domains: domain k has
  // Values = values[k][0 .. levels) (the leaf's levelValues[levelIdx:]) and
  // Count = domains[k].count.  A view of the entry tags the device wrote
  // beside the entries (kueue_tas_last_entry_tags), or own_values.
  const std::string* const* values = nullptr;
  std::vector<const std::string*> own_values;
  DomainValues value(size_t k, int32_t levels) const { return {values[k], levels, domains[k].count}; }
  std::string reason;
  void materialize() {
    if (domains.n && domains.p != own.data()) {
      own.assign(domains.p, domains.p + domains.n);
      domains.p = own.data();
    }
    if (values && values != own_values.data()) {
      own_values.assign(values, values + domains.n);
      values = own_values.data();
    }
  }
};

struct Gates {  // pkg/features/kube_features.go (TASProfileMixed: Beta, default true)
  bool profileMixed = true, multiLayer = false, balanced = false, elastic = false;
};

// One findTopologyAssignment call compiled for the device.
struct GroupEval {
  bool compiled = false;
  const TASPodSetRequests* workers = nullptr;
  const TASPodSetRequests* leader = nullptr;
  std::vector<const TASPodSetRequests*> members;  // all PodSets of the group (result order)
  std::string early_reason;                        // host-side validation failure
  kueue_tas_eval_req req{};
  int32_t slice_size = 1;
  std::vector<std::string> layer_names;            // multi-layer message labels
  std::vector<int32_t> taint_row;                  // per taint profile
  // required node affinity (KUEUE_TAS_F_AFFINITY): requirements with `begin`
  // relative to aff_vals; build_pass rebases them into the batch tables
  std::vector<kueue_tas_affinity_req> aff;
  std::vector<int32_t> aff_vals;
  // nodeSelector pairs beyond the inline ones (KUEUE_TAS_F_SELECTOR_EXT), as
  // requirements relative to sel_vals, rebased the same way
  std::vector<kueue_tas_affinity_req> sel_ext;
  std::vector<int32_t> sel_vals;
  // TASBalancedPlacement applies (:907: gate on, not required, not
  // unconstrained): the host runs it over the device's phase-1 counters
  bool balanced = false;
};

struct Workload {
  std::vector<TASPodSetRequests> podsets;
  std::vector<GroupEval> groups;
};

class FlavorSnapshot {
 public:
  std::string topologyName = "default";
  mutable std::string topoQuoted, topoQuotedFor;
  const std::string& topology_quoted() const {  // strconv.Quote(topologyName), kept between failures
    if (topoQuoted.empty() || topoQuotedFor != topologyName) {
      topoQuoted = go_quote(topologyName);
      topoQuotedFor = topologyName;
    }
    return topoQuoted;
  }
  std::vector<std::string> levelKeys;
  std::vector<Toleration> flavorTolerations;
  bool lowestIsHostname = false;
  Gates gates;

  // tree (levels sorted lexicographically by levelValues)
  std::vector<std::vector<std::vector<std::string>>> values;  // [l][i]
  // values[L-1][leaf].data() per leaf: the Values views of TopologyAssignment
  // domains (one flat lookup per domain instead of a vector header each)
  mutable std::vector<const std::string*> leafVals;
  const std::string* const* leaf_values() const {
    const auto& lv = values.back();
    if (leafVals.size() != lv.size()) {
      leafVals.resize(lv.size());
      for (size_t i = 0; i < lv.size(); i++) leafVals[i] = lv[i].data();
    }
    return leafVals.data();
  }
  std::vector<std::vector<int32_t>> childOff;                 // [l][D_l + 1]
  std::vector<std::string> leafId;
  LeafIndex leafById;  // DomainID -> leaf
  std::vector<const NodeInfo*> leafNode;
  // Leaves whose last node left in place (kueue_tas_snapshot_set_leaf_live):
  // out of the snapshot until that node returns; every domain above keeps a
  // live leaf (liveUnder per leaf parent, leaf level L-2; the whole leaf
  // level for L == 1), so the tree itself never changes in place.
  std::vector<uint8_t> leafDead;
  std::vector<int32_t> leafParent, liveUnder;
  std::unordered_map<std::string, std::pair<int32_t, size_t>> leftNodes;  // node name -> (leaf, nodes[] slot)
  int32_t live_leaf(const std::string& id) const {
    const int32_t l = leafById.find(id);
    return (l < 0 || leafDead[size_t(l)]) ? -1 : l;
  }
  LeafVec<Requests> freeCap, tasUsage;
  // non-TAS pod cache mirror (tas_non_tas_pod_cache.go:30-120), kept so pod
  // events update leaves in place: allocatable sum and member nodes per leaf
  LeafVec<Requests> leafAlloc;
  std::vector<std::vector<std::string>> leafNodeNames;
  std::unordered_map<std::string, std::string> nodeToLeaf;
  std::map<std::string, std::pair<std::string, Requests>> podUsage;
  std::map<std::string, Requests> nodeUsage;
  std::vector<std::vector<int32_t>> idRank;  // [l][i]
  // columns / profiles / labels
  std::vector<std::string> cols;
  std::map<std::string, int32_t> colByName;
  // resources some request, usage record or Fits term has named: the only
  // ones CountInWithLimitingResource / Fits ever read (requests.go:174-217
  // iterate the request's keys), kept as columns even when the snapshot has
  // more resource names than KUEUE_TAS_MAX_COLS (see wanted_columns)
  std::set<std::string> reqNames;
  std::vector<std::vector<Taint>> profiles;
  std::vector<std::vector<int32_t>> profileTaintIds;  // taintIdByString[taint_string(t)] per profile taint
  std::vector<int32_t> leafProfile;
  std::vector<std::string> taintStrings;
  std::map<std::string, int32_t> taintIdByString;
  std::vector<std::string> labelKeys;
  std::map<std::string, int32_t> labelCol;
  std::vector<std::unordered_map<std::string, int32_t>> labelDict;  // value -> id (hashed: the hostname
                                                                   // column holds a value per leaf)
  std::vector<int32_t> labelValues;  // [K][labStride]: column k at k * labStride (leaves 0..N-1)
  size_t labStride = 0;              // >= N, with headroom: joined leaves shift each column in place
  std::deque<NodeInfo> nodes;  // stable addresses: leafNode points into it, nodes join in place
  std::map<std::string, std::string> flavorLabels;
  std::unordered_map<std::string, size_t> nodeIdx;  // node name -> nodes[]
  // hostname leaves by their node's name (matchFields metadata.name) and the
  // leaves whose node has no name (nodeaffinity ignores matchFields there)
  LeafIndex leafByNodeName;
  std::vector<int32_t> unnamedLeaves;

  kueue_tas_ctx* ctx = nullptr;
  bool stageTiming = true;  // kueue_tas_set_stage_timing of ctx
  bool dirty = true;
  std::string err;
  kueue_tas_config cfg{};

  ~FlavorSnapshot() {
    if (ctx) kueue_tas_ctx_destroy(ctx);
  }

  int N() const { return values.empty() ? 0 : int(values.back().size()); }
  int L() const { return int(levelKeys.size()); }

  // ---- construction (harness semantics: tas_cache_test.go:6270-6300) ----
  // The snapshot is assembled from the caches' state, which events keep
  // current: nodesCache (Ready && !Unschedulable nodes by name, first-seen
  // order; tas_nodes_cache.go:38-50), nonTasUsageCache (podUsage/nodeUsage,
  // tas_non_tas_pod_cache.go:46-120) and the TAS usage per domain
  // (TASFlavorCache.updateUsage, tas_flavor.go:154-171, plus the
  // AddUsage/RemoveUsage updates since).  A rebuild re-assembles from that
  // state: nothing is re-parsed and no event log is kept.
  // first-seen order of the cache's nodes (the tie rule where two nodes share
  // a hostname leaf); leaving nodes are tombstoned in O(1) and compacted lazily
  std::vector<std::string> nodeCacheOrder;
  std::vector<char> nodeOrderLive;
  std::unordered_map<std::string, size_t> nodeOrderPos;
  size_t nodeOrderDead = 0;
  std::unordered_map<std::string, NodeInfo> nodeCache;
  std::map<std::string, Requests> usageByDomain;

  void build(const kjson::Node& c) {
    for (auto& l : c["levels"].items) levelKeys.push_back(l.s());
    if (levelKeys.empty()) throw std::runtime_error("no topology levels");
    if (int(levelKeys.size()) > KUEUE_TAS_MAX_LEVELS) throw std::runtime_error("too many topology levels");
    lowestIsHostname = levelKeys.back() == kHostname;
    if (!c["topologyName"].null()) topologyName = c["topologyName"].s();
    for (auto& t : c["flavorTolerations"].items)
      flavorTolerations.push_back({t["key"].s(), t["operator"].s(), t["value"].s(), t["effect"].s()});
    const kjson::Node& fg = c["featureGates"];
    if (auto p = fg.find("TASProfileMixed")) gates.profileMixed = p->b();
    if (auto p = fg.find("TASMultiLayerTopology")) gates.multiLayer = p->b();
    if (auto p = fg.find("TASBalancedPlacement")) gates.balanced = p->b();
    if (auto p = fg.find("ElasticJobsViaWorkloadSlicesWithTAS")) gates.elastic = p->b();
    for (auto& kv : c["nodeLabels"].fields) flavorLabels[kv.first] = kv.second.s();
    for (auto& n : c["nodes"].items) sync_node(n);
    for (auto& u : c["tasUsage"].items) {
      std::string id;
      for (size_t k = 0; k < u["values"].items.size(); k++) id += (k ? "," : "") + u["values"].items[k].s();
      const int64_t cnt = u["count"].i64();
      Requests& dst = usageByDomain[id];
      for (auto& kv : u["singlePodRequests"].fields) dst[kv.first] = add64(dst[kv.first], mul64(kv.second.i64(), cnt));
      dst["pods"] = add64(dst["pods"], cnt);
    }
    podUsage.clear();
    nodeUsage.clear();
    for (auto& p : c["pods"].items) apply_pod(p, nullptr);
    assemble();
  }

  // nodesCache.sync (tas_nodes_cache.go:38-50): a Ready, schedulable node is
  // (re)placed under its name, any other node leaves the cache.
  static NodeInfo parse_node(const kjson::Node& n, bool* ready, bool* unschedulable) {
    NodeInfo ni;
    ni.name = n["name"].s();
    *ready = false;
    for (auto& cond : n["conditions"].items)
      if (cond["type"].s() == "Ready") {
        *ready = cond["status"].s() == "True";
        break;
      }
    *unschedulable = n["unschedulable"].b();
    for (auto& kv : n["labels"].fields) ni.labels[kv.first] = kv.second.s();
    for (auto& t : n["taints"].items) ni.taints.push_back({t["key"].s(), t["value"].s(), t["effect"].s()});
    for (auto& kv : n["allocatable"].fields) ni.allocatable[kv.first] = kv.second.i64();
    return ni;
  }
  void sync_node(const kjson::Node& n) {
    bool ready, unsched;
    NodeInfo ni = parse_node(n, &ready, &unsched);
    sync_node(std::move(ni), ready, unsched);
  }
  // the cache state's copy of an event's node (nodesCache.sync,
  // tas_nodes_cache.go:38-50), from the event's parsed form
  void sync_node(NodeInfo ni, bool ready, bool unsched) {
    auto it = nodeCache.find(ni.name);
    if (ready && !unsched) {
      if (it == nodeCache.end()) {
        nodeOrderPos[ni.name] = nodeCacheOrder.size();
        nodeCacheOrder.push_back(ni.name);
        nodeOrderLive.push_back(1);
        nodeCache.emplace(ni.name, std::move(ni));
      } else {
        it->second = std::move(ni);
      }
    } else if (it != nodeCache.end()) {
      auto p = nodeOrderPos.find(ni.name);
      nodeOrderLive[p->second] = 0;
      nodeOrderPos.erase(p);
      nodeCache.erase(it);
      if (++nodeOrderDead > 64 && 2 * nodeOrderDead > nodeCacheOrder.size()) compact_node_order();
    }
  }
  void compact_node_order() {
    size_t k = 0;
    for (size_t i = 0; i < nodeCacheOrder.size(); i++)
      if (nodeOrderLive[i]) {
        nodeOrderPos[nodeCacheOrder[i]] = k;
        if (k != i) nodeCacheOrder[k] = std::move(nodeCacheOrder[i]);
        k++;
      }
    nodeCacheOrder.resize(k);
    nodeOrderLive.assign(k, 1);
    nodeOrderDead = 0;
  }
  // A new snapshot with this one's settings and cache state (for a rebuild).
  // Usage deltas applied on the device — admissions (kueue_tas_host_admit)
  // and other ranks' delta lists (kueue_tas_host_apply_deltas) — reach the
  // host mirror (tasUsage, usageByDomain: updateTASUsage,
  // tas_flavor_snapshot.go:257-293) only when a reader needs it (an upload, a
  // column change, a node join, a rebuild): the device copy is the one
  // evaluations read.  The device keeps a shadow of the usage columns as of
  // the mirror's last sync (kueue_tas_snapshot_usage_mark); a flush asks it
  // for the (leaf, column) entries that moved since (usage_changes: one diff
  // kernel, absolute values) and sets those mirror entries.  Admission rounds
  // cost the mirror nothing, and a reader pays for the entries that changed,
  // however many rounds went by.
  bool deviceAhead = false;
  void device_applied() { deviceAhead = true; }
  // The two map entries a (column, leaf) value lives in — tasUsage[leaf][res]
  // and usageByDomain[leaf id][res] — cached by key after their first use:
  // std::map nodes never move and keys are never erased here, so an update
  // is two pointer stores instead of two string-keyed map walks.  Cleared
  // when leaves are renumbered (flush_joins) or the columns change (recolumn).
  std::vector<std::pair<int64_t*, int64_t*>> mirrorPtr;  // [R][N]
  void clear_mirror_cache() { mirrorPtr.clear(); }
  std::pair<int64_t*, int64_t*> mirror_entries(int32_t leaf, int32_t col) {
    const size_t N = size_t(this->N()), R = cols.size();
    const bool cached = N * R < (size_t(1) << 28);
    if (cached && mirrorPtr.size() != N * R) mirrorPtr.assign(N * R, {nullptr, nullptr});
    std::pair<int64_t*, int64_t*>* e = cached ? &mirrorPtr[size_t(col) * N + size_t(leaf)] : nullptr;
    if (e && e->first) return *e;
    const std::string& res = cols[size_t(col)];
    const std::pair<int64_t*, int64_t*> p{&tasUsage[size_t(leaf)][res], &usageByDomain[leafId[size_t(leaf)]][res]};
    if (e) *e = p;
    return p;
  }
  // deltas the device did not take (a stale device snapshot reloads from the
  // mirror).  The mirror first takes what the device applied since the last
  // mark: the upload's own flush would otherwise overwrite these deltas with
  // the device's absolute values, which do not hold them.
  void apply_to_mirror(const kueue_tas_delta* d, size_t n) {
    flush_mirror();
    for (size_t i = 0; i < n; i++) {
      auto e = mirror_entries(d[i].leaf, d[i].col);
      *e.first = add64(*e.first, d[i].delta);
      *e.second = add64(*e.second, d[i].delta);
    }
  }
  void flush_mirror() {
    if (!deviceAhead) return;
    deviceAhead = false;
    if (!ctx) return;
    const kueue_tas_delta* ch = nullptr;
    size_t k = 0;
    if (kueue_tas_snapshot_usage_changes(ctx, &ch, &k))
      throw std::runtime_error(std::string("host mirror sync: ") + kueue_tas_last_error(ctx));
    for (size_t i = 0; i < k; i++) {  // absolute values: the device's usage as of now
      auto e = mirror_entries(ch[i].leaf, ch[i].col);
      *e.first = ch[i].delta;
      *e.second = ch[i].delta;
    }
  }
  std::unique_ptr<FlavorSnapshot> fork_state() {
    flush_mirror();
    auto ns = std::make_unique<FlavorSnapshot>();
    ns->topologyName = topologyName;
    ns->levelKeys = levelKeys;
    ns->flavorTolerations = flavorTolerations;
    ns->lowestIsHostname = lowestIsHostname;
    ns->gates = gates;
    ns->flavorLabels = flavorLabels;
    ns->cfg = cfg;
    compact_node_order();
    ns->nodeCacheOrder = nodeCacheOrder;
    ns->nodeOrderLive = nodeOrderLive;
    ns->nodeOrderPos = nodeOrderPos;
    ns->reqNames = reqNames;
    ns->nodeCache = nodeCache;
    ns->usageByDomain = usageByDomain;
    ns->podUsage = podUsage;
    ns->nodeUsage = nodeUsage;
    return ns;
  }

  // TASFlavorCache.snapshot (tas_flavor.go:118-138) over the cache state.
  void assemble() {
    nodes.clear();
    for (size_t o = 0; o < nodeCacheOrder.size(); o++) {  // nodesCache.find: NodeMatchesFlavor (util/tas/node.go:21-33)
      if (!nodeOrderLive[o]) continue;
      const NodeInfo& ni = nodeCache.at(nodeCacheOrder[o]);
      bool match = true;
      for (auto& kv : flavorLabels) {
        auto it = ni.labels.find(kv.first);
        if ((it == ni.labels.end() ? std::string() : it->second) != kv.second) match = false;
      }
      for (auto& l : levelKeys)
        if (!ni.labels.count(l)) match = false;
      if (match) nodes.push_back(ni);
    }
    // addNode (:160-195): leaves keyed by hostname or DomainID(levelValues)
    struct LeafTmp {
      std::vector<std::string> lv;
      const NodeInfo* node;
      Requests cap;
    };
    std::vector<LeafTmp> tmp;
    std::unordered_map<std::string, int32_t> tmpById;
    nodeToLeaf.clear();
    for (auto& ni : nodes) {
      std::vector<std::string> lv;
      for (auto& k : levelKeys) {
        auto it = ni.labels.find(k);
        lv.push_back(it == ni.labels.end() ? "" : it->second);
      }
      std::string id;
      if (lowestIsHostname) {
        auto it = ni.labels.find(kHostname);
        id = it == ni.labels.end() ? "" : it->second;
      } else {
        for (size_t i = 0; i < lv.size(); i++) id += (i ? "," : "") + lv[i];
      }
      auto it = tmpById.find(id);
      if (it == tmpById.end()) {
        tmpById[id] = int32_t(tmp.size());
        tmp.push_back({lv, lowestIsHostname ? &ni : nullptr, {}});
        it = tmpById.find(id);
      }
      req_add(tmp[it->second].cap, ni.allocatable);
      nodeToLeaf[ni.name] = id;
    }
    // sort leaves by levelValues; build levels + CSR
    std::vector<int32_t> perm(tmp.size());
    for (size_t i = 0; i < perm.size(); i++) perm[i] = int32_t(i);
    std::sort(perm.begin(), perm.end(), [&](int32_t a, int32_t b) { return tmp[a].lv < tmp[b].lv; });
    const int L = this->L();
    values.assign(L, {});
    leafVals.clear();
    childOff.assign(L > 1 ? L - 1 : 0, {});
    std::vector<std::vector<std::string>> sortedLeaves;
    for (int32_t p : perm) sortedLeaves.push_back(tmp[p].lv);
    for (int l = 0; l < L; l++) {
      auto& lvl = values[l];
      for (auto& lv : sortedLeaves) {
        std::vector<std::string> pre(lv.begin(), lv.begin() + l + 1);
        if (lvl.empty() || lvl.back() != pre) lvl.push_back(std::move(pre));
      }
    }
    for (int l = 0; l + 1 < L; l++) {
      auto& off = childOff[l];
      off.assign(values[l].size() + 1, 0);
      size_t j = 0;
      for (size_t i = 0; i < values[l].size(); i++) {
        off[i] = int32_t(j);
        while (j < values[l + 1].size() &&
               std::equal(values[l][i].begin(), values[l][i].end(), values[l + 1][j].begin()))
          j++;
      }
      off[values[l].size()] = int32_t(j);
    }
    const int N = this->N();
    leafId.resize(N);
    leafNode.resize(N);
    freeCap.resize(N);
    tasUsage.resize(N);
    for (int i = 0; i < N; i++) {
      const LeafTmp& t = tmp[perm[i]];
      std::string id;
      if (lowestIsHostname) {
        auto it = t.node->labels.find(kHostname);
        id = it == t.node->labels.end() ? "" : it->second;
      } else {
        for (size_t k = 0; k < t.lv.size(); k++) id += (k ? "," : "") + t.lv[k];
      }
      leafId[i] = id;
      leafById.set(id, i);
      leafNode[i] = t.node;
      freeCap[i] = t.cap;
    }
    leafAlloc = freeCap;
    nodeIdx.clear();
    for (size_t i = 0; i < nodes.size(); i++) nodeIdx[nodes[i].name] = i;
    leafNodeNames.assign(N, {});
    for (auto& kv : nodeToLeaf) leafNodeNames[size_t(leafById.at(kv.second))].push_back(kv.first);
    leafDead.assign(size_t(N), 0);
    leftNodes.clear();
    leafParent.assign(size_t(N), 0);
    liveUnder.assign(L >= 2 ? values[size_t(L - 2)].size() : 1, 0);
    for (int i = 0; i < N; i++) {
      if (L >= 2) {
        const auto& co = childOff[size_t(L - 2)];
        leafParent[size_t(i)] = int32_t(std::upper_bound(co.begin(), co.end(), i) - co.begin()) - 1;
      }
      liveUnder[size_t(leafParent[size_t(i)])]++;
    }
    // DomainID ranks per level (multiLayerNotFitMessage tie-break)
    idRank.assign(L, {});
    for (int l = 0; l < L; l++) {
      size_t D = values[l].size();
      std::vector<std::string> ids(D);
      for (size_t i = 0; i < D; i++) {
        if (l == L - 1) {
          ids[i] = leafId[i];
        } else {
          for (size_t k = 0; k < values[l][i].size(); k++) ids[i] += (k ? "," : "") + values[l][i][k];
        }
      }
      std::vector<int32_t> ord(D);
      for (size_t i = 0; i < D; i++) ord[i] = int32_t(i);
      std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return ids[a] < ids[b]; });
      idRank[l].assign(D, 0);
      for (size_t r = 0; r < D; r++) idRank[l][ord[r]] = int32_t(r);
    }
    // TAS usage per domain (TASFlavorCache.updateUsage, tas_flavor.go:154-171): leaves only
    for (auto& kv : usageByDomain) {
      const int32_t l = leafById.find(kv.first);
      if (l >= 0) req_add(tasUsage[size_t(l)], kv.second);
    }
    // non-TAS pods (tas_non_tas_pod_cache.go:46-120)
    for (auto& kv : nodeUsage) {
      auto it = nodeToLeaf.find(kv.first);
      if (it != nodeToLeaf.end()) req_sub(freeCap[size_t(leafById.at(it->second))], kv.second);
    }
    // resource columns
    for (int i = 0; i < N; i++)
      for (auto& kv : tasUsage[i]) reqNames.insert(kv.first);  // usage of admitted workloads: requested names
    recolumn();
    // taint profiles + label dictionaries (filters apply only with hostname leaves)
    leafProfile.assign(N, 0);
    if (lowestIsHostname) {
      std::map<std::vector<Taint>, int32_t> pid;
      for (int i = 0; i < N; i++) {
        std::vector<Taint> ts;
        for (auto& t : leafNode[i]->taints)
          if (t.effect == "NoSchedule" || t.effect == "NoExecute") ts.push_back(t);
        auto it = pid.find(ts);
        if (it == pid.end()) {
          it = pid.emplace(ts, int32_t(profiles.size())).first;
          profiles.push_back(ts);
        }
        leafProfile[i] = it->second;
        for (auto& t : ts) {
          std::string s = taint_string(t);
          if (!taintIdByString.count(s)) {
            taintIdByString[s] = int32_t(taintStrings.size());
            taintStrings.push_back(s);
          }
        }
      }
      std::set<std::string> keys;
      for (int i = 0; i < N; i++)
        for (auto& kv : leafNode[i]->labels) keys.insert(kv.first);
      for (auto& k : keys) {
        labelCol[k] = int32_t(labelKeys.size());
        labelKeys.push_back(k);
      }
      labelDict.assign(labelKeys.size(), {});
      labStride = size_t(N) + size_t(N) / 8 + 64;
      labelValues.assign(labelKeys.size() * labStride, 0);
      for (size_t k = 0; k < labelKeys.size(); k++) {
        for (int i = 0; i < N; i++) {
          auto it = leafNode[i]->labels.find(labelKeys[k]);
          if (it == leafNode[i]->labels.end()) continue;
          auto& dict = labelDict[k];
          auto d = dict.find(it->second);
          if (d == dict.end()) d = dict.emplace(it->second, int32_t(dict.size()) + 1).first;
          labelValues[k * labStride + size_t(i)] = d->second;
        }
      }
    }
    if (profiles.empty()) profiles.push_back({});
    profileTaintIds.assign(profiles.size(), {});
    for (size_t p = 0; p < profiles.size(); p++)
      for (auto& t : profiles[p]) profileTaintIds[p].push_back(taintIdByString.at(taint_string(t)));
    leafByNodeName.clear();
    unnamedLeaves.clear();
    if (lowestIsHostname)
      for (int i = 0; i < N; i++) {
        if (leafNode[i]->name.empty()) unnamedLeaves.push_back(i);
        else leafByNodeName.add(leafNode[i]->name, i);
      }
  }

  // nonTasUsageCache.update (tas_non_tas_pod_cache.go:46-73): a terminated
  // pod leaves the cache, any other replaces its previous entry; per-node
  // totals gain pods:1 per pod and are dropped at pods <= 0 (removeNodeUsage
  // :101-116), keeping zero-valued keys otherwise (Requests.Sub).
  // {"delete": true} is nonTasUsageCache.delete (:76-83).
  void apply_pod(const kjson::Node& p, std::set<std::string>* touched) {
    const std::string key = p["namespace"].s() + "/" + p["name"].s();
    const std::string& phase = p["phase"].s();
    auto remove_usage = [&](const std::string& node, const Requests& u) {
      if (touched) touched->insert(node);
      auto it = nodeUsage.find(node);
      if (it == nodeUsage.end()) return;
      req_sub(it->second, u);
      it->second["pods"] = sub64(it->second["pods"], 1);
      if (it->second["pods"] <= 0) nodeUsage.erase(it);
    };
    auto old = podUsage.find(key);
    if (old != podUsage.end()) remove_usage(old->second.first, old->second.second);
    if (phase == "Succeeded" || phase == "Failed" || p["delete"].b()) {
      podUsage.erase(key);
      return;
    }
    Requests r;
    for (auto& kv : p["requests"].fields) r[kv.first] = kv.second.i64();
    const std::string& node = p["nodeName"].s();
    podUsage[key] = {node, r};
    Requests& nu = nodeUsage[node];
    req_add(nu, r);
    nu["pods"] = add64(nu["pods"], 1);
    if (touched) touched->insert(node);
  }
  // Pod events on a built snapshot: the touched leaves' freeCapacity is
  // recomputed as allocatable - Σ non-TAS usage of their nodes
  // (TASFlavorCache.snapshot :124-137) and replaced on the device; a resource
  // with no column yet re-columns (the next evaluation reloads).
  int update_pods(const kjson::Node& arr) {
    std::set<std::string> touched;
    for (auto& p : arr.items) apply_pod(p, &touched);
    std::set<int32_t> leaves;
    for (auto& n : touched) {
      auto it = nodeToLeaf.find(n);
      if (it != nodeToLeaf.end()) leaves.insert(leafById.at(it->second));
    }
    return push_leaves(leaves, false);
  }

  // ---- node events (nodesCache.sync, tas_nodes_cache.go:38-72) ----
  // Applied in place:
  //  * an update of a node in the snapshot that keeps it a member (Ready,
  //    schedulable, matching the flavor, every level label) at the same
  //    topology position: leaf attributes only — allocatable (freeCapacity, addCapacity :243-248), taint profile,
  //    selector label columns;
  //  * a node leaving the snapshot (NotReady, cordoned, no longer matching):
  //    its leaf loses its capacity, or, as its last node, leaves the snapshot
  //    (kueue_tas_snapshot_set_leaf_live) while its parent keeps a live leaf;
  //  * such a node returning to the same position (the leaf comes back);
  //  * an event for a node that is not and stays not in the snapshot;
  //  * a new node, or a member moving to another position: it joins in place
  //    (add_node splices its leaf into the tree);
  //  * a new taint profile or label value: registered, the compiled
  //    requests recompile.
  // A domain losing its last leaf, a node under a hostname another node
  // shares, or a second node joining an existing hostname returns false: the
  // caller rebuilds the snapshot, as the reference does every cycle.
  bool member_of(const NodeInfo& ni, bool ready, bool unsched) const {  // nodesCache.find (util/tas/node.go:21-33)
    if (!ready || unsched) return false;
    for (auto& kv : flavorLabels) {
      auto it = ni.labels.find(kv.first);
      if ((it == ni.labels.end() ? std::string() : it->second) != kv.second) return false;
    }
    for (auto& l : levelKeys)
      if (!ni.labels.count(l)) return false;
    return true;
  }
  // The taint profile of `ni`, its taint strings and its label keys / values
  // registered (appended) when new.  *changed: compiled requests are stale
  // (taint rows hold one entry per profile, selectors and affinity hold label
  // value ids); *relayout: a new label column (the device arrays reload).
  int32_t register_attrs(const NodeInfo& ni, bool* changed, bool* relayout) {
    if (!lowestIsHostname) return 0;
    std::vector<Taint> ts;
    for (auto& t : ni.taints)
      if (t.effect == "NoSchedule" || t.effect == "NoExecute") ts.push_back(t);
    int32_t prof;
    auto pit = std::find(profiles.begin(), profiles.end(), ts);
    if (pit == profiles.end()) {
      prof = int32_t(profiles.size());
      profiles.push_back(ts);
      std::vector<int32_t> ids;
      for (auto& t : ts) {
        const std::string s = taint_string(t);
        auto it = taintIdByString.find(s);
        if (it == taintIdByString.end()) {
          it = taintIdByString.emplace(s, int32_t(taintStrings.size())).first;
          taintStrings.push_back(s);
        }
        ids.push_back(it->second);
      }
      profileTaintIds.push_back(std::move(ids));
      *changed = true;
    } else {
      prof = int32_t(pit - profiles.begin());
    }
    for (auto& kv : ni.labels) {
      auto c = labelCol.find(kv.first);
      if (c == labelCol.end()) {  // a new label column, absent on every other leaf
        c = labelCol.emplace(kv.first, int32_t(labelKeys.size())).first;
        labelKeys.push_back(kv.first);
        labelDict.emplace_back();
        labelValues.resize(labelKeys.size() * labStride, 0);
        *changed = *relayout = true;
      }
      auto& dict = labelDict[size_t(c->second)];
      if (!dict.count(kv.second)) {
        dict.emplace(kv.second, int32_t(dict.size()) + 1);
        *changed = true;
      }
    }
    return prof;
  }
  // Compiled requests and host results refer to this layout (leaf indices,
  // profiles, label ids): a new generation makes the host recompile.
  void new_layout() {
    col_gen = next_gen();
    compile_gen++;
  }
  bool spliced = false;  // a node joined at a new topology position since the host last looked
  void set_attrs(NodeInfo& cur, NodeInfo&& ni, int32_t leaf, int32_t prof) {
    nodeCache[ni.name] = ni;
    cur.labels = std::move(ni.labels);
    cur.taints = std::move(ni.taints);
    cur.allocatable = std::move(ni.allocatable);
    leafProfile[size_t(leaf)] = prof;
    if (lowestIsHostname) {
      for (size_t k = 0; k < labelKeys.size(); k++) {
        auto it = cur.labels.find(labelKeys[k]);
        labelValues[k * labStride + size_t(leaf)] = it == cur.labels.end() ? 0 : labelDict[k].at(it->second);
      }
    }
  }
  void realloc_leaf(int32_t leaf) {
    Requests alloc;
    for (auto& nm : leafNodeNames[size_t(leaf)]) req_add(alloc, nodes[nodeIdx.at(nm)].allocatable);
    leafAlloc[size_t(leaf)] = std::move(alloc);
  }
  // `ni`, `ready`, `unsched`: the event's node as parse_node reads it (the
  // batch's events are parsed on the host pool first)
  bool node_event_in_place(NodeInfo&& ni, bool ready, bool unsched, std::set<int32_t>* touched,
                           std::set<int32_t>* liveChanged) {
    const bool member = member_of(ni, ready, unsched);
    const int L = this->L();
    auto ix = nodeIdx.find(ni.name);
    if (!joins.empty() && (ix != nodeIdx.end() || member)) {  // reads the tree: pending joins merge first
      bool join = ix == nodeIdx.end() && !leftNodes.count(ni.name);
      if (join) {
        const std::string id = lowestIsHostname ? ni.labels.at(kHostname) : [&] {
          std::string s;
          for (size_t k = 0; k < levelKeys.size(); k++) s += (k ? "," : "") + ni.labels.at(levelKeys[k]);
          return s;
        }();
        join = !joinIds.count(id) && !leafById.count(id);
      }
      if (!join) flush_joins(touched, liveChanged);
    }
    if (ix == nodeIdx.end()) {
      if (!member) {  // not in the snapshot before or after
        sync_node(std::move(ni), ready, unsched);
        return true;
      }
      auto left = leftNodes.find(ni.name);
      if (left == leftNodes.end()) return add_node(std::move(ni), touched, liveChanged);  // a new node
      const int32_t leaf = left->second.first;
      const size_t slot = left->second.second;
      std::vector<std::string> lv;
      for (auto& k : levelKeys) lv.push_back(ni.labels.at(k));
      if (lv != values[size_t(L - 1)][size_t(leaf)] ||
          (lowestIsHostname && ni.labels.at(kHostname) != leafId[size_t(leaf)])) {  // back at another position
        leftNodes.erase(left);
        return add_node(std::move(ni), touched, liveChanged);
      }
      bool changed = false, relayout = false;
      const int32_t prof = register_attrs(ni, &changed, &relayout);
      if (changed) new_layout();
      if (relayout) dirty = true;
      // back in: the node's slot, its leaf (alive again when it was its last node)
      sync_node(ni, true, false);
      nodeIdx[ni.name] = slot;
      nodeToLeaf[ni.name] = leafId[size_t(leaf)];
      leafNodeNames[size_t(leaf)].push_back(ni.name);
      leftNodes.erase(left);
      set_attrs(nodes[slot], std::move(ni), leaf, prof);
      if (leafDead[size_t(leaf)]) {
        leafDead[size_t(leaf)] = 0;
        liveUnder[size_t(leafParent[size_t(leaf)])]++;
        liveChanged->insert(leaf);
      }
      realloc_leaf(leaf);
      touched->insert(leaf);
      return true;
    }
    NodeInfo& cur = nodes[ix->second];
    const int32_t leaf = leafById.at(nodeToLeaf.at(ni.name));
    // a hostname shared by two nodes: the leaf's taints and labels are the
    // first node's in cache order (leafDomain.node, tas_flavor_snapshot.go:
    // 160-195); an event on that node is rebuilt, one on any later node
    // touches the leaf's capacity only
    if (lowestIsHostname && leafNodeNames[size_t(leaf)].size() > 1) {
      if (leafNode[size_t(leaf)] == &cur) return false;
      return later_host_node_event(std::move(ni), member, ix, leaf, ready, unsched, touched, liveChanged);
    }
    bool moved = false;  // a member at another topology position: leaves, then joins there
    for (auto& l : levelKeys) {
      auto a = ni.labels.find(l), b = cur.labels.find(l);
      moved = moved || a == ni.labels.end() || b == cur.labels.end() || a->second != b->second;
    }
    if (!member || moved) {  // leaves the snapshot
      auto& names = leafNodeNames[size_t(leaf)];
      if (names.size() == 1) {
        if (liveUnder[size_t(leafParent[size_t(leaf)])] <= 1) return false;  // its domain would vanish
        leafDead[size_t(leaf)] = 1;
        liveUnder[size_t(leafParent[size_t(leaf)])]--;
        liveChanged->insert(leaf);
      }
      names.erase(std::find(names.begin(), names.end(), ni.name));
      leftNodes[ni.name] = {leaf, ix->second};
      nodeToLeaf.erase(ni.name);
      nodeIdx.erase(ix);
      if (!moved) {
        sync_node(std::move(ni), ready, unsched);
        realloc_leaf(leaf);
        touched->insert(leaf);
        return true;
      }
      sync_node(ni, ready, unsched);
      realloc_leaf(leaf);
      touched->insert(leaf);
      leftNodes.erase(ni.name);
      return add_node(std::move(ni), touched, liveChanged);
    }
    bool changed = false, relayout = false;
    const int32_t prof = register_attrs(ni, &changed, &relayout);
    if (changed) new_layout();
    if (relayout) dirty = true;
    sync_node(ni, true, false);
    set_attrs(cur, std::move(ni), leaf, prof);
    realloc_leaf(leaf);
    touched->insert(leaf);
    return true;
  }
  // A member node that is not in the snapshot joins it (nodesCache.sync,
  // tas_nodes_cache.go:38-50, then addNode / initialize, :160-241).  Into an
  // existing aggregated leaf (the lowest level is not hostname: addCapacity
  // :243-248) it only adds capacity; otherwise its leaf — and any missing
  // ancestor — joins the tree at its lexicographic position (queued, merged
  // by flush_joins): the new leaf's capacity is allocatable - its non-TAS
  // usage and its TAS usage the cache's for its DomainID (tas_flavor.go:
  // 118-171), exactly what a rebuild from the cache state would assemble.
  // The device arrays reload (one upload); compiled requests recompile
  // (new_layout).  false (rebuild) only for a second node under an existing
  // hostname (leafDomain.node is the first one, :165-191).
  bool add_node(NodeInfo&& ni, std::set<int32_t>* touched, std::set<int32_t>* liveChanged) {  // a member: ready, schedulable
    const int L = this->L();
    std::vector<std::string> lv;
    for (auto& k : levelKeys) lv.push_back(ni.labels.at(k));
    std::string id;
    if (lowestIsHostname) id = ni.labels.at(kHostname);
    else
      for (size_t k = 0; k < lv.size(); k++) id += (k ? "," : "") + lv[k];
    if (const int32_t leaf = leafById.find(id); leaf >= 0) {
      if (lowestIsHostname) {
        // another node under a leaf's hostname: addNode finds the leaf and
        // only adds capacity (tas_flavor_snapshot.go:160-195) when the leaf's
        // node stays the first in cache order — the joining node is appended
        // to the cache unless it was there already (a non-member becoming
        // one); a dead leaf would take this node's attributes: both rebuilt
        if (leafDead[size_t(leaf)] || leafNodeNames[size_t(leaf)].empty()) return false;
        auto mine = nodeOrderPos.find(ni.name);
        if (mine != nodeOrderPos.end() && mine->second < nodeOrderPos.at(leafNode[size_t(leaf)]->name)) return false;
      } else if (values[size_t(L - 1)][size_t(leaf)] != lv) {
        return false;
      }
      sync_node(ni, true, false);  // another node of the leaf
      nodes.push_back(std::move(ni));
      const NodeInfo& nd = nodes.back();
      nodeIdx[nd.name] = nodes.size() - 1;
      nodeToLeaf[nd.name] = id;
      leafNodeNames[size_t(leaf)].push_back(nd.name);
      if (leafDead[size_t(leaf)]) {
        leafDead[size_t(leaf)] = 0;
        liveUnder[size_t(leafParent[size_t(leaf)])]++;
        liveChanged->insert(leaf);
      }
      realloc_leaf(leaf);
      touched->insert(leaf);
      return true;
    }
    bool changed = false, relayout = false;
    const int32_t prof = register_attrs(ni, &changed, &relayout);
    sync_node(ni, true, false);
    nodes.push_back(std::move(ni));
    const NodeInfo& nd = nodes.back();
    nodeIdx[nd.name] = nodes.size() - 1;
    nodeToLeaf[nd.name] = id;
    joinIds.insert(id);
    joins.push_back({&nd, std::move(id), std::move(lv), prof});
    (void)touched;
    (void)liveChanged;
    return true;
  }
  // An event on a node of a hostname leaf that is not the leaf's first node
  // (a capacity-only member, add_node): it stays (allocatable, labels and
  // taints of its own, which the leaf does not read), or leaves the leaf —
  // and joins another hostname's leaf if it is still a member.
  bool later_host_node_event(NodeInfo&& ni, bool member, std::unordered_map<std::string, size_t>::iterator ix,
                             int32_t leaf, bool ready, bool unsched, std::set<int32_t>* touched,
                             std::set<int32_t>* liveChanged) {
    NodeInfo& cur = nodes[ix->second];
    const bool renamed = ni.labels.at(kHostname) != leafId[size_t(leaf)];
    if (member && !renamed) {
      sync_node(ni, true, false);
      nodeCache[ni.name] = ni;
      cur.labels = std::move(ni.labels);
      cur.taints = std::move(ni.taints);
      cur.allocatable = std::move(ni.allocatable);
      realloc_leaf(leaf);
      touched->insert(leaf);
      return true;
    }
    auto& names = leafNodeNames[size_t(leaf)];
    names.erase(std::find(names.begin(), names.end(), ni.name));
    nodeToLeaf.erase(ni.name);
    nodeIdx.erase(ix);
    realloc_leaf(leaf);
    touched->insert(leaf);
    if (!member) {
      sync_node(std::move(ni), ready, unsched);
      return true;
    }
    return add_node(std::move(ni), touched, liveChanged);
  }
  // Nodes joining at new topology positions, merged into the tree together
  // (flush_joins) — before the next event that reads the tree, and at the
  // end of the batch.
  struct Join {
    const NodeInfo* node;
    std::string id;
    std::vector<std::string> lv;
    int32_t prof;
  };
  std::vector<Join> joins;
  std::unordered_set<std::string> joinIds;
  std::string domain_id(int l, size_t i) const {  // utiltas.DomainID (util/tas/tas.go:29-31)
    if (l == L() - 1) return leafId[i];
    std::string s;
    for (size_t k = 0; k < values[size_t(l)][i].size(); k++) s += (k ? "," : "") + values[size_t(l)][i][k];
    return s;
  }
  // One merge of the pending joins: every level gains its missing prefixes at
  // their lexicographic positions (binary searches, O(K log D) comparisons),
  // and the level arrays, CSR offsets, DomainID ranks and every leaf-indexed
  // array move to the new indices in one O(D) pass — what a rebuild from the
  // cache state would assemble (tas_flavor.go:118-171), without re-sorting
  // or re-reading a node.  Leaf sets the batch's earlier events recorded move
  // with the leaves.
  double flush_ms[4] = {0, 0, 0, 0};  // last flush_joins: host-mirror fold, levels + CSR, leaf arrays, maps + ranks
  void flush_joins(std::set<int32_t>* touched, std::set<int32_t>* liveChanged) {
    for (double& x : flush_ms) x = 0;
    if (joins.empty()) return;
    double tf = now_ms();
    auto lap = [&](int k) {
      const double t = now_ms();
      flush_ms[k] = t - tf;
      tf = t;
    };
    flush_mirror();  // tasUsage rows move
    clear_mirror_cache();
    lap(0);
    const int L = this->L();
    std::sort(joins.begin(), joins.end(), [](const Join& a, const Join& b) { return a.lv < b.lv; });
    std::vector<std::vector<int32_t>> remap(static_cast<size_t>(L)), fresh(static_cast<size_t>(L));  // [l][old] -> new; [l] inserted
    std::vector<size_t> pos(joins.size());
    std::vector<uint8_t> found(joins.size());
    std::vector<std::vector<std::vector<std::string>>> adds(static_cast<size_t>(L));  // [l] the level's new prefixes
    for (int l = 0; l < L; l++) {
      auto& lvl = values[size_t(l)];
      // each join's prefix searched in the (unchanged) level on the pool,
      // then the new prefixes collected in order, repeats dropped
      auto prefix_less = [l](const std::vector<std::string>& v, const std::vector<std::string>& jl) {
        return std::lexicographical_compare(v.begin(), v.end(), jl.begin(), jl.begin() + l + 1);
      };
      ktas_pool::HostPool::get().run(joins.size(), 8, [&](size_t b, size_t e) {
        for (size_t k = b; k < e; k++) {
          const auto& jl = joins[k].lv;
          auto it = std::lower_bound(lvl.begin(), lvl.end(), jl, prefix_less);
          pos[k] = size_t(it - lvl.begin());
          found[k] = it != lvl.end() && std::equal(it->begin(), it->end(), jl.begin(), jl.begin() + l + 1);
        }
      });
      auto& add = adds[size_t(l)];
      std::vector<size_t> at;
      for (size_t k = 0; k < joins.size(); k++) {
        const auto& jl = joins[k].lv;
        if (found[k]) continue;
        if (!add.empty() && std::equal(add.back().begin(), add.back().end(), jl.begin(), jl.begin() + l + 1)) continue;
        at.push_back(pos[k]);
        add.emplace_back(jl.begin(), jl.begin() + l + 1);
      }
      // every old domain moves right by the number of prefixes inserted
      // before it (the moves themselves run on the pool, move_level below)
      const size_t D0 = lvl.size();
      auto& rm = remap[size_t(l)];
      rm.resize(D0);
      auto& fr = fresh[size_t(l)];
      for (size_t a = 0, i = 0; i < D0; i++) {
        while (a < add.size() && at[a] == i) a++;
        rm[i] = int32_t(i + a);
      }
      for (size_t a = 0; a < add.size(); a++) fr.push_back(int32_t(at[a] + a));
    }
    // a level grows in place (from the back, so no slot is overwritten before
    // it moved; a moved vector keeps its buffer, so the leaves' Values
    // addresses survive the move)
    auto move_level = [&](int l) {
      auto& lvl = values[size_t(l)];
      const auto& lrm = remap[size_t(l)];
      const auto& lfr = fresh[size_t(l)];
      auto& add = adds[size_t(l)];
      if (add.empty()) return;
      const size_t D0 = lvl.size();
      lvl.resize(D0 + add.size());
      for (size_t i = D0; i-- > 0;)
        if (size_t(lrm[i]) != i) lvl[size_t(lrm[i])] = std::move(lvl[i]);
      for (size_t a = 0; a < add.size(); a++) lvl[size_t(lfr[a])] = std::move(add[a]);
    };
    lap(1);
    // leaf-indexed arrays (joins are in leaf order: fresh[L-1][k] is joins[k]'s leaf)
    const auto& rm = remap[size_t(L - 1)];
    const auto& fr = fresh[size_t(L - 1)];
    const size_t N0 = rm.size(), N = N0 + fr.size();
    // every leaf-indexed array grows in place the same way (from the back),
    // the arrays on the host pool's workers at once
    auto move_leaves = [&](auto& vec, auto make) {
      vec.resize(N);
      for (size_t i = N0; i-- > 0;)
        if (size_t(rm[i]) != i) vec[size_t(rm[i])] = std::move(vec[i]);
      for (size_t k = 0; k < fr.size(); k++) vec[size_t(fr[k])] = make(joins[k]);
    };
    auto move_boxed = [&](LeafVec<Requests>& vec, auto make) {
      move_leaves(vec.v, [&](const Join& j) { return std::make_unique<Requests>(make(j)); });
    };
    std::vector<std::function<void()>> tasks;
    for (int l = L; l-- > 0;) tasks.emplace_back([&, l] { move_level(l); });  // the leaf level first: the longest
    tasks.emplace_back([&] { move_leaves(leafId, [](const Join& j) { return j.id; }); });
    tasks.emplace_back([&] { move_leaves(leafNode, [](const Join& j) { return j.node; }); });
    tasks.emplace_back([&] { move_boxed(leafAlloc, [](const Join& j) { return j.node->allocatable; }); });
    tasks.emplace_back([&] {
      move_boxed(freeCap, [&](const Join& j) {
        Requests f = j.node->allocatable;
        if (auto u = nodeUsage.find(j.node->name); u != nodeUsage.end()) req_sub(f, u->second);
        return f;
      });
    });
    tasks.emplace_back([&] {
      move_boxed(tasUsage, [&](const Join& j) {
        auto u = usageByDomain.find(j.id);
        return u == usageByDomain.end() ? Requests() : u->second;
      });
    });
    tasks.emplace_back([&] { move_leaves(leafNodeNames, [](const Join& j) { return std::vector<std::string>{j.node->name}; }); });
    tasks.emplace_back([&] {
      move_leaves(leafDead, [](const Join&) { return uint8_t(0); });
      move_leaves(leafProfile, [](const Join& j) { return j.prof; });
    });
    if (!labelKeys.empty()) {  // each label column shifts in place (its stride has room), one task per column
      const size_t K = labelKeys.size();
      if (N > labStride) {  // out of room: every column moves to a wider stride first
        const size_t ns = N + N / 8 + 64;
        std::vector<int32_t> wide(K * ns, 0);
        for (size_t k = 0; k < K; k++) memcpy(wide.data() + k * ns, labelValues.data() + k * labStride, N0 * 4);
        labelValues.swap(wide);
        labStride = ns;
      }
      for (size_t k = 0; k < K; k++)
        tasks.emplace_back([&, k] {
          int32_t* col = labelValues.data() + k * labStride;
          for (size_t i = N0; i-- > 0;)
            if (size_t(rm[i]) != i) col[size_t(rm[i])] = col[i];
          for (size_t j = 0; j < fr.size(); j++) {
            auto it = joins[j].node->labels.find(labelKeys[k]);
            col[size_t(fr[j])] = it == joins[j].node->labels.end() ? 0 : labelDict[k].at(it->second);
          }
        });
    }
    ktas_pool::HostPool::get().run(tasks.size(), 1, [&](size_t b, size_t e) {
      for (size_t t = b; t < e; t++) tasks[t]();
    });
    // CSR offsets: children per (new) parent, then a prefix sum
    for (int l = 0; l + 1 < L; l++) {
      auto& off = childOff[size_t(l)];
      const auto& up = values[size_t(l)];
      std::vector<int32_t> cnt(up.size(), 0);
      for (size_t p = 0; p + 1 < off.size(); p++) cnt[size_t(remap[size_t(l)][p])] = off[p + 1] - off[p];
      for (int32_t c : fresh[size_t(l + 1)]) {
        const auto& v = values[size_t(l + 1)][size_t(c)];
        const std::vector<std::string> pre(v.begin(), v.begin() + l + 1);
        cnt[size_t(std::lower_bound(up.begin(), up.end(), pre) - up.begin())]++;
      }
      off.assign(up.size() + 1, 0);
      for (size_t p = 0; p < up.size(); p++) off[p + 1] = off[p] + cnt[p];
    }
    lap(2);
    // then, on the pool again: the leaf-index maps, the leaves' parents and
    // live counts, and each level's DomainID ranks
    std::vector<std::function<void()>> tasks2;
    tasks2.emplace_back([&] {  // leaf indices held in maps: remapped in place (no re-hashing), then the joins added
      leafById.remap(rm);
      for (size_t k = 0; k < fr.size(); k++) leafById.set(joins[k].id, fr[k]);
      for (auto& kv : leftNodes) kv.second.first = rm[size_t(kv.second.first)];
    });
    if (lowestIsHostname)
      tasks2.emplace_back([&] {
        leafByNodeName.remap(rm);
        for (auto& u : unnamedLeaves) u = rm[size_t(u)];
        for (size_t k = 0; k < fr.size(); k++) {
          if (joins[k].node->name.empty()) unnamedLeaves.push_back(fr[k]);
          else leafByNodeName.add(joins[k].node->name, fr[k]);
        }
        std::sort(unnamedLeaves.begin(), unnamedLeaves.end());
      });
    // leaf parents and live leaves per parent, in chunks of parents
    const std::vector<int32_t>* pco = L >= 2 ? &childOff[size_t(L - 2)] : nullptr;
    leafParent.resize(N);
    liveUnder.assign(L >= 2 ? values[size_t(L - 2)].size() : 1, 0);
    if (!pco) {
      for (size_t i = 0; i < N; i++) {
        leafParent[i] = 0;
        if (!leafDead[i]) liveUnder[0]++;
      }
    }
    constexpr size_t kChunk = 8192;
    const size_t P = pco ? pco->size() - 1 : 0;
    for (size_t p0 = 0; p0 < P; p0 += kChunk / 16)
      tasks2.emplace_back([&, p0] {
        const auto& co = *pco;
        for (size_t p = p0; p < std::min(P, p0 + kChunk / 16); p++) {
          int32_t live = 0;
          for (int32_t i = co[p]; i < co[p + 1]; i++) {
            leafParent[size_t(i)] = int32_t(p);
            live += leafDead[size_t(i)] ? 0 : 1;
          }
          liveUnder[p] = live;
        }
      });
    // DomainID ranks (multiLayerNotFitMessage tie-break): each new id's
    // position among the old ones by a binary search over the old rank order;
    // an old domain's rank grows by the new ids placed before it.  The O(D)
    // passes (old rank order, new ranks) run in chunks.
    std::vector<std::vector<int32_t>> byRank(static_cast<size_t>(L)), newRank(static_cast<size_t>(L));
    for (int l = 0; l < L; l++) {
      if (fresh[size_t(l)].empty()) continue;
      const size_t D0 = idRank[size_t(l)].size();
      byRank[size_t(l)].resize(D0);
      for (size_t c0 = 0; c0 < D0; c0 += kChunk)
        tasks2.emplace_back([&, l, c0] {
          const auto& rk = idRank[size_t(l)];
          const auto& rml = remap[size_t(l)];
          auto& br = byRank[size_t(l)];
          for (size_t i = c0; i < std::min(rk.size(), c0 + kChunk); i++) br[size_t(rk[i])] = rml[i];  // new indices in old rank order
        });
    }
    ktas_pool::HostPool::get().run(tasks2.size(), 1, [&](size_t b, size_t e) {
      for (size_t t = b; t < e; t++) tasks2[t]();
    });
    std::vector<std::function<void()>> tasks3;
    std::vector<std::vector<int32_t>> qpos(static_cast<size_t>(L));
    std::vector<std::vector<std::pair<std::string, int32_t>>> newIds(static_cast<size_t>(L));
    for (int l = 0; l < L; l++) {
      const auto& f = fresh[size_t(l)];
      if (f.empty()) continue;
      const auto& br = byRank[size_t(l)];
      const size_t D0 = br.size();
      auto& ids = newIds[size_t(l)];
      for (int32_t c : f) ids.emplace_back(domain_id(l, size_t(c)), c);
      std::sort(ids.begin(), ids.end());
      auto& q = qpos[size_t(l)];
      q.resize(ids.size());
      for (size_t k = 0; k < ids.size(); k++) {
        size_t lo = 0, hi = D0;
        while (lo < hi) {
          const size_t mid = (lo + hi) / 2;
          if (domain_id(l, size_t(br[mid])) < ids[k].first) lo = mid + 1;
          else hi = mid;
        }
        q[k] = int32_t(lo);
      }
      auto& out = newRank[size_t(l)];
      out.resize(D0 + ids.size());
      for (size_t j = 0; j < ids.size(); j++) out[size_t(ids[j].second)] = q[j] + int32_t(j);
      for (size_t c0 = 0; c0 < D0; c0 += kChunk)
        tasks3.emplace_back([&, l, c0] {
          const auto& brl = byRank[size_t(l)];
          const auto& ql = qpos[size_t(l)];
          auto& o = newRank[size_t(l)];
          const size_t e = std::min(brl.size(), c0 + kChunk);
          size_t k = size_t(std::upper_bound(ql.begin(), ql.end(), int32_t(c0)) - ql.begin());
          for (size_t r = c0; r < e; r++) {
            while (k < ql.size() && size_t(ql[k]) <= r) k++;
            o[size_t(brl[r])] = int32_t(r + k);
          }
        });
    }
    ktas_pool::HostPool::get().run(tasks3.size(), 1, [&](size_t b, size_t e) {
      for (size_t t = b; t < e; t++) tasks3[t]();
    });
    for (int l = 0; l < L; l++)
      if (!fresh[size_t(l)].empty()) idRank[size_t(l)] = std::move(newRank[size_t(l)]);
    lap(3);
    leafVals.clear();
    for (auto& j : joins)
      for (auto& kv : j.node->allocatable)
        if (!colByName.count(kv.first)) {
          recolumn();
          break;
        }
    for (std::set<int32_t>* set : {touched, liveChanged}) {
      std::set<int32_t> moved;
      for (int32_t l : *set) moved.insert(rm[size_t(l)]);
      *set = std::move(moved);
    }
    // the device follows by a splice (its leaf columns gathered into the new
    // numbering, the joined rows uploaded with it) unless a reload is due anyway
    if (!dirty && ctx) {
      if (!splicePending) {
        spliceSrc.resize(N0);
        for (size_t i = 0; i < N0; i++) spliceSrc[i] = int32_t(i);
      }
      std::vector<int32_t> src(N, -1);
      for (size_t i = 0; i < N0; i++) src[size_t(rm[i])] = spliceSrc[i];
      spliceSrc = std::move(src);
      splicePending = true;
    } else {
      dirty = true;
      touched->insert(fr.begin(), fr.end());
    }
    joins.clear();
    joinIds.clear();
    new_layout();
    spliced = true;
  }
  // kueue_tas_snapshot_splice of the pending joins: the tree and the joined
  // leaves' rows from the host mirror; every other leaf's row stays on the device
  bool splicePending = false;
  std::vector<int32_t> spliceSrc;  // per current leaf: its index on the device, -1 joined since
  bool namesStale = false;         // domain names to reload before a v1beta2 encode
  double splice_ms[3] = {0, 0, 0};  // last splice: host rows, kueue_tas_snapshot_splice, leaf tags
  int upload_splice() {
    splicePending = false;
    const double t0 = now_ms();
    const int L = this->L(), N = this->N(), R = int(cols.size());
    std::vector<int32_t> sizes(L), co, ranks;
    for (int l = 0; l < L; l++) sizes[l] = int32_t(values[l].size());
    for (int l = 0; l + 1 < L; l++) co.insert(co.end(), childOff[l].begin(), childOff[l].end());
    for (int l = 0; l < L; l++) ranks.insert(ranks.end(), idRank[l].begin(), idRank[l].end());
    std::vector<int32_t> fresh;
    for (int j = 0; j < N; j++)
      if (spliceSrc[size_t(j)] < 0) fresh.push_back(j);
    const size_t k = fresh.size(), K = labelKeys.size();
    std::vector<int64_t> fr(size_t(R) * k, 0), us(size_t(R) * k, 0);
    std::vector<uint32_t> fp(k, 0), up(k, 0);
    std::vector<int32_t> prof(k, 0), lab(K * k, 0);
    for (size_t q = 0; q < k; q++) {
      const size_t j = size_t(fresh[q]);
      for (auto& kv : freeCap[j]) {
        const auto c = colByName.find(kv.first);
        if (c == colByName.end()) continue;
        fr[size_t(c->second) * k + q] = kv.second;
        fp[q] |= 1u << c->second;
      }
      for (auto& kv : tasUsage[j]) {
        const auto c = colByName.find(kv.first);
        if (c == colByName.end()) continue;
        us[size_t(c->second) * k + q] = kv.second;
        up[q] |= 1u << c->second;
      }
      prof[q] = leafProfile[j];
      for (size_t c = 0; c < K; c++) lab[c * k + q] = labelValues[c * labStride + j];
    }
    kueue_tas_snapshot_desc d{};
    d.num_levels = L;
    d.level_sizes = sizes.data();
    d.child_offsets = co.data();
    d.num_cols = R;
    d.lowest_is_hostname = lowestIsHostname ? 1 : 0;
    d.num_label_cols = int32_t(K);
    d.domain_id_rank = ranks.data();
    kueue_tas_splice_desc sd{};
    sd.topo = &d;
    sd.leaf_src = spliceSrc.data();
    sd.num_new = int32_t(k);
    sd.new_free_capacity = fr.data();
    sd.new_tas_usage = us.data();
    sd.new_free_present = fp.data();
    sd.new_usage_present = up.data();
    sd.new_taint_profile = lowestIsHostname ? prof.data() : nullptr;
    sd.new_label_values = K ? lab.data() : nullptr;
    // with leaf tags on the device, the resident leaves' tags move with them
    // (a moved Values vector keeps its buffer): only the joined leaves' go up
    std::vector<uint64_t> ntags;
    if (tagsSet && !(cfg.flags & KUEUE_TAS_CFG_HOST_VALUES)) {
      const int32_t lvl = lowestIsHostname ? L - 1 : 0;
      const std::string* const* lv = leaf_values();
      for (size_t q = 0; q < k; q++) ntags.push_back(uint64_t(reinterpret_cast<uintptr_t>(lv[size_t(fresh[q])] + lvl)));
      sd.new_leaf_tags = ntags.data();
    }
    const double t1 = now_ms();
    int rc = kueue_tas_snapshot_splice(ctx, &sd);
    spliceSrc.clear();
    if (!rc) rc = kueue_tas_snapshot_usage_mark(ctx);  // device usage == host mirror
    if (rc) {
      err = std::string("snapshot splice: ") + kueue_tas_last_error(ctx);
      return rc;
    }
    namesStale = true;
    const double t2 = now_ms();
    if (!sd.new_leaf_tags) rc = set_tags();
    splice_ms[0] = t1 - t0;
    splice_ms[1] = t2 - t1;
    splice_ms[2] = now_ms() - t2;
    return rc;
  }
  bool tagsSet = false;  // the device holds every leaf's tag (set_tags since the last load)
  int set_tags() {  // entry tags: each leaf's Values address (Values come back with the entries)
    tagsSet = false;
    if (cfg.flags & KUEUE_TAS_CFG_HOST_VALUES) return 0;
    const int L = this->L(), N = this->N();
    const int32_t lvl = lowestIsHostname ? L - 1 : 0;
    const std::string* const* lv = leaf_values();
    std::vector<uint64_t> tags(size_t(N), 0);
    for (int i = 0; i < N; i++) tags[size_t(i)] = uint64_t(reinterpret_cast<uintptr_t>(lv[i] + lvl));
    const int rc = kueue_tas_snapshot_set_leaf_tags(ctx, tags.data(), tags.size());
    if (rc) err = std::string("leaf tags: ") + kueue_tas_last_error(ctx);
    tagsSet = rc == 0;
    return rc;
  }
  int load_names() {  // own label value of every domain, for the v1beta2 encoder's leaf mode
    std::string names;
    std::vector<int64_t> name_off(1, 0);
    for (int l = 0; l < L(); l++)
      for (auto& v : values[size_t(l)]) {
        names += v.back();
        name_off.push_back(int64_t(names.size()));
      }
    const int rc = kueue_tas_snapshot_load_names(ctx, names.data(), names.size(), name_off.data());
    if (rc) err = std::string("snapshot names: ") + kueue_tas_last_error(ctx);
    namesStale = rc != 0;
    return rc;
  }
  int push_liveness(const std::set<int32_t>& leaves) {
    if (dirty || !ctx || leaves.empty()) return 0;  // a reload applies leafDead itself
    std::vector<int32_t> ls(leaves.begin(), leaves.end()), live(ls.size());
    for (size_t i = 0; i < ls.size(); i++) live[i] = leafDead[size_t(ls[i])] ? 0 : 1;
    int rc = kueue_tas_snapshot_set_leaf_live(ctx, ls.data(), ls.size(), live.data());
    if (rc) err = std::string("leaf liveness: ") + kueue_tas_last_error(ctx);
    return rc;
  }
  // Pushes touched leaves to the device: free-capacity rows (allocatable -
  // non-TAS usage) and, with hostname leaves, taint profile + label columns.
  int push_leaves(const std::set<int32_t>& leaves, bool attrs) {
    bool new_col = false;
    for (int32_t l : leaves) {
      Requests f = leafAlloc[size_t(l)];
      for (auto& n : leafNodeNames[size_t(l)]) {
        auto u = nodeUsage.find(n);
        if (u != nodeUsage.end()) req_sub(f, u->second);
      }
      for (auto& kv : f) new_col |= !colByName.count(kv.first);
      freeCap[size_t(l)] = std::move(f);
    }
    if (new_col && recolumn()) return 0;  // dirty: the next upload() takes the host mirror
    if (dirty || !ctx || leaves.empty()) return 0;
    const size_t R = cols.size();
    std::vector<int32_t> ls(leaves.begin(), leaves.end());
    std::vector<int64_t> rows(ls.size() * R, 0);
    std::vector<uint32_t> pres(ls.size(), 0);
    for (size_t i = 0; i < ls.size(); i++)
      for (auto& kv : freeCap[size_t(ls[i])]) {
        const auto c = colByName.find(kv.first);
        if (c == colByName.end()) continue;  // a resource no request reads (wanted_columns)
        rows[i * R + size_t(c->second)] = kv.second;
        pres[i] |= 1u << c->second;
      }
    int rc = kueue_tas_snapshot_set_free(ctx, ls.data(), ls.size(), rows.data(), pres.data());
    if (rc) {
      err = std::string("set free: ") + kueue_tas_last_error(ctx);
      return rc;
    }
    if (!attrs || !lowestIsHostname) return 0;
    const size_t K = labelKeys.size();
    std::vector<int32_t> prof(ls.size()), lab(ls.size() * K);
    for (size_t i = 0; i < ls.size(); i++) {
      prof[i] = leafProfile[size_t(ls[i])];
      for (size_t k = 0; k < K; k++) lab[i * K + k] = labelValues[k * labStride + size_t(ls[i])];
    }
    rc = kueue_tas_snapshot_set_leaf_attrs(ctx, ls.data(), ls.size(), prof.data(), K ? lab.data() : nullptr);
    if (rc) err = std::string("set leaf attrs: ") + kueue_tas_last_error(ctx);
    return rc;
  }

  // Column sets are numbered process-wide: compiled requests hold column
  // indices, so a request compiled against an older set must be recompiled.
  uint64_t col_gen = 0;
  static uint64_t next_gen() {  // process-wide: a generation is never reused by another snapshot
    static std::atomic<uint64_t> gen_counter{0};
    return ++gen_counter;
  }
  void set_columns(const std::set<std::string>& names) {
    flush_mirror();  // pending records name columns of the old set
    col_gen = next_gen();
    cols.assign(names.begin(), names.end());
    colByName.clear();
    colOfId.clear();
    for (size_t i = 0; i < cols.size(); i++) {
      colByName[cols[i]] = int32_t(i);
      const size_t id = size_t(intern_resource(cols[i]));
      if (colOfId.size() <= id) colOfId.resize(id + 1, -1);
      colOfId[id] = int32_t(i);
    }
    auto pc = colByName.find("pods");
    podsCol = pc == colByName.end() ? -1 : pc->second;
    dirty = true;
    compile_gen++;
  }
  // The device columns: every resource name of the snapshot (free capacity,
  // TAS usage, requests) when they fit KUEUE_TAS_MAX_COLS; otherwise only
  // "pods" and the names requests / usage records / Fits terms have used —
  // a resource no request names never changes a count (CountIn and Fits
  // iterate the request's keys, requests.go:174-217), and the host mirror
  // keeps every resource for SerializeFreeCapacityPerDomain.  More than
  // KUEUE_TAS_MAX_COLS requested names in one flavor is the only limit.
  std::set<std::string> wanted_columns() const {
    std::set<std::string> all(reqNames);
    all.insert("pods");
    for (const Requests& f : freeCap) {
      for (auto& kv : f) all.insert(kv.first);
      if (all.size() > KUEUE_TAS_MAX_COLS) break;
    }
    if (all.size() <= KUEUE_TAS_MAX_COLS) return all;
    std::set<std::string> req(reqNames);
    req.insert("pods");
    if (req.size() > KUEUE_TAS_MAX_COLS)
      throw std::runtime_error("more than " + std::to_string(KUEUE_TAS_MAX_COLS) +
                               " distinct requested resources in one TAS flavor");
    return req;
  }
  // Re-derives the column set; returns true when it changed (compiled
  // requests are stale, the next upload() reloads).
  bool recolumn() {
    flush_mirror();
    clear_mirror_cache();
    const std::set<std::string> want = wanted_columns();
    if (want.size() == cols.size() && std::equal(want.begin(), want.end(), cols.begin())) return false;
    set_columns(want);
    return true;
  }
  // Requests may name resources no node has: they become all-absent columns.
  // Returns true when the column set changed (compiled requests are stale).
  std::vector<int32_t> colOfId;  // interned resource id -> column, -1 when none
  int32_t podsCol = -1;
  int32_t col_of(int32_t id) const { return size_t(id) < colOfId.size() ? colOfId[size_t(id)] : -1; }
  bool ensure_columns_for(const std::vector<TASPodSetRequests>& podsets) {
    bool known = true;
    for (auto& p : podsets)
      for (auto& kv : p.requestIds) known = known && col_of(kv.first) >= 0;
    if (known) return false;
    for (auto& p : podsets)
      for (auto& kv : p.singlePodRequests) reqNames.insert(kv.first);
    return recolumn();
  }

  int upload() {
    if (!dirty) return splicePending && ctx ? upload_splice() : 0;
    splicePending = false;
    spliceSrc.clear();
    flush_mirror();
    if (!ctx) {
      ctx = kueue_tas_ctx_create(&cfg);
      if (!ctx) {
        err = "kueue_tas_ctx_create failed: no usable HIP device (the TAS path has no CPU fallback)";
        return KUEUE_TAS_EDEVICE;
      }
      kueue_tas_set_stage_timing(ctx, stageTiming ? 1 : 0);
    }
    const int L = this->L(), N = this->N(), R = int(cols.size());
    std::vector<int32_t> sizes(L), co;
    for (int l = 0; l < L; l++) sizes[l] = int32_t(values[l].size());
    for (int l = 0; l + 1 < L; l++) co.insert(co.end(), childOff[l].begin(), childOff[l].end());
    std::vector<int64_t> fr(size_t(R) * N, 0), us(size_t(R) * N, 0);
    std::vector<uint32_t> fp(N, 0), up(N, 0);
    parallel_ranges(size_t(N), 8192, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; i++) {  // resources without a column are read by no request (wanted_columns)
        for (auto& kv : freeCap[i]) {
          const auto c = colByName.find(kv.first);
          if (c == colByName.end()) continue;
          fr[size_t(c->second) * size_t(N) + i] = kv.second;
          fp[i] |= 1u << c->second;
        }
        for (auto& kv : tasUsage[i]) {
          const auto c = colByName.find(kv.first);
          if (c == colByName.end()) continue;
          us[size_t(c->second) * size_t(N) + i] = kv.second;
          up[i] |= 1u << c->second;
        }
      }
    });
    std::vector<int32_t> ranks;
    for (int l = 0; l < L; l++) ranks.insert(ranks.end(), idRank[l].begin(), idRank[l].end());
    kueue_tas_snapshot_desc d{};
    d.num_levels = L;
    d.level_sizes = sizes.data();
    d.child_offsets = co.data();
    d.num_cols = R;
    d.free_capacity = fr.data();
    d.tas_usage = us.data();
    d.free_present = fp.data();
    d.usage_present = up.data();
    d.lowest_is_hostname = lowestIsHostname ? 1 : 0;
    d.taint_profile = leafProfile.data();
    d.num_label_cols = int32_t(labelKeys.size());
    std::vector<int32_t> labPacked;  // [K][N] for the load
    if (!labelValues.empty() && labStride != size_t(N)) {
      labPacked.resize(labelKeys.size() * size_t(N));
      for (size_t k = 0; k < labelKeys.size(); k++)
        memcpy(labPacked.data() + k * size_t(N), labelValues.data() + k * labStride, size_t(N) * 4);
    }
    d.label_values = labelValues.empty() ? nullptr : labStride != size_t(N) ? labPacked.data() : labelValues.data();
    d.domain_id_rank = ranks.data();
    int rc = kueue_tas_snapshot_load(ctx, &d);
    if (!rc) rc = kueue_tas_snapshot_usage_mark(ctx);  // device usage == host mirror
    if (rc) {
      err = std::string("snapshot load: ") + kueue_tas_last_error(ctx);
      return rc;
    }
    if ((rc = load_names())) return rc;
    if ((rc = set_tags())) return rc;
    {  // a load puts every leaf in: take the dead ones out again
      std::vector<int32_t> dl, live;
      for (int i = 0; i < N; i++)
        if (leafDead[size_t(i)]) dl.push_back(i);
      live.assign(dl.size(), 0);
      rc = dl.empty() ? 0 : kueue_tas_snapshot_set_leaf_live(ctx, dl.data(), dl.size(), live.data());
      if (rc) {
        err = std::string("leaf liveness: ") + kueue_tas_last_error(ctx);
        return rc;
      }
    }
    dirty = false;
    return 0;
  }

  // ---- usage updates and the admission re-check ----
  // One workload.TopologyDomainRequests (pkg/workload/workload.go:260-269).
  struct DomainUsage {
    std::string id;  // utiltas.DomainID(Values) (util/tas/tas.go:29-31)
    Requests single;
    int32_t count = 0;
  };
  static std::vector<DomainUsage> parse_usage(const kjson::Node& arr) {
    std::vector<DomainUsage> us;
    for (auto& u : arr.items) {
      DomainUsage d;
      for (size_t k = 0; k < u["values"].items.size(); k++) d.id += (k ? "," : "") + u["values"].items[k].s();
      for (auto& kv : u["singlePodRequests"].fields) d.single[kv.first] = kv.second.i64();
      d.count = int32_t(u["count"].i64());
      us.push_back(std::move(d));
    }
    return us;
  }
  // ClusterQueueSnapshot.AddUsage/RemoveUsage -> updateTASUsage
  // (clusterqueue_snapshot.go:94-119; tas_flavor_snapshot.go:257-293): the
  // leaf's tasUsage gains (or loses) SinglePodRequests.ScaledUp(count) plus
  // pods:count; domains that are not leaves are skipped.  The device replica
  // is updated in place by a delta launch; a resource no column holds yet
  // changes the column set, and then the next evaluation reloads the snapshot.
  // The device's own pending changes (admissions) stay pending: the mirror,
  // the device usage and the device's shadow of the mirror all take the same
  // deltas, so O(#records) work and no diff (updateTASUsage is O(#domains)).
  int update_usage(const std::vector<DomainUsage>& us, bool add, bool device = true) {
    {  // the mirror alone takes these deltas (stale device, or a new column reloads it): in step first
      bool known = !dirty && device;
      for (auto& u : us)
        for (auto& kv : u.single) known = known && colByName.count(kv.first);
      if (!known) flush_mirror();
    }
    std::vector<kueue_tas_delta> deltas;
    bool new_col = false;
    for (auto& u : us) {
      Requests tot;
      for (auto& kv : u.single) tot[kv.first] = mul64(kv.second, u.count);
      tot["pods"] = add64(tot["pods"], u.count);
      {  // the cache's usage per domain, kept for domains that are not leaves (yet)
        Requests& d = usageByDomain[u.id];
        for (auto& kv : tot) d[kv.first] = add ? add64(d[kv.first], kv.second) : sub64(d[kv.first], kv.second);
      }
      const int32_t leaf = leafById.find(u.id);
      if (leaf < 0) continue;
      for (auto& kv : tot) {
        Requests& mine = tasUsage[leaf];
        mine[kv.first] = add ? add64(mine[kv.first], kv.second) : sub64(mine[kv.first], kv.second);
        auto c = colByName.find(kv.first);
        if (c == colByName.end()) {
          new_col = true;
          continue;
        }
        deltas.push_back({leaf, c->second, add ? kv.second : sub64(0, kv.second)});
      }
    }
    if (new_col) {
      for (auto& u : us)
        for (auto& kv : u.single) reqNames.insert(kv.first);
      if (recolumn()) return 0;  // dirty: the next upload() takes the host mirror
    }
    if (!device || dirty || !ctx || deltas.empty()) return 0;
    int rc = kueue_tas_snapshot_apply_deltas_mirrored(ctx, deltas.data(), deltas.size());  // the mirror has them
    if (rc) err = std::string("apply deltas: ") + kueue_tas_last_error(ctx);
    return rc;
  }
  // Columns for every resource of a usage list (a removal overlay needs one).
  bool ensure_columns_for_usage(const std::vector<DomainUsage>& us) {
    bool known = true;
    for (auto& u : us)
      for (auto& kv : u.single) known = known && colByName.count(kv.first);
    if (known) return false;
    for (auto& u : us)
      for (auto& kv : u.single) reqNames.insert(kv.first);
    return recolumn();
  }
  // RemoveUsage(us) as an evaluation overlay: the leaf's tasUsage loses
  // SinglePodRequests x count + pods:count (updateTASUsage :257-293), so the
  // remaining capacity gains it; fillInCounts computes
  // free - (used - x) - assumed == free - used - (assumed - x) in Go's
  // wrapping int64, and both Subs create the key (requests.go:90-94).
  // Unknown domains are skipped like removeTASUsage does.
  std::vector<kueue_tas_assumed> removal(const std::vector<DomainUsage>& us) const {
    std::map<std::pair<int32_t, int32_t>, int64_t> o;
    for (auto& u : us) {
      const int32_t leaf = leafById.find(u.id);
      if (leaf < 0 || leafDead[size_t(leaf)]) continue;
      for (auto& kv : u.single) {
        int64_t& slot = o[{leaf, colByName.at(kv.first)}];
        slot = sub64(slot, mul64(kv.second, u.count));
      }
      int64_t& pods = o[{leaf, colByName.at("pods")}];
      pods = sub64(pods, u.count);
    }
    std::vector<kueue_tas_assumed> r;
    r.reserve(o.size());
    for (auto& kv : o) r.push_back({kv.first.first, kv.first.second, kv.second});
    return r;
  }
  // TASFlavorSnapshot.Fits (tas_flavor_snapshot.go:401-415), on the device.
  int fits(const std::vector<DomainUsage>& us, bool* out) {
    ensure_columns_for_usage(us);  // a term's resource must be a column to be read
    int rc = upload();
    if (rc) return rc;
    std::vector<kueue_tas_fits_req> reqs;
    std::vector<kueue_tas_fits_term> terms;
    for (auto& u : us) {
      kueue_tas_fits_req r{live_leaf(u.id), u.count, int32_t(terms.size()), 0};
      for (auto& kv : u.single) {
        auto c = colByName.find(kv.first);
        terms.push_back({kv.second, c == colByName.end() ? -1 : c->second, 0});
        r.num_terms++;
      }
      reqs.push_back(r);
    }
    std::vector<int32_t> f(reqs.size(), 0);
    rc = kueue_tas_fits(ctx, reqs.data(), reqs.size(), terms.data(), terms.size(), f.data());
    if (rc) {
      err = std::string("fits: ") + kueue_tas_last_error(ctx);
      return rc;
    }
    *out = std::all_of(f.begin(), f.end(), [](int32_t x) { return x != 0; });
    return 0;
  }

  // ---- request compilation: findTopologyAssignment prelude (:804-897) ----
  int resolve(const std::string& key) const {
    for (size_t i = 0; i < levelKeys.size(); i++)
      if (levelKeys[i] == key) return int(i);
    return -1;
  }
  static bool slice_only(const std::optional<TopologyRequest>& tr) {  // :1148-1153
    if (!tr || tr->required || tr->preferred) return false;
    return tr->sliceRequiredTopology.has_value() || !tr->constraints.empty();
  }
  const std::string* level_key(const TASPodSetRequests& r) const {  // :1112-1138
    const auto& tr = r.topologyRequest;
    if (tr) {
      if (tr->required) return &*tr->required;
      if (tr->preferred) return &*tr->preferred;
      if (slice_only(tr)) return &levelKeys.front();
      if (tr->unconstrained.value_or(false)) return &levelKeys.back();
    }
    if (r.implied) return &levelKeys.back();
    return nullptr;
  }
  // requests + pods:1 (:820-826) written as (column, value) in column order
  // (std::map order == column order: columns are the sorted names)
  int32_t emit_requests(const std::vector<std::pair<int32_t, int64_t>>& r, int32_t* col, int64_t* val) const {
    if (podsCol < 0) throw std::runtime_error("internal: no pods column");
    int32_t n = 0;
    bool pods = false;
    for (auto& kv : r) {
      const int32_t c = col_of(kv.first);
      if (c < 0) throw std::runtime_error("internal: request resource without a column");
      if (!pods && c >= podsCol) {
        pods = true;
        if (c == podsCol) {
          col[n] = c;
          val[n++] = add64(kv.second, 1);
          continue;
        }
        col[n] = podsCol;
        val[n++] = 1;
      }
      col[n] = c;
      val[n++] = kv.second;
    }
    if (!pods) {
      col[n] = podsCol;
      val[n++] = 1;
    }
    return n;
  }

  uint64_t compile_gen = 1;  // bumped whenever compiled requests may change
  void compile_group(GroupEval& g, bool simulateEmpty) {
    compile_gen++;
    compile_group_only(g, simulateEmpty);
  }
  // The columns every request of the PodSets names exist (ensure_columns_for
  // would not change anything); safe to call from several threads.
  bool columns_known(const std::vector<TASPodSetRequests>& podsets) const {
    for (auto& p : podsets)
      for (auto& kv : p.requestIds)
        if (col_of(kv.first) < 0) return false;
    return true;
  }
  // compile_group without the generation bump: reads the snapshot and writes
  // only g, so different groups compile concurrently (the caller bumps
  // compile_gen once for the batch)
  void compile_group_only(GroupEval& g, bool simulateEmpty) const {
    const TASPodSetRequests& w = *g.workers;
    kueue_tas_eval_req& q = g.req;
    memset(&q, 0, sizeof q);
    g.compiled = true;
    g.early_reason.clear();
    g.layer_names.clear();
    g.sel_ext.clear();
    g.sel_vals.clear();
    g.balanced = false;
    const auto& tr = w.topologyRequest;
    // getSliceSizeWithSinglePodAsDefault (:1162-1180)
    int32_t sliceSize = 1;
    if (tr) {
      if (!tr->constraints.empty()) sliceSize = tr->constraints[0].size;
      else if (tr->sliceRequiredTopology) {
        if (!tr->sliceSize) {
          g.early_reason = "slice topology requested, but slice size not provided";
          return;
        }
        sliceSize = *tr->sliceSize;
      }
    }
    if (sliceSize == 0) {
      g.early_reason = "panic: integer divide by zero";
      return;
    }
    g.slice_size = sliceSize;
    bool required = tr && tr->required.has_value();
    bool unconstrained = (tr && tr->unconstrained.value_or(false)) || w.implied || slice_only(tr);
    const std::string* key = level_key(w);
    if (!key) {
      g.early_reason = "topology level not specified";
      return;
    }
    int reqLevel = resolve(*key);
    if (reqLevel < 0) {
      g.early_reason = "no requested topology level: " + *key;
      return;
    }
    const std::string* sliceKeyP = &levelKeys.back();
    if (tr) {
      if (tr->sliceRequiredTopology) sliceKeyP = &*tr->sliceRequiredTopology;
      else if (!tr->constraints.empty()) sliceKeyP = &tr->constraints[0].topology;
    }
    const std::string& sliceKey = *sliceKeyP;
    int sliceLevel = resolve(sliceKey);
    if (sliceLevel < 0) {
      g.early_reason = "no requested topology level for slices: " + sliceKey;
      return;
    }
    if (reqLevel > sliceLevel) {
      g.early_reason = "podset slice topology " + sliceKey + " is above the podset topology " + *key;
      return;
    }
    // buildSliceSizeAtLevel (:1018-1063)
    std::map<int, int32_t> ssal;
    if (gates.multiLayer && tr) {
      int32_t prevSize = sliceSize;
      int prevLevel = sliceLevel;
      for (size_t i = 1; i < tr->constraints.size(); i++) {
        const auto& layer = tr->constraints[i];
        int inner = resolve(layer.topology);
        if (inner < 0) {
          g.early_reason = "no requested topology level for additional slice layer: " + layer.topology;
          return;
        }
        if (inner <= prevLevel) {
          g.early_reason = "additional slice layer topology " + layer.topology + " must be at a lower level than " +
                           levelKeys[prevLevel];
          return;
        }
        if (layer.size == 0) {
          g.early_reason = "panic: integer divide by zero";
          return;
        }
        if (prevSize % layer.size != 0) {
          g.early_reason = "additional slice layer size " + std::to_string(layer.size) +
                           " must evenly divide parent layer size " + std::to_string(prevSize);
          return;
        }
        for (int lvl = prevLevel + 1; lvl <= inner; lvl++) ssal[lvl] = layer.size;
        prevSize = layer.size;
        prevLevel = inner;
      }
    }
    bool multilayer = gates.multiLayer && !ssal.empty();
    q.flags = (required ? KUEUE_TAS_F_REQUIRED : 0u) | (unconstrained ? KUEUE_TAS_F_UNCONSTRAINED : 0u) |
              ((unconstrained && gates.profileMixed) ? KUEUE_TAS_F_LFC : 0u) |
              (simulateEmpty ? KUEUE_TAS_F_SIMULATE_EMPTY : 0u) | (g.leader ? KUEUE_TAS_F_LEADER : 0u) |
              (multilayer ? KUEUE_TAS_F_MULTILAYER : 0u);
    q.count = w.count;
    q.slice_size = sliceSize;
    q.requested_level = reqLevel;
    q.slice_level = sliceLevel;
    for (auto& kv : ssal) q.slice_size_at_level[kv.first] = kv.second;
    if (multilayer) {
      for (auto& c : tr->constraints) {
        int t = resolve(c.topology);
        if (t < 0) continue;  // multiLayerNotFitMessage skips unresolved layers (:1778-1781)
        if (q.num_layers >= KUEUE_TAS_MAX_LAYERS) break;
        if (c.size == 0) {
          g.early_reason = "panic: integer divide by zero";
          return;
        }
        q.layer_level[q.num_layers] = t;
        q.layer_size[q.num_layers] = c.size;
        g.layer_names.push_back(c.topology);
        q.num_layers++;
      }
    }
    // columns were ensured by ensure_columns_for()
    q.num_req = emit_requests(w.requestIds, q.req_col, q.req_val);
    if (g.leader) q.num_leader_req = emit_requests(g.leader->requestIds, q.leader_col, q.leader_val);
    // tolerations = podset + flavor (:877); first untolerated NoSchedule/NoExecute taint per profile
    g.taint_row.assign(profiles.size(), -1);
    if (lowestIsHostname) {
      for (size_t p = 0; p < profiles.size(); p++) {
        for (size_t k = 0; k < profiles[p].size(); k++) {
          const Taint& t = profiles[p][k];
          bool ok = false;
          for (auto& tol : w.tolerations) ok = ok || tolerates(tol, t);
          for (auto& tol : flavorTolerations) ok = ok || tolerates(tol, t);
          if (!ok) {
            g.taint_row[p] = profileTaintIds[p][k];
            break;
          }
        }
      }
      // nodeSelector: labels.ValidatedSelectorFromSet (only with hostname leaves, :879-887)
      if (w.nodeSelector) {
        const std::string e = labelsel::node_selector_failure(*w.nodeSelector);
        if (!e.empty()) {
          g.early_reason = e;
          return;
        }
      }
      if (w.nodeSelector && !w.nodeSelector->empty() && !labelKeys.empty()) {
        // any number of pairs (one Equals requirement per key): the first
        // KUEUE_TAS_MAX_SELECTORS inline, the rest as requirements of the
        // batch affinity table (a key or value no leaf has: id -1, no match)
        for (auto& kv : *w.nodeSelector) {
          auto it = labelCol.find(kv.first);
          int col = it == labelCol.end() ? 0 : it->second;
          int val = -1;
          if (it != labelCol.end()) {
            auto d = labelDict[col].find(kv.second);
            if (d != labelDict[col].end()) val = d->second;
          }
          if (q.num_selectors < KUEUE_TAS_MAX_SELECTORS) {
            q.sel_col[q.num_selectors] = col;
            q.sel_val[q.num_selectors] = val;
            q.num_selectors++;
          } else {
            g.sel_ext.push_back({0, col, 0, int32_t(g.sel_vals.size()), 1});
            g.sel_vals.push_back(val);
          }
        }
        if (!g.sel_ext.empty()) q.flags |= KUEUE_TAS_F_SELECTOR_EXT;
      }
    }
    // required node affinity: validated always, filters only hostname leaves (:889-897, :1605-1610)
    g.aff.clear();
    g.aff_vals.clear();
    if (w.affinity) {
      const std::string e = labelsel::affinity_failure(*w.affinity);
      if (!e.empty()) {
        g.early_reason = e;
        return;
      }
      if (lowestIsHostname) compile_affinity(*w.affinity, g);
    }
    // TASBalancedPlacement branches after fillInCounts (:907-917): the
    // device computes phase 1, the host layer the balanced placement
    g.balanced = gates.balanced && !required && !unconstrained;
  }

  // Required node affinity compiled against the snapshot's label
  // dictionaries (nodeaffinity.NodeSelector.Match, nodeaffinity.go:84-201;
  // labels.Requirement.Matches, selector.go:247-294): every requirement
  // becomes a sorted set of label-value ids of one column (0 = label absent)
  // XOR negate, or a set of leaf indices for matchFields on metadata.name;
  // requirements with the same outcome on every leaf fold away.  Sets
  // KUEUE_TAS_F_AFFINITY unless every leaf matches; no remaining term means
  // no leaf matches.  Matching runs in the fill kernels (affinity_match).
  void compile_affinity(const labelsel::RequiredAffinity& terms, GroupEval& g) const {
    int32_t term_id = 0;
    auto add = [&](int32_t col, std::vector<int32_t> ids, bool negate) {
      std::sort(ids.begin(), ids.end());
      ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
      g.aff.push_back({term_id, col, negate ? 1 : 0, int32_t(g.aff_vals.size()), int32_t(ids.size())});
      g.aff_vals.insert(g.aff_vals.end(), ids.begin(), ids.end());
    };
    for (const labelsel::Term& t : terms) {
      if (t.empty()) continue;  // an empty term is dropped by NewLazyErrorNodeSelector (:60-64)
      const size_t mark_r = g.aff.size(), mark_v = g.aff_vals.size();
      bool never = false;
      for (const labelsel::Expr& e : t.exprs) {
        const auto c = labelCol.find(e.key);
        if (c == labelCol.end()) {  // no leaf has the key: constant outcome
          never |= !(e.op == "NotIn" || e.op == "DoesNotExist");
          continue;
        }
        const auto& dict = labelDict[size_t(c->second)];
        std::vector<int32_t> ids;
        if (e.op == "In" || e.op == "NotIn") {
          for (auto& v : *e.values) {
            auto d = dict.find(v);
            if (d != dict.end()) ids.push_back(d->second);
          }
          if (ids.empty()) {  // no leaf carries any of the values
            never |= e.op == "In";
            continue;
          }
          add(c->second, std::move(ids), e.op == "NotIn");
        } else if (e.op == "Exists" || e.op == "DoesNotExist") {
          add(c->second, {0}, e.op == "Exists");
        } else {  // Gt / Lt over the column's distinct values that parse as int64
          int64_t rv = 0, lv = 0;
          labelsel::parse_int((*e.values)[0], &rv);
          for (auto& kv : dict)
            if (labelsel::parse_int(kv.first, &lv) && (e.op == "Gt" ? lv > rv : lv < rv)) ids.push_back(kv.second);
          if (ids.empty()) {
            never = true;
            continue;
          }
          add(c->second, std::move(ids), false);
        }
      }
      // matchFields: field value is the node name for metadata.name, "" for
      // any other key; ignored on a node without a name (:197)
      for (const labelsel::Expr& e : t.fields) {
        const std::string& v = (*e.values)[0];
        const bool in = e.op == "In";
        std::vector<int32_t> ids;
        if (e.key == "metadata.name") {
          const int32_t named = leafByNodeName.find(v);
          if (in) {
            if (named >= 0) ids.push_back(named);
            ids.insert(ids.end(), unnamedLeaves.begin(), unnamedLeaves.end());
            if (ids.empty()) never = true;
            else add(KUEUE_TAS_AFFINITY_LEAF, std::move(ids), false);
          } else if (named >= 0) {
            add(KUEUE_TAS_AFFINITY_LEAF, {named}, true);
          }
        } else if (in != v.empty()) {  // In "x" / NotIn "": only unnamed leaves pass
          if (unnamedLeaves.empty()) never = true;
          else add(KUEUE_TAS_AFFINITY_LEAF, unnamedLeaves, false);
        }
      }
      if (never) {  // the term matches no leaf
        g.aff.resize(mark_r);
        g.aff_vals.resize(mark_v);
        continue;
      }
      if (g.aff.size() == mark_r) {  // the term matches every leaf, so does the selector
        g.aff.clear();
        g.aff_vals.clear();
        return;
      }
      term_id++;
    }
    g.req.flags |= KUEUE_TAS_F_AFFINITY;
  }

  // ---- snapshot queries of the scheduler's callers ----
  // HasLevel (tas_flavor_snapshot.go:1065-1088): the request's level key
  // (levelKey :1120-1138, no implied fallback) and its slice level key
  // (sliceLevelKeyWithDefault :1090-1100, default the lowest level) resolve;
  // with TASMultiLayerTopology every additional layer's topology too.
  bool has_level(const std::optional<TopologyRequest>& tr) const {
    if (!tr) return false;
    const std::string* key = nullptr;
    if (tr->required) key = &*tr->required;
    else if (tr->preferred) key = &*tr->preferred;
    else if (slice_only(tr)) key = &levelKeys.front();
    else if (tr->unconstrained.value_or(false)) key = &levelKeys.back();
    if (!key) return false;
    const std::string& sliceKey = tr->sliceRequiredTopology ? *tr->sliceRequiredTopology
                                  : !tr->constraints.empty() ? tr->constraints[0].topology
                                                              : levelKeys.back();
    if (resolve(*key) < 0 || resolve(sliceKey) < 0) return false;
    if (gates.multiLayer)
      for (auto& c : tr->constraints)
        if (resolve(c.topology) < 0) return false;
    return true;
  }
  // DomainID -> present, for every level (TASFlavorSnapshot.domains)
  // (the tree of a snapshot object never changes: node events that move a
  // node rebuild it into a new object)
  mutable std::unordered_map<std::string, int32_t> upperDomainIds;  // levels 0..L-2, built on first use
  mutable bool upperBuilt = false;
  bool has_domain(const std::string& id) const {
    if (live_leaf(id) >= 0) return true;
    if (!upperBuilt) {
      upperDomainIds.clear();
      for (int l = 0; l + 1 < L(); l++)
        for (size_t i = 0; i < values[size_t(l)].size(); i++) {
          std::string d;
          for (size_t k = 0; k < values[size_t(l)][i].size(); k++) d += (k ? "," : "") + values[size_t(l)][i][k];
          upperDomainIds.emplace(std::move(d), l);
        }
      upperBuilt = true;
    }
    return upperDomainIds.count(id) != 0;
  }
  // IsTopologyAssignmentStale (:733-743): the first domain whose
  // DomainID(Values) is not a domain of the snapshot -> (true, Values[0]).
  bool assignment_stale(const kjson::Node& ta, std::string* domain) const {
    for (auto& d : ta["domains"].items) {
      std::string id;
      const auto& vs = d["values"].items;
      for (size_t k = 0; k < vs.size(); k++) id += (k ? "," : "") + vs[k].s();
      if (!has_domain(id)) {
        *domain = vs.empty() ? std::string() : vs[0].s();
        return true;
      }
    }
    return false;
  }
  // SerializeFreeCapacityPerDomain (:320-355): every leaf's freeCapacity and
  // tasUsage as resources.ResourceQuantityString values, json.Marshal of the
  // maps (keys sorted).
  std::string free_capacity_json() {
    flush_mirror();
    std::vector<int32_t> ord(static_cast<size_t>(N()));
    for (int i = 0; i < N(); i++) ord[size_t(i)] = i;
    std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return leafId[size_t(a)] < leafId[size_t(b)]; });
    std::string out = "{";
    auto reqs = [&](const Requests& r) {
      out += "{";
      bool first = true;
      for (auto& kv : r) {
        if (!first) out += ",";
        first = false;
        labelsel::json_escape(out, kv.first);
        out += ":";
        labelsel::json_escape(out, resource_quantity_string(kv.first, kv.second));
      }
      out += "}";
    };
    bool firstLeaf = true;
    for (size_t k = 0; k < ord.size(); k++) {
      if (leafDead[size_t(ord[k])]) continue;  // not a leaf of the snapshot
      if (!firstLeaf) out += ",";
      firstLeaf = false;
      labelsel::json_escape(out, leafId[size_t(ord[k])]);
      out += ":{\"freeCapacity\":";
      reqs(freeCap[size_t(ord[k])]);
      out += ",\"tasUsage\":";
      reqs(tasUsage[size_t(ord[k])]);
      out += "}";
    }
    return out + "}";
  }

  // ---- failure strings ----
  // ExclusionStats reasons (:480-499) in sorted order.  Every reason is
  // "<prefix><count>" with a distinct prefix ending in ": ", so sorting the
  // full strings is sorting the prefixes: that order is computed once per
  // (taints, columns) set, not per failure.
  mutable std::vector<std::pair<std::string, int32_t>> reasonOrder;  // (prefix, kind: -3..-1 fixed, t, T + c)
  mutable size_t reasonFor = size_t(-1);
  void reason_order() const {
    const size_t key = taintStrings.size() * 1000003u + cols.size() * 7919u + compile_gen;
    if (reasonFor == key) return;
    reasonOrder.clear();
    reasonOrder.emplace_back("nodeSelector: ", -1);
    reasonOrder.emplace_back("affinity: ", -2);
    reasonOrder.emplace_back("topologyDomain: ", -3);
    for (size_t t = 0; t < taintStrings.size(); t++)
      reasonOrder.emplace_back("taint " + go_quote(taintStrings[t]) + ": ", int32_t(t));
    for (size_t c = 0; c < cols.size(); c++)
      reasonOrder.emplace_back("resource " + go_quote(cols[c]) + ": ", int32_t(taintStrings.size() + c));
    std::sort(reasonOrder.begin(), reasonOrder.end());
    reasonFor = key;
  }
  void format_stats(std::string& out, const kueue_tas_eval_out& o, const int32_t* taints, const int32_t* res) const {
    reason_order();
    const int32_t T = int32_t(taintStrings.size());
    bool first = true;
    for (const auto& r : reasonOrder) {
      const int32_t k = r.second;
      const int32_t v = k == -1 ? o.excl_selector : k == -2 ? o.excl_affinity : k == -3 ? o.excl_topology
                                                         : k < T ? taints[k] : res[k - T];
      if (v <= 0) continue;
      if (first) {
        out += ". Total nodes: ";
        append_int(out, o.total_nodes);
        out += "; excluded: ";
        first = false;
      } else {
        out += ", ";
      }
      out += r.first;
      append_int(out, v);
    }
  }
  // notFitMessage / multiLayerNotFitMessage text written into m (cleared
  // first; its storage is reused from one failure to the next)
  void failure_reason(std::string& m, const GroupEval& g, const kueue_tas_eval_out& o, const int32_t* taints,
                      const int32_t* res) const {
    m.clear();
    auto put = [&](int64_t v) { append_int(m, v); };
    switch (o.status) {
      case KUEUE_TAS_ST_NO_DOMAINS:
        m += "no topology domains at level: ";
        m += levelKeys[o.a];
        return;
      case KUEUE_TAS_ST_NOT_FIT: {
        m += "topology ";
        m += topology_quoted();
        if (o.a == 0) {
          m += " doesn't allow to fit any of ";
        } else {
          m += " allows to fit only ";
          put(o.a);
          m += " out of ";
        }
        put(o.b);
        m += g.slice_size == 1 ? " pod(s)" : " slice(s)";
        format_stats(m, o, taints, res);
        return;
      }
      case KUEUE_TAS_ST_MULTILAYER: {
        m += "topology ";
        m += topology_quoted();
        m += " doesn't allow to fit";
        if (values[o.a].empty()) return;
        for (int c = 0; c < g.req.num_layers; c++) {
          m += "; ";
          put(o.ml_fit[c]);
          m += "/";
          put(o.ml_need[c]);
          m += " slice(s) fit on level ";
          m += g.layer_names[c];
        }
        format_stats(m, o, taints, res);
        return;
      }
      default:
        m += "internal: device evaluation exceeded its list/output capacity";
    }
  }
  std::string failure_reason(const GroupEval& g, const kueue_tas_eval_out& o, const int32_t* taints,
                             const int32_t* res) const {
    std::string m;
    failure_reason(m, g, o, taints, res);
    return m;
  }
};

// FindTopologyAssignmentsForFlavor (:519-594): groups in first-seen order
// (GroupEval storage is reused across calls: a regroup keeps the vectors' capacity)
static void make_groups(Workload& wl) {
  bool named = false;
  for (auto& p : wl.podsets) named |= p.podSetGroupName.has_value();
  if (!named) {  // every PodSet is its own group
    wl.groups.resize(wl.podsets.size());
    for (size_t i = 0; i < wl.podsets.size(); i++) {
      GroupEval& g = wl.groups[i];
      g.compiled = false;
      g.members.assign(1, &wl.podsets[i]);
      g.workers = &wl.podsets[i];
      g.leader = nullptr;
    }
    return;
  }
  std::vector<std::string> order;
  std::map<std::string, std::vector<const TASPodSetRequests*>> grouped;
  for (size_t i = 0; i < wl.podsets.size(); i++) {
    const auto& p = wl.podsets[i];
    std::string key = p.podSetGroupName ? *p.podSetGroupName : std::to_string(i);
    if (std::find(order.begin(), order.end(), key) == order.end()) order.push_back(key);
    grouped[key].push_back(&p);
  }
  wl.groups.clear();
  for (auto& k : order) {
    auto& trs = grouped[k];
    GroupEval g;
    g.members = trs;
    g.workers = trs[0];
    if (trs.size() > 1) {  // findLeaderAndWorkers (:596-609)
      g.leader = trs[1];
      if (g.leader->count > g.workers->count) {
        g.leader = trs[0];
        g.workers = trs[1];
      }
    }
    wl.groups.push_back(std::move(g));
  }
}

// PodSpec.Affinity.NodeAffinity.RequiredDuringSchedulingIgnoredDuringExecution
// in its Kubernetes JSON shape; nullopt when any step is absent or null.
static std::optional<labelsel::RequiredAffinity> parse_required_affinity(const kjson::Node& aff) {
  if (aff.type != kjson::Node::kObject) return std::nullopt;
  const kjson::Node& na = aff["nodeAffinity"];
  if (na.type != kjson::Node::kObject) return std::nullopt;
  const kjson::Node& req = na["requiredDuringSchedulingIgnoredDuringExecution"];
  if (req.type != kjson::Node::kObject) return std::nullopt;
  auto exprs = [](const kjson::Node& arr) {
    std::vector<labelsel::Expr> out;
    for (auto& r : arr.items) {
      labelsel::Expr e;
      e.key = r["key"].s();
      e.op = r["operator"].s();
      if (r["values"].type == kjson::Node::kArray) {
        e.values.emplace();
        for (auto& v : r["values"].items) e.values->push_back(v.s());
      }
      out.push_back(std::move(e));
    }
    return out;
  };
  labelsel::RequiredAffinity terms;
  for (auto& t : req["nodeSelectorTerms"].items) terms.push_back({exprs(t["matchExpressions"]), exprs(t["matchFields"])});
  return terms;
}

// kueue.PodSetTopologyRequest in its JSON shape (nullopt for null)
static std::optional<TopologyRequest> parse_topology_request(const kjson::Node& tr) {
  if (tr.null()) return std::nullopt;
  TopologyRequest t;
  if (!tr["required"].null()) t.required = tr["required"].s();
  if (!tr["preferred"].null()) t.preferred = tr["preferred"].s();
  if (!tr["unconstrained"].null()) t.unconstrained = tr["unconstrained"].b();
  if (!tr["podSetSliceRequiredTopology"].null()) t.sliceRequiredTopology = tr["podSetSliceRequiredTopology"].s();
  if (!tr["podSetSliceSize"].null()) t.sliceSize = int32_t(tr["podSetSliceSize"].i64());
  for (auto& c : tr["podsetSliceRequiredTopologyConstraints"].items)
    t.constraints.push_back({c["topology"].s(), int32_t(c["size"].i64())});
  return t;
}

static std::vector<TASPodSetRequests> parse_podsets(const kjson::Node& arr) {
  std::vector<TASPodSetRequests> out;
  for (auto& ps : arr.items) {
    TASPodSetRequests r;
    r.name = ps["name"].s();
    const kjson::Node& tr = ps["topologyRequest"];
    r.topologyRequest = parse_topology_request(tr);
    r.implied = tr.null();
    if (auto im = ps.find("implied")) r.implied = im->b();
    for (auto& kv : ps["requests"].fields) r.singlePodRequests[kv.first] = kv.second.i64();
    for (auto& kv : r.singlePodRequests) r.requestIds.emplace_back(intern_resource(kv.first), kv.second);
    r.count = int32_t(ps["count"].i64());
    if (!ps["podSetGroupName"].null()) r.podSetGroupName = ps["podSetGroupName"].s();
    for (auto& t : ps["tolerations"].items)
      r.tolerations.push_back({t["key"].s(), t["operator"].s(), t["value"].s(), t["effect"].s()});
    if (ps["nodeSelector"].type == kjson::Node::kObject) {
      std::map<std::string, std::string> m;
      for (auto& kv : ps["nodeSelector"].fields) m[kv.first] = kv.second.s();
      r.nodeSelector = m;
    }
    r.affinity = parse_required_affinity(ps["affinity"]);
    if (auto pa = ps.find("previousAssignment"))
      if (!pa->null()) r.previousAssignment = parse_explicit(*pa);
    out.push_back(std::move(r));
  }
  return out;
}

// Batched driver: pass p evaluates group p of every workload still running
// (groups of one workload are sequential through assumedUsage, :543-591).
using ktas_pool::HostPool;


// A workload's assumedUsage overlay across its PodSet groups (addAssumedUsage
// :658-666): records appended per assigned domain, sorted by (leaf, column)
// and merged (wrapping add: order-free) before the next pass reads them.
struct AssumedUsage {
  std::vector<kueue_tas_assumed> v;
  size_t merged = 0;  // v is sorted with distinct keys when merged == v.size()
  void add(int32_t leaf, int32_t col, int64_t x) { v.push_back({leaf, col, x}); }
  const std::vector<kueue_tas_assumed>& records() {
    if (merged != v.size()) {
      std::stable_sort(v.begin(), v.end(), [](const kueue_tas_assumed& a, const kueue_tas_assumed& b) {
        return a.leaf < b.leaf || (a.leaf == b.leaf && a.col < b.col);
      });
      size_t o = 0;
      for (size_t i = 0; i < v.size(); i++) {
        if (o > 0 && v[o - 1].leaf == v[i].leaf && v[o - 1].col == v[i].col) v[o - 1].value = add64(v[o - 1].value, v[i].value);
        else v[o++] = v[i];
      }
      v.resize(o);
      merged = o;
    }
    return v;
  }
};

struct Evaluator {
  FlavorSnapshot* snap;
  float ms[4] = {0, 0, 0, 0};
  float stage_ms[KUEUE_TAS_NUM_STAGES] = {};
  double dev_host_ms[8] = {};
  double host_ms[4] = {0, 0, 0, 0};  // prepare, eval call (incl. device), decode, total
  double detail_ms[4] = {0, 0, 0, 0};  // grouping + column check, request compile, build_pass, Values
  int64_t counts[3] = {0, 0, 0};
  int64_t stats[6] = {0, 0, 0, 0, 0, 0};  // kueue_tas_last_stats summed over the run's batches, [4] fill paths,
                                          // [5] alias fill rows
  std::vector<const kueue_tas_eval_req*> reqs;  // the batch's requests: the groups' own records, by address
  std::vector<int32_t> taint_table;
  std::vector<kueue_tas_assumed> assumed;
  std::vector<kueue_tas_affinity_req> aff;
  std::vector<int32_t> affv;
  std::vector<kueue_tas_eval_out> outs;
  std::vector<int64_t> offsets;
  std::vector<int32_t> entries, taint_counts, res_counts;
  std::vector<std::pair<size_t, GroupEval*>> batch;
  // first pass (every workload's first group, no assumed usage) cached for
  // repeated runs over the same compiled workloads (run_compiled)
  const std::vector<Workload>* p0_for = nullptr;
  uint64_t p0_gen = 0;
  std::vector<const kueue_tas_eval_req*> p0_reqs;
  std::vector<int32_t> p0_taint;
  std::vector<kueue_tas_affinity_req> p0_aff;
  std::vector<int32_t> p0_affv;
  std::vector<std::pair<size_t, GroupEval*>> p0_batch, p0_early;
  std::vector<size_t> used;  // results set per workload in this run
  std::string reasonBuf;

  // Results are updated in place (member order = first set in this run), so
  // repeated runs reuse the strings' and vectors' storage.
  void set_result(std::vector<PodSetResult>& rs, size_t& n, const std::string& name, bool has,
                  const DomainAssignment* d, size_t nd, const std::string& reason) {
    for (size_t k = 0; k < n; k++)
      if (rs[k].name == name) {
        rs[k].has_assignment = has;
        rs[k].domains = DomainSpan{d, nd};
        rs[k].values = nullptr;
        rs[k].reason = reason;
        return;
      }
    if (n == rs.size()) rs.emplace_back();
    PodSetResult& r = rs[n++];
    r.name = name;
    r.has_assignment = has;
    r.domains = DomainSpan{d, nd};  // zero-copy view of the batch's entries
    r.values = nullptr;
    r.reason = reason;
  }

  // requests of one pass: taint rows shared through rowOff, assumed usage per workload
  void build_pass(std::vector<Workload>& wls, size_t pass, const std::vector<char>& done,
                  std::vector<AssumedUsage>& assumedBy,
                  std::vector<const kueue_tas_eval_req*>& rq, std::vector<int32_t>& tt, std::vector<kueue_tas_assumed>& as,
                  std::vector<kueue_tas_affinity_req>& af, std::vector<int32_t>& afv,
                  std::vector<std::pair<size_t, GroupEval*>>& bt, std::vector<std::pair<size_t, GroupEval*>>& early) {
    rq.clear();
    tt.clear();
    as.clear();
    af.clear();
    afv.clear();
    bt.clear();
    early.clear();
    std::map<std::vector<int32_t>, int32_t> rowOff;
    const std::vector<int32_t>* lastRow = nullptr;
    int32_t lastOff = 0;
    for (size_t w = 0; w < wls.size(); w++) {
      if (done[w] || pass >= wls[w].groups.size()) continue;
      GroupEval& g = wls[w].groups[pass];
      if (!g.early_reason.empty()) {
        early.emplace_back(w, &g);
        continue;
      }
      // the batch tables' offsets go into the group's own record, which the
      // batch references in place (kueue_tas_eval_batch_ptrs: no copy)
      kueue_tas_eval_req& q = g.req;
      rq.push_back(&q);
      if (!lastRow || *lastRow != g.taint_row) {  // consecutive requests mostly share a row
        auto it = rowOff.find(g.taint_row);
        if (it == rowOff.end()) {
          it = rowOff.emplace(g.taint_row, int32_t(tt.size())).first;
          tt.insert(tt.end(), g.taint_row.begin(), g.taint_row.end());
        }
        lastRow = &g.taint_row;
        lastOff = it->second;
      }
      q.taint_table = lastOff;
      q.affinity_begin = int32_t(af.size());
      if (q.flags & KUEUE_TAS_F_AFFINITY) {  // rebase the group's requirements into the batch tables
        const int32_t vb = int32_t(afv.size());
        for (auto r : g.aff) {
          r.begin += vb;
          af.push_back(r);
        }
        afv.insert(afv.end(), g.aff_vals.begin(), g.aff_vals.end());
      }
      q.affinity_end = int32_t(af.size());
      q.selector_begin = q.selector_end = int32_t(af.size());
      if (q.flags & KUEUE_TAS_F_SELECTOR_EXT) {  // nodeSelector pairs beyond the inline ones, same tables
        const int32_t vb = int32_t(afv.size());
        for (auto r : g.sel_ext) {
          r.begin += vb;
          af.push_back(r);
        }
        afv.insert(afv.end(), g.sel_vals.begin(), g.sel_vals.end());
        q.selector_end = int32_t(af.size());
      }
      q.assumed_begin = int32_t(as.size());
      const std::vector<kueue_tas_assumed>& mine = assumedBy[w].records();
      if (base && !(*base)[w].empty()) {  // merge the base overlay with the group's assumed usage
        const Overlay& b = (*base)[w];
        size_t k = 0;
        for (const kueue_tas_assumed& r : mine) {
          while (k < b.size() && (b[k].leaf < r.leaf || (b[k].leaf == r.leaf && b[k].col < r.col))) as.push_back(b[k++]);
          if (k < b.size() && b[k].leaf == r.leaf && b[k].col == r.col)
            as.push_back({r.leaf, r.col, add64(b[k++].value, r.value)});
          else
            as.push_back(r);
        }
        as.insert(as.end(), b.begin() + int64_t(k), b.end());
      } else {
        as.insert(as.end(), mine.begin(), mine.end());
      }
      q.assumed_end = int32_t(as.size());
      bt.emplace_back(w, &g);
    }
  }

  // build_pass for the first pass without a base overlay (the batch of
  // every timed step), assembled by the pool's static parts: part t holds
  // the workloads whose groups thread t compiled, so it reads them from its
  // own cache.  Each part first lays out its share in local tables, then —
  // once the parts' sizes give their offsets — writes it into the batch
  // tables and rebases its records' offsets.  Same batch as build_pass
  // (taint rows are deduplicated within a part only: equal rows compare
  // equal by value wherever they are).
  struct alignas(64) PartBatch {  // one per host part, on cache lines of its own
    std::vector<const kueue_tas_eval_req*> rq;
    std::vector<std::pair<size_t, GroupEval*>> bt, early;
    std::vector<int32_t> tt;
    std::vector<std::pair<const std::vector<int32_t>*, int32_t>> rows;  // distinct rows of the part, local offsets
    std::vector<kueue_tas_affinity_req> af;
    std::vector<int32_t> afv;
    size_t rqb = 0, ttb = 0, afb = 0, afvb = 0;
  };
  std::vector<PartBatch> partBatch;
  void build_pass0_static(std::vector<Workload>& wls, const std::vector<char>& done,
                          std::vector<const kueue_tas_eval_req*>& rq, std::vector<int32_t>& tt,
                          std::vector<kueue_tas_assumed>& as, std::vector<kueue_tas_affinity_req>& af,
                          std::vector<int32_t>& afv, std::vector<std::pair<size_t, GroupEval*>>& bt,
                          std::vector<std::pair<size_t, GroupEval*>>& early) {
    HostPool& pool = HostPool::get();
    const size_t T = pool.parts(), W = wls.size();
    partBatch.resize(T);
    // every part is cleared here, not in its task: run_static skips empty
    // parts (W < parts()), and a part left from a larger batch would still
    // be merged below with pointers into that batch's workloads
    for (auto& pb : partBatch) {
      pb.rq.clear();
      pb.bt.clear();
      pb.early.clear();
      pb.tt.clear();
      pb.rows.clear();
      pb.af.clear();
      pb.afv.clear();
    }
    auto part_of = [&](size_t b) {
      size_t t = 0;
      while (t + 1 < T && HostPool::part_begin(W, t + 1, T) <= b) t++;
      return t;
    };
    pool.run_static(W, [&](size_t b, size_t e) {
      PartBatch& pb = partBatch[part_of(b)];
      for (size_t w = b; w < e; w++) {
        if (done[w] || wls[w].groups.empty()) continue;
        GroupEval& g = wls[w].groups[0];
        if (!g.early_reason.empty()) {
          pb.early.emplace_back(w, &g);
          continue;
        }
        kueue_tas_eval_req& q = g.req;
        pb.rq.push_back(&q);
        int32_t off = -1;
        for (auto& r : pb.rows)  // a handful of distinct rows per batch
          if (r.first == &g.taint_row || *r.first == g.taint_row) {
            off = r.second;
            break;
          }
        if (off < 0) {
          off = int32_t(pb.tt.size());
          pb.rows.emplace_back(&g.taint_row, off);
          pb.tt.insert(pb.tt.end(), g.taint_row.begin(), g.taint_row.end());
        }
        q.taint_table = off;  // part-local offsets: rebased below
        q.affinity_begin = int32_t(pb.af.size());
        if (q.flags & KUEUE_TAS_F_AFFINITY) {
          const int32_t vb = int32_t(pb.afv.size());
          for (auto r : g.aff) {
            r.begin += vb;
            pb.af.push_back(r);
          }
          pb.afv.insert(pb.afv.end(), g.aff_vals.begin(), g.aff_vals.end());
        }
        q.affinity_end = int32_t(pb.af.size());
        q.selector_begin = q.selector_end = int32_t(pb.af.size());
        if (q.flags & KUEUE_TAS_F_SELECTOR_EXT) {
          const int32_t vb = int32_t(pb.afv.size());
          for (auto r : g.sel_ext) {
            r.begin += vb;
            pb.af.push_back(r);
          }
          pb.afv.insert(pb.afv.end(), g.sel_vals.begin(), g.sel_vals.end());
          q.selector_end = int32_t(pb.af.size());
        }
        q.assumed_begin = q.assumed_end = 0;  // no assumed usage before the first pass
        pb.bt.emplace_back(w, &g);
      }
    });
    size_t nrq = 0, ntt = 0, naf = 0, nafv = 0;
    early.clear();
    for (auto& pb : partBatch) {
      pb.rqb = nrq;
      pb.ttb = ntt;
      pb.afb = naf;
      pb.afvb = nafv;
      nrq += pb.rq.size();
      ntt += pb.tt.size();
      naf += pb.af.size();
      nafv += pb.afv.size();
      early.insert(early.end(), pb.early.begin(), pb.early.end());
    }
    rq.resize(nrq);
    bt.resize(nrq);
    tt.resize(ntt);
    af.resize(naf);
    afv.resize(nafv);
    as.clear();
    pool.run_static(W, [&](size_t b, size_t) {
      PartBatch& pb = partBatch[part_of(b)];
      const int32_t ttb = int32_t(pb.ttb), afb = int32_t(pb.afb), afvb = int32_t(pb.afvb);
      for (size_t k = 0; k < pb.rq.size(); k++) {
        kueue_tas_eval_req& q = pb.bt[k].second->req;
        q.taint_table += ttb;
        q.affinity_begin += afb;
        q.affinity_end += afb;
        q.selector_begin += afb;
        q.selector_end += afb;
        rq[pb.rqb + k] = pb.rq[k];
        bt[pb.rqb + k] = pb.bt[k];
      }
      std::copy(pb.tt.begin(), pb.tt.end(), tt.begin() + int64_t(pb.ttb));
      for (size_t k = 0; k < pb.af.size(); k++) {
        kueue_tas_affinity_req r = pb.af[k];
        r.begin += afvb;
        af[pb.afb + k] = r;
      }
      std::copy(pb.afv.begin(), pb.afv.end(), afv.begin() + int64_t(pb.afvb));
    });
  }

  // ---- TASBalancedPlacement (tas_flavor_snapshot.go:906-917) ----
  // For the batch's balanced groups: their phase-1 counters from a second
  // device batch of just those requests (kueue_tas_last_counters), then the
  // host algorithm (tas_balanced.h).  balOut[i].used: useBalancedPlacement;
  // otherwise the first batch's findLevelWithFitDomains result stands.  The
  // first batch's entries are copied first (the second batch reuses the
  // view buffer), and *ent_view / offsets then index the copy.
  struct BalancedOut {
    bool used = false;
    std::string reason;
    std::vector<DomainAssignment> workers, leaders;
  };
  std::vector<BalancedOut> balOut;
  std::vector<int32_t> balEnt, balCtr;
  std::vector<kueue_tas_eval_req> balReq;
  std::vector<kueue_tas_eval_out> balOuts;
  std::vector<int64_t> balOffs;
  int balanced_pass(const std::vector<const kueue_tas_eval_req*>& rq, const std::vector<int32_t>& tt,
                    const std::vector<kueue_tas_affinity_req>* af, const std::vector<int32_t>* afv,
                    const std::vector<std::pair<size_t, GroupEval*>>& bt, const int32_t** ent_view) {
    const size_t n = bt.size();
    balOut.assign(n, BalancedOut{});
    std::vector<size_t> idx;
    for (size_t i = 0; i < n; i++)
      if (bt[i].second->balanced) idx.push_back(i);
    if (idx.empty()) return 0;
    balEnt.clear();
    int64_t pos = 0;
    for (size_t i = 0; i < n; i++) {
      const int64_t cnt = outs[i].status == KUEUE_TAS_ST_OK ? int64_t(outs[i].num_workers + outs[i].num_leaders) : 0;
      balEnt.insert(balEnt.end(), *ent_view + offsets[i] * 2, *ent_view + (offsets[i] + cnt) * 2);
      offsets[i] = pos;
      pos += cnt;
    }
    offsets[n] = pos;
    *ent_view = balEnt.data();
    const FlavorSnapshot& s = *snap;
    const int L = s.L();
    size_t total = 0;
    for (int l = 0; l < L; l++) total += s.values[size_t(l)].size();
    const size_t chunk = size_t(s.cfg.max_batch > 0 ? s.cfg.max_batch : 1024);
    // the first batch's last device chunk still holds its requests' phase-1
    // counters (kueue_tas_last_counters): those are read in place; only the
    // balanced requests of earlier chunks are evaluated again
    const size_t last0 = n > 0 ? (n - 1) / chunk * chunk : 0;
    std::vector<size_t> again, here;
    for (size_t i : idx) (i >= last0 ? here : again).push_back(i);
    auto place = [&](size_t i, size_t slot) -> int {  // the counters of request `slot` of the last batch -> balOut[i]
      balCtr.resize(std::max<size_t>(5 * total, 1));
      int rc = kueue_tas_last_counters(s.ctx, slot, balCtr.data(), balCtr.size());
      if (rc) return rc;
      ktas_balanced::Tree t;
      t.L = L;
      t.ctr.resize(size_t(L));
      size_t g0 = 0;
      for (int l = 0; l < L; l++) {
        const size_t D = s.values[size_t(l)].size();
        t.size.push_back(int32_t(D));
        if (l + 1 < L) t.co.push_back(&s.childOff[size_t(l)]);
        auto& cl = t.ctr[size_t(l)];
        cl.resize(D);
        for (size_t d = 0; d < D; d++) {
          const size_t g = g0 + d;
          cl[d] = {balCtr[g], balCtr[total + g], balCtr[2 * total + g], balCtr[3 * total + g], balCtr[4 * total + g]};
        }
        g0 += D;
      }
      const kueue_tas_eval_req& q = *rq[i];
      ktas_balanced::Params p;
      p.count = q.count;
      p.sliceSize = q.slice_size;
      p.leaderCount = (q.flags & KUEUE_TAS_F_LEADER) ? 1 : 0;
      p.requestedLevelIdx = q.requested_level;
      p.sliceLevelIdx = q.slice_level;
      p.sliceSizeAtLevel = q.slice_size_at_level;
      const ktas_balanced::Result r = ktas_balanced::Placement(t, p).run();
      BalancedOut& o = balOut[i];
      o.used = r.used;
      o.reason = r.reason;
      for (auto& x : r.workers) o.workers.push_back({x.first, x.second});
      for (auto& x : r.leaders) o.leaders.push_back({x.first, x.second});
      return 0;
    };
    for (size_t i : here)
      if (int rc = place(i, i)) {  // the batch index: the last chunk's requests keep theirs
        snap->err = std::string("balanced placement: ") + kueue_tas_last_error(s.ctx);
        return rc;
      }
    for (size_t c0 = 0; c0 < again.size(); c0 += chunk) {  // every request of a call in one device chunk
      const size_t m = std::min(chunk, again.size() - c0);
      balReq.clear();
      for (size_t k = 0; k < m; k++) balReq.push_back(*rq[again[c0 + k]]);
      balOuts.resize(m);
      balOffs.resize(m + 1);
      int rc = kueue_tas_eval_batch(s.ctx, balReq.data(), m, tt.data(), tt.size(), int32_t(s.taintStrings.size()),
                                    assumed.data(), assumed.size(), af->data(), af->size(), afv->data(), afv->size(),
                                    balOuts.data(), balOffs.data(), nullptr, 0, nullptr, nullptr);
      for (size_t k = 0; k < m && rc == 0; k++) rc = place(again[c0 + k], k);
      if (rc) {
        snap->err = std::string("balanced placement: ") + kueue_tas_last_error(s.ctx);
        return rc;
      }
    }
    return 0;
  }

  // base: optional per-workload starting overlay, records sorted by (leaf,
  // column) with distinct keys, subtracted from the remaining capacity: the
  // negated usage of the workloads a preemption candidate set removes
  // (SimulateUsageRemoval).
  using Overlay = std::vector<kueue_tas_assumed>;
  const std::vector<Overlay>* base = nullptr;
  int run(std::vector<Workload>& wls, bool simulateEmpty, std::vector<std::vector<PodSetResult>>* results,
          bool precompiled = false, const std::vector<Overlay>* base_overlay = nullptr, bool regroup = false) {
    base = base_overlay;
    ms[0] = ms[1] = ms[2] = ms[3] = 0;
    for (auto& v : stage_ms) v = 0;
    for (auto& v : dev_host_ms) v = 0;
    counts[0] = counts[1] = counts[2] = 0;
    stats[0] = stats[1] = stats[2] = stats[3] = stats[4] = stats[5] = 0;
    host_ms[0] = host_ms[1] = host_ms[2] = host_ms[3] = 0;
    detail_ms[0] = detail_ms[1] = detail_ms[2] = detail_ms[3] = 0;
    const double t_start = now_ms();
    double t_prep = t_start;  // start of the current pass's preparation
    results->resize(wls.size());
    used.assign(wls.size(), 0);
    if (!precompiled) {
      // grouping (FindTopologyAssignmentsForFlavor :528-541) and the
      // findTopologyAssignment prelude (:804-897) per workload, over the host
      // pool: every workload writes only its own groups; new resource
      // columns (rare: they reload the snapshot) are added serially between
      HostPool& pool = HostPool::get();
      std::atomic<bool> unknown{false};
      pool.run_static(wls.size(), [&](size_t b, size_t e) {
        bool u = false;
        for (size_t w = b; w < e; w++) {
          if (wls[w].groups.empty() || regroup) make_groups(wls[w]);
          u = u || !snap->columns_known(wls[w].podsets);
        }
        if (u) unknown.store(true, std::memory_order_relaxed);
      });
      bool changed = false;
      if (unknown.load())
        for (auto& wl : wls) changed |= snap->ensure_columns_for(wl.podsets);
      const double t_c = now_ms();
      detail_ms[0] += t_c - t_start;
      snap->compile_gen++;
      std::string perr;
      std::mutex perr_mu;
      pool.run_static(wls.size(), [&](size_t b, size_t e) {
        try {
          for (size_t w = b; w < e; w++)
            for (auto& g : wls[w].groups)
              if (!g.compiled || changed) snap->compile_group_only(g, simulateEmpty);
        } catch (const std::exception& x) {
          std::lock_guard<std::mutex> lk(perr_mu);
          if (perr.empty()) perr = x.what();
        }
      });
      if (!perr.empty()) throw std::runtime_error(perr);
      detail_ms[1] += now_ms() - t_c;
    }
    int rc = snap->upload();  // (re)load when columns were added
    if (rc) return rc;
    std::vector<char> done(wls.size(), 0);
    std::vector<AssumedUsage> assumedBy(wls.size());
    size_t maxGroups = 0;
    for (auto& wl : wls) maxGroups = std::max(maxGroups, wl.groups.size());
    const size_t T = snap->taintStrings.size();
    const size_t R = snap->cols.size();
    std::vector<std::pair<size_t, GroupEval*>> early;
    for (size_t pass = 0; pass < maxGroups; pass++) {
      const std::vector<const kueue_tas_eval_req*>* rq = &reqs;
      const std::vector<int32_t>* tt = &taint_table;
      const std::vector<kueue_tas_affinity_req>* af = &aff;
      const std::vector<int32_t>* afv = &affv;
      const std::vector<std::pair<size_t, GroupEval*>>* bt = &batch;
      const std::vector<std::pair<size_t, GroupEval*>>* ea = &early;
      const double t_bp = now_ms();
      if (pass == 0 && precompiled && !base) {  // no assumed usage yet: reuse the compiled first pass
        if (p0_for != &wls || p0_gen != snap->compile_gen) {
          build_pass(wls, 0, done, assumedBy, p0_reqs, p0_taint, assumed, p0_aff, p0_affv, p0_batch, p0_early);
          p0_for = &wls;
          p0_gen = snap->compile_gen;
        }
        rq = &p0_reqs;
        tt = &p0_taint;
        af = &p0_aff;
        afv = &p0_affv;
        bt = &p0_batch;
        ea = &p0_early;
        assumed.clear();
      } else if (pass == 0 && !base) {
        build_pass0_static(wls, done, reqs, taint_table, assumed, aff, affv, batch, early);
        p0_for = nullptr;  // the groups' records now hold this batch's table offsets
      } else {
        build_pass(wls, pass, done, assumedBy, reqs, taint_table, assumed, aff, affv, batch, early);
        if (pass == 0) p0_for = nullptr;
      }
      detail_ms[2] += now_ms() - t_bp;
      for (auto& we : *ea) {
        for (auto* m : we.second->members)
          set_result((*results)[we.first], used[we.first], m->name, false, nullptr, 0, we.second->early_reason);
        done[we.first] = 1;
      }
      if (bt->empty()) continue;
      if (pass > 0)  // the next batch reuses the entries buffer the earlier views point into
        for (size_t w = 0; w < wls.size(); w++)
          for (size_t k = 0; k < used[w]; k++) (*results)[w][k].materialize();
      const double t_call = now_ms();
      host_ms[0] += t_call - t_prep;  // this pass's preparation only
      const size_t n = bt->size();
      outs.resize(n);
      offsets.resize(n + 1);
      taint_counts.resize(n * std::max<size_t>(T, 1));
      res_counts.resize(n * R);
      const bool packed = (snap->cfg.flags & KUEUE_TAS_CFG_PACKED_ENTRIES) != 0;
      if (packed && entries.size() < 2 * 64 * n) entries.resize(2 * 64 * n);
      rc = kueue_tas_eval_batch_ptrs(snap->ctx, rq->data(), n, tt->data(), tt->size(), int32_t(T), assumed.data(),
                                assumed.size(), af->data(), af->size(), afv->data(), afv->size(), outs.data(), offsets.data(), packed ? entries.data() : nullptr,
                                packed ? entries.size() / 2 : 0, taint_counts.data(), res_counts.data());
      if (rc == KUEUE_TAS_EOVERFLOW && packed) {
        entries.resize(size_t(offsets[n]) * 2 + 2);
        rc = kueue_tas_fetch_entries(snap->ctx, entries.data(), entries.size() / 2);
      }
      if (rc) {
        snap->err = std::string("eval: ") + kueue_tas_last_error(snap->ctx);
        return rc;
      }
      // zero-copy view (pinned, strided regions) or the packed copy
      const int32_t* ent_view = packed ? entries.data() : kueue_tas_last_entries(snap->ctx, nullptr);
      float t4[4];
      kueue_tas_last_timings(snap->ctx, t4);
      for (int k = 0; k < 4; k++) ms[k] += t4[k];
      float st[KUEUE_TAS_NUM_STAGES];
      kueue_tas_last_stage_times(snap->ctx, st, KUEUE_TAS_NUM_STAGES);
      for (int k = 0; k < KUEUE_TAS_NUM_STAGES; k++) stage_ms[k] += st[k];
      double ht[8];
      kueue_tas_last_host_times(snap->ctx, ht, 8);
      for (int k = 0; k < 8; k++) dev_host_ms[k] += ht[k];
      int64_t st4[4];
      kueue_tas_last_stats(snap->ctx, st4);
      for (int k = 0; k < 3; k++) stats[k] += st4[k];
      stats[3] = std::max(stats[3], st4[3]);
      stats[4] |= int64_t(kueue_tas_last_fill_paths(snap->ctx));
      stats[5] += kueue_tas_last_alias_fills(snap->ctx);
      rc = balanced_pass(*rq, *tt, af, afv, *bt, &ent_view);  // after the diagnostics: it may run a batch
      if (rc) return rc;
      const double t_decode = now_ms();
      host_ms[1] += t_decode - t_call;
      counts[0]++;
      counts[1] += int64_t(n);
      // decode: every eval of the pass writes only its own workload's
      // results, assumed usage and done flag, so the evals decode in parallel
      // (the failure-text caches are filled first: they are shared)
      snap->reason_order();
      (void)snap->topology_quoted();
      std::atomic<int64_t> leaders{0};
      HostPool::get().run_static(n, [&](size_t i0, size_t i1) {
      std::string reasonBuf;
      int64_t nlead = 0;
      for (size_t i = i0; i < i1; i++) {
        const size_t w = (*bt)[i].first;
        GroupEval& g = *(*bt)[i].second;
        const kueue_tas_eval_out& o = outs[i];
        nlead += (g.req.flags & KUEUE_TAS_F_LEADER) ? 1 : 0;
        const BalancedOut* bo = g.balanced && balOut[i].used ? &balOut[i] : nullptr;
        if (bo && !bo->reason.empty()) {  // TAS Balanced Placement failure (tas_balanced_placement.go:149-184, :295-314)
          for (auto* m : g.members) set_result((*results)[w], used[w], m->name, false, nullptr, 0, bo->reason);
          done[w] = 1;
          continue;
        }
        if (!bo && o.status != KUEUE_TAS_ST_OK) {
          snap->failure_reason(reasonBuf, g, o, taint_counts.data() + i * std::max<size_t>(T, 1), res_counts.data() + i * R);
          for (auto* m : g.members) set_result((*results)[w], used[w], m->name, false, nullptr, 0, reasonBuf);
          done[w] = 1;
          continue;
        }
        const DomainAssignment* e = bo ? bo->workers.data()
                                       : reinterpret_cast<const DomainAssignment*>(ent_view + size_t(offsets[i]) * 2);
        const int32_t nw = bo ? int32_t(bo->workers.size()) : o.num_workers;
        const int32_t nl = bo ? int32_t(bo->leaders.size()) : o.num_leaders;
        const DomainAssignment* ld = bo ? bo->leaders.data() : e + o.num_workers;
        // addAssumedUsage (:658-666) only matters for the workload's later groups:
        // SinglePodRequests x count (no pods term)
        if (pass + 1 < wls[w].groups.size()) {
          auto add = [&](const TASPodSetRequests* tr, const DomainAssignment* ds, int32_t nd) {
            for (int32_t k = 0; k < nd; k++)
              for (auto& kv : tr->requestIds)
                assumedBy[w].add(ds[k].leaf, snap->col_of(kv.first), mul64(kv.second, ds[k].count));
          };
          add(g.workers, e, nw);
          if (g.leader) add(g.leader, ld, nl);
        }
        static const std::string kEmpty;
        for (auto* m : g.members) {
          if (m == g.workers) set_result((*results)[w], used[w], m->name, true, e, size_t(nw), kEmpty);
          else if (m == g.leader) set_result((*results)[w], used[w], m->name, true, ld, size_t(nl), kEmpty);
          else set_result((*results)[w], used[w], m->name, false, nullptr, 0, kEmpty);
        }
        if (bo)  // the balanced result lives in balOut until the next batch
          for (size_t k = 0; k < used[w]; k++) (*results)[w][k].materialize();
      }
      leaders.fetch_add(nlead, std::memory_order_relaxed);
      });
      counts[2] += leaders.load();
      t_prep = now_ms();
      host_ms[2] += t_prep - t_decode;
    }
    for (size_t w = 0; w < wls.size(); w++) (*results)[w].resize(used[w]);
    host_ms[3] = now_ms() - t_start;
    return 0;
  }
};

static void emit_results(std::string& out, const FlavorSnapshot& s, const std::vector<PodSetResult>& rs) {
  out += "[";
  const int L = s.L();
  const size_t levelIdx = s.lowestIsHostname ? size_t(L - 1) : 0;
  for (size_t i = 0; i < rs.size(); i++) {
    if (i) out += ",";
    out += "{\"name\":";
    kjson::write_string(out, rs[i].name);
    out += ",\"assignment\":";
    if (!rs[i].has_assignment) {
      out += "null";
    } else {
      out += "{\"levels\":[";
      for (size_t l = levelIdx; l < size_t(L); l++) {
        if (l > levelIdx) out += ",";
        kjson::write_string(out, s.levelKeys[l]);
      }
      out += "],\"domains\":[";
      for (size_t k = 0; k < rs[i].domains.size(); k++) {
        if (k) out += ",";
        out += "{\"values\":[";
        const auto& lv = s.values[L - 1][rs[i].domains[k].leaf];
        for (size_t l = levelIdx; l < lv.size(); l++) {
          if (l > levelIdx) out += ",";
          kjson::write_string(out, l == size_t(L - 1) && s.lowestIsHostname ? s.leafId[rs[i].domains[k].leaf] : lv[l]);
        }
        out += "],\"count\":" + std::to_string(rs[i].domains[k].count) + "}";
      }
      out += "]}";
    }
    out += ",\"reason\":";
    kjson::write_string(out, rs[i].reason);
    out += "}";
  }
  out += "]";
}

// ---- v1beta2 TopologyAssignment (apis/kueue/v1beta2; tas_assignment.go:135-259) ----
// One single-slice encoding from the device's per-level lengths; value(j, k)
// is domain j's value at encoding level k.
template <class ValueAt, class CountAt>
static void write_v1beta2(std::string& out, const std::vector<std::string>& levels, size_t n,
                          const kueue_tas_level_enc* enc, int32_t same, ValueAt value, CountAt count) {
  out += "{\"levels\":[";
  for (size_t l = 0; l < levels.size(); l++) {
    if (l) out += ",";
    kjson::write_string(out, levels[l]);
  }
  out += "],\"slices\":[";
  if (n == 0) {
    out += "]}";
    return;
  }
  out += "{\"domainCount\":" + std::to_string(n) + ",\"podCounts\":";
  if (same) {
    out += "{\"universal\":" + std::to_string(count(0)) + "}";
  } else {
    out += "{\"individual\":[";
    for (size_t j = 0; j < n; j++) out += (j ? "," : "") + std::to_string(count(j));
    out += "]}";
  }
  out += ",\"valuesPerLevel\":[";
  for (size_t k = 0; k < levels.size(); k++) {
    if (k) out += ",";
    const kueue_tas_level_enc& e = enc[k];
    const std::string_view v0 = value(0, k);
    if (e.universal) {
      out += "{\"universal\":";
      kjson::write_string(out, v0);
      out += "}";
      continue;
    }
    out += "{\"individual\":{";
    if (e.prefix_len > 0) {
      out += "\"prefix\":";
      kjson::write_string(out, v0.substr(0, size_t(e.prefix_len)));
      out += ",";
    }
    if (e.suffix_len > 0) {
      out += "\"suffix\":";
      kjson::write_string(out, v0.substr(v0.size() - size_t(e.suffix_len)));
      out += ",";
    }
    out += "\"roots\":[";
    for (size_t j = 0; j < n; j++) {
      if (j) out += ",";
      const std::string_view vj = value(j, k);
      kjson::write_string(out, vj.substr(size_t(e.prefix_len), vj.size() - size_t(e.prefix_len) - size_t(e.suffix_len)));
    }
    out += "]}}";
  }
  out += "]}]}";
}

// V1Beta2From of the snapshot's results (leaf mode, resident names): one
// device launch for every assignment of `rs`; writes [v1beta2 | null] per result.
static int encode_results(FlavorSnapshot& s, const std::vector<const PodSetResult*>& rs, std::vector<std::string>* out) {
  const int L = s.L();
  const int first = s.lowestIsHostname ? L - 1 : 0;
  std::vector<int32_t> pairs;
  std::vector<int64_t> off(1, 0);
  std::vector<size_t> which;
  for (size_t i = 0; i < rs.size(); i++) {
    if (!rs[i]->has_assignment) continue;
    for (auto& d : rs[i]->domains) {
      pairs.push_back(d.leaf);
      pairs.push_back(d.count);
    }
    off.push_back(int64_t(pairs.size() / 2));
    which.push_back(i);
  }
  const int nl = L - first;
  std::vector<kueue_tas_level_enc> enc(which.size() * size_t(nl));
  std::vector<int32_t> same(which.size());
  if (!which.empty()) {
    if (s.namesStale)
      if (int rc = s.load_names()) return rc;
    int rc = kueue_tas_encode_v1beta2_leaves(s.ctx, pairs.data(), off.data(), which.size(), first, enc.data(),
                                             same.data());
    if (rc) {
      s.err = std::string("encode: ") + kueue_tas_last_error(s.ctx);
      return rc;
    }
  }
  std::vector<std::string> levels(s.levelKeys.begin() + first, s.levelKeys.end());
  out->assign(rs.size(), "null");
  // The strings are the host's share (Go would allocate them too): independent
  // per assignment, so large batches are split over threads by domain count.
  auto write_range = [&](size_t a0, size_t a1) {
    for (size_t a = a0; a < a1; a++) {
      const DomainSpan& d = rs[which[a]]->domains;
      std::string& o = (*out)[which[a]];
      o.clear();
      o.reserve(d.size() * (levels.size() * 24 + 8) + 64);
      write_v1beta2(
          o, levels, d.size(), enc.data() + a * size_t(nl), same[a],
          [&](size_t j, size_t k) -> std::string_view {
            const auto& lv = s.values[L - 1][size_t(d[j].leaf)];
            return lv[size_t(first) + k];
          },
          [&](size_t j) { return d[j].count; });
    }
  };
  const size_t total = size_t(off.back());
  const size_t nthreads = std::min<size_t>({8, std::max<unsigned>(1, std::thread::hardware_concurrency()),
                                            total / 8192 + 1, which.size()});
  if (nthreads <= 1) {
    write_range(0, which.size());
    return 0;
  }
  std::vector<std::thread> pool;
  size_t a0 = 0;
  for (size_t t = 0; t < nthreads && a0 < which.size(); t++) {
    const size_t goal = total * (t + 1) / nthreads;  // domain-balanced cut
    size_t a1 = a0 + 1;
    while (a1 < which.size() && size_t(off[a1]) < goal) a1++;
    if (t + 1 == nthreads) a1 = which.size();
    pool.emplace_back(write_range, a0, a1);
    a0 = a1;
  }
  for (auto& th : pool) th.join();
  return 0;
}

// V1Beta2From over explicit internal assignments (explicit-string mode).
static int v1beta2_from_json(kueue_tas_ctx* ctx, const kjson::Node& arr, std::string* out, std::string* err) {
  std::string bytes;
  std::vector<int64_t> str_off(1, 0);
  std::vector<int32_t> ids, counts;
  std::vector<int64_t> off(1, 0);
  struct Item {
    bool null;
    std::vector<std::string> levels;
    size_t first_dom, first_id, n;  // string ids of domain j, level k: first_id + j * levels + k
  };
  std::vector<Item> items;
  std::vector<int32_t> nlev;
  size_t ndom = 0;
  for (auto& ta : arr.items) {
    Item it{ta.null(), {}, ndom, ids.size(), 0};
    if (!it.null) {
      for (auto& l : ta["levels"].items) it.levels.push_back(l.s());
      for (auto& d : ta["domains"].items) {
        if (d["values"].items.size() != it.levels.size()) throw std::runtime_error("values/levels length mismatch");
        for (auto& v : d["values"].items) {
          ids.push_back(int32_t(str_off.size() - 1));
          bytes += v.s();
          str_off.push_back(int64_t(bytes.size()));
        }
        counts.push_back(int32_t(d["count"].i64()));
        it.n++;
      }
    }
    ndom += it.n;
    items.push_back(std::move(it));
  }
  // one launch per distinct level count (assignments of one batch share it)
  std::vector<std::vector<kueue_tas_level_enc>> enc(items.size());
  std::vector<int32_t> same(items.size(), 0);
  std::map<size_t, std::vector<size_t>> by_levels;
  for (size_t i = 0; i < items.size(); i++)
    if (!items[i].null && !items[i].levels.empty()) by_levels[items[i].levels.size()].push_back(i);
  for (auto& kv : by_levels) {
    const size_t nl = kv.first;
    std::vector<int32_t> gids, gcounts;
    std::vector<int64_t> goff(1, 0);
    for (size_t i : kv.second) {
      const Item& it = items[i];
      gids.insert(gids.end(), ids.begin() + int64_t(it.first_id), ids.begin() + int64_t(it.first_id + it.n * nl));
      gcounts.insert(gcounts.end(), counts.begin() + int64_t(it.first_dom), counts.begin() + int64_t(it.first_dom + it.n));
      goff.push_back(int64_t(gcounts.size()));
    }
    std::vector<kueue_tas_level_enc> e(kv.second.size() * nl);
    std::vector<int32_t> sm(kv.second.size());
    int rc = kueue_tas_encode_v1beta2(ctx, bytes.data(), bytes.size(), str_off.data(), str_off.size() - 1, gids.data(),
                                      gcounts.data(), goff.data(), kv.second.size(), int32_t(nl), e.data(), sm.data());
    if (rc) {
      *err = std::string("encode: ") + kueue_tas_last_error(ctx);
      return rc;
    }
    for (size_t q = 0; q < kv.second.size(); q++) {
      enc[kv.second[q]].assign(e.begin() + int64_t(q * nl), e.begin() + int64_t((q + 1) * nl));
      same[kv.second[q]] = sm[q];
    }
  }
  *out = "[";
  for (size_t i = 0; i < items.size(); i++) {
    if (i) *out += ",";
    const Item& it = items[i];
    if (it.null) {
      *out += "null";
      continue;
    }
    const size_t nl = it.levels.size();
    if (nl == 0) {  // no levels: only the slice shape and pod counts remain
      *out += "{\"levels\":[],\"slices\":[";
      if (it.n) {
        bool eq = true;
        for (size_t j = 1; j < it.n; j++) eq = eq && counts[it.first_dom + j] == counts[it.first_dom];
        *out += "{\"domainCount\":" + std::to_string(it.n) + ",\"podCounts\":";
        if (eq) {
          *out += "{\"universal\":" + std::to_string(counts[it.first_dom]) + "}";
        } else {
          *out += "{\"individual\":[";
          for (size_t j = 0; j < it.n; j++) *out += (j ? "," : "") + std::to_string(counts[it.first_dom + j]);
          *out += "]}";
        }
        *out += ",\"valuesPerLevel\":[]}";
      }
      *out += "]}";
      continue;
    }
    write_v1beta2(
        *out, it.levels, it.n, enc[i].data(), same[i],
        [&](size_t j, size_t k) -> std::string_view {
          const size_t sid = it.first_id + j * nl + k;
          return std::string_view(bytes.data() + str_off[sid], size_t(str_off[sid + 1] - str_off[sid]));
        },
        [&](size_t j) { return counts[it.first_dom + j]; });
  }
  *out += "]";
  return 0;
}

// InternalFrom / InternalSeqFrom (tas_assignment.go:103-133): wire format ->
// internal assignment (string expansion only; runs where the JSON is).
static void internal_from_json(const kjson::Node& arr, std::string* out) {
  *out = "[";
  bool first_item = true;
  for (auto& ta : arr.items) {
    if (!first_item) *out += ",";
    first_item = false;
    if (ta.null()) {
      *out += "null";
      continue;
    }
    const auto& levels = ta["levels"].items;
    *out += "{\"levels\":[";
    for (size_t l = 0; l < levels.size(); l++) {
      if (l) *out += ",";
      kjson::write_string(*out, levels[l].s());
    }
    *out += "],\"domains\":[";
    bool first = true;
    for (auto& sl : ta["slices"].items) {
      const int64_t dc = sl["domainCount"].i64();
      const kjson::Node& pc = sl["podCounts"];
      const kjson::Node* uc = pc.find("universal");
      for (int64_t i = 0; i < dc; i++) {
        if (!first) *out += ",";
        first = false;
        *out += "{\"values\":[";
        for (size_t l = 0; l < levels.size(); l++) {
          const kjson::Node& v = sl["valuesPerLevel"].items.at(l);
          std::string val;
          if (const kjson::Node* u = v.find("universal")) {  // valueAtIndex (:40-48)
            val = u->s();
          } else {
            const kjson::Node& ind = v["individual"];
            const kjson::Node* p = ind.find("prefix");
            const kjson::Node* x = ind.find("suffix");
            val = (p ? p->s() : std::string()) + ind["roots"].items.at(size_t(i)).s() + (x ? x->s() : std::string());
          }
          if (l) *out += ",";
          kjson::write_string(*out, val);
        }
        const int64_t c = uc ? uc->i64() : pc["individual"].items.at(size_t(i)).i64();  // countAtIndex (:50-55)
        *out += "],\"count\":" + std::to_string(c) + "}";
      }
    }
    *out += "]}";
  }
  *out += "]";
}

static char* dup(const std::string& s) {
  char* p = static_cast<char*>(malloc(s.size() + 1));
  memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

}  // namespace kueue_tas

using namespace kueue_tas;

struct kueue_tas_host {
  std::unique_ptr<FlavorSnapshot> snap;
  std::string err;
  std::vector<Workload> compiled;
  uint64_t compiled_gen = 0;  // bumped when the compiled workload set is replaced
  std::unique_ptr<Evaluator> ev;
  std::vector<std::vector<PodSetResult>> last;
  float ms[4] = {0, 0, 0, 0};
  int64_t counts[3] = {0, 0, 0};
  int64_t stats[6] = {0, 0, 0, 0, 0, 0};
  uint64_t compiled_cols = 0;  // FlavorSnapshot::col_gen the compiled workloads were compiled against
  // this rank's shard of the compiled workloads (indices into `compiled`)
  // and its own compiled copies; empty: run_compiled evaluates them all
  std::vector<int32_t> shard_ids;
  std::vector<Workload> shard;
  std::vector<Workload>& active() { return shard_ids.empty() ? compiled : shard; }
  std::vector<kueue_tas_delta> last_deltas;  // usage deltas the last kueue_tas_host_admit applied
  double admit_ms[3] = {0, 0, 0};            // last admit: host prep, kueue_tas_admit, delta list
  // admit's working storage (kept between rounds)
  std::vector<int32_t> admit_seen, admit_ids, admit_adm;
  std::array<uint64_t, 3> admit_table_key{0, 0, 0};  // (compiled set, compile_gen, col_gen) of the device admission table
  std::vector<int32_t> admit_pseen;  // [part][workload] of the record passes on the host pool
  std::vector<int64_t> admit_pcnt;
  std::vector<int64_t> admit_start, admit_off;
  std::vector<std::array<int32_t, 3>> admit_doms;
  std::vector<kueue_tas_fits_req> admit_fr;
  std::vector<kueue_tas_fits_term> admit_terms;
  std::vector<int64_t> admit_toff;  // per admitted-round workload: first term
  std::vector<PodSetResult*> values_rest;  // RUN_VALUES: results whose Values the host builds
  std::vector<const std::string*> values_flat;  // host-built Values pointers in the entry view's layout
  float stage_accum[KUEUE_TAS_NUM_STAGES] = {};  // kueue_tas_host_stage_accum
  // last kueue_tas_host_update_nodes: parse, node events, flush_joins, splice
  // (host rows, device call, leaf tags), evaluator reset, pushes, total, and
  // flush_joins' parts (host-mirror fold, levels + CSR, leaf arrays, maps + ranks)
  double upd_ms[13] = {};
  int64_t accum_runs = 0, accum_fills = 0;
  void recompile_all() {
    for (auto& wl : compiled) snap->ensure_columns_for(wl.podsets);
    for (auto* v : {&compiled, &shard})
      for (auto& wl : *v)
        for (auto& g : wl.groups) snap->compile_group(g, false);
    compiled_cols = snap->col_gen;
  }
};

extern "C" {

kueue_tas_host* kueue_tas_host_create(const char* snapshot_json, const kueue_tas_config* cfg) {
  auto* h = new kueue_tas_host();
  try {
    h->snap = std::make_unique<FlavorSnapshot>();
    if (cfg) h->snap->cfg = *cfg;
    kjson::Node c = kjson::parse(snapshot_json);
    h->snap->build(c);
    if (h->snap->upload()) {
      h->err = h->snap->err;
      return h;
    }
  } catch (const std::exception& e) {
    h->err = e.what();
  }
  return h;
}

void kueue_tas_host_destroy(kueue_tas_host* h) { delete h; }

const char* kueue_tas_host_last_error(kueue_tas_host* h) { return h ? h->err.c_str() : "null host"; }

// ---- node replacement (tas_flavor_snapshot.go:546-562, :614-678) ----------
struct Replacement {
  const kueue_tas_host* h;
  FlavorSnapshot& s;
  static int32_t go_mod32(int32_t a, int32_t b) {
    if (b == 0) throw std::runtime_error("panic: runtime error: integer divide by zero");
    return b == -1 ? 0 : a % b;
  }
  static bool slices_requested(const std::optional<TopologyRequest>& tr) {  // :1155-1160
    return tr && ((tr->sliceRequiredTopology && tr->sliceSize) || !tr->constraints.empty());
  }
  static int32_t slice_size(const std::optional<TopologyRequest>& tr) {  // getSliceSizeWithSinglePodAsDefault
    if (!tr) return 1;
    if (!tr->constraints.empty()) return tr->constraints[0].size;
    if (!tr->sliceRequiredTopology) return 1;
    return tr->sliceSize ? *tr->sliceSize : 0;
  }
  // the leaf behind DomainID(values) at the node level (domainsPerLevel[nodeLevel]), or -1
  int32_t leaf_of(const std::vector<std::string>& values) const {
    return s.live_leaf(join_values(values));
  }
  // domain.id of the leaf's ancestor at `level` (the leaf's own id at the node level)
  std::string ancestor_id(int32_t leaf, int level) const {
    if (level == s.L() - 1) return s.leafId[size_t(leaf)];
    const auto& lv = s.values[size_t(s.L() - 1)][size_t(leaf)];
    return join_values(std::vector<std::string>(lv.begin(), lv.begin() + level + 1));
  }
  // findIncompleteSliceDomain (:760-792); the first qualifying domain in
  // assignment order (Go ranges over a map: random among several)
  std::string incomplete_slice_domain(const ExplicitAssignment& ta, int32_t missing, int32_t sliceSize,
                                      const std::string& topologyKey) const {
    const int sliceLevel = s.resolve(topologyKey);
    if (sliceLevel < 0) return "";
    std::vector<std::string> order;
    std::map<std::string, int32_t> usage;
    for (auto& d : ta.domains) {
      const int32_t leaf = leaf_of(d.first);
      if (leaf < 0) continue;
      const std::string id = ancestor_id(leaf, sliceLevel);
      if (!usage.count(id)) order.push_back(id);
      usage[id] = int32_t(uint32_t(usage[id]) + uint32_t(d.second));
    }
    for (auto& id : order)
      if (go_mod32(int32_t(uint32_t(usage[id]) + uint32_t(missing)), sliceSize) == 0) return id;
    return "";
  }
  // requiredReplacementDomain (:680-731)
  std::string required_domain(const TASPodSetRequests& tr, const ExplicitAssignment& ta) const {
    const std::string* key = s.level_key(tr);
    if (!key) return "";
    const int levelIdx = s.resolve(*key);
    if (levelIdx < 0 || ta.domains.empty()) return "";
    const auto& req = tr.topologyRequest;
    const int32_t ss = slice_size(req);
    if (slices_requested(req) && go_mod32(tr.count, ss) != 0) {
      const auto& cs = req->constraints;
      if (cs.size() > 1)
        for (size_t i = cs.size(); i-- > 0;)
          if (go_mod32(tr.count, cs[i].size) != 0) return incomplete_slice_domain(ta, tr.count, cs[i].size, cs[i].topology);
      const std::string sliceKey = req->sliceRequiredTopology ? *req->sliceRequiredTopology
                                   : !req->constraints.empty() ? req->constraints[0].topology
                                                               : s.levelKeys.back();
      return incomplete_slice_domain(ta, tr.count, ss, sliceKey);
    }
    if (!(req && req->required)) return "";
    if (ta.domains[0].first.empty()) return "";
    const int32_t leaf = leaf_of(ta.domains[0].first);
    return leaf < 0 ? "" : ancestor_id(leaf, levelIdx);
  }
  // belongsToRequiredDomain (:1649-1656) as a leaf index range: the leaves
  // whose DomainID(levelValues) starts with `id` (lexicographic leaf order
  // keeps them contiguous; checked)
  void domain_range(const std::string& id, int32_t* begin, int32_t* end) const {
    int32_t lo = -1, hi = -1;
    for (int32_t i = 0; i < s.N(); i++) {
      const std::string d = join_values(s.values[size_t(s.L() - 1)][size_t(i)]);
      if (d.compare(0, id.size(), id) != 0) continue;
      if (lo < 0) lo = i;
      else if (hi != i) throw std::runtime_error("internal: required replacement domain is not one leaf range");
      hi = i + 1;
    }
    *begin = lo < 0 ? 0 : lo;
    *end = lo < 0 ? 0 : hi;
  }
  // mergeTopologyAssignments (:1796-1826)
  ExplicitAssignment merge(const ExplicitAssignment& a, const ExplicitAssignment& b) const {
    std::vector<std::pair<std::string, const std::pair<std::vector<std::string>, int32_t>*>> keyed;
    for (auto* ta : {&a, &b})
      for (auto& d : ta->domains) {
        const int32_t leaf = leaf_of(d.first);
        if (leaf < 0) throw std::runtime_error("panic: runtime error: invalid memory address or nil pointer dereference");
        keyed.push_back({join_values(s.values[size_t(s.L() - 1)][size_t(leaf)]), &d});
      }
    std::stable_sort(keyed.begin(), keyed.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    ExplicitAssignment out;
    out.levels = a.levels;
    for (auto& kd : keyed) {
      if (!out.domains.empty() && join_values(out.domains.back().first) == join_values(kd.second->first))
        out.domains.back().second = int32_t(uint32_t(out.domains.back().second) + uint32_t(kd.second->second));
      else
        out.domains.push_back(*kd.second);
    }
    return out;
  }
};

static void emit_explicit(std::string& out, const std::string& name, const std::optional<ExplicitAssignment>& a,
                          const std::string& reason) {
  out += "{\"name\":";
  kjson::write_string(out, name);
  out += ",\"assignment\":";
  if (!a) {
    out += "null";
  } else {
    out += "{\"levels\":[";
    for (size_t l = 0; l < a->levels.size(); l++) {
      if (l) out += ",";
      kjson::write_string(out, a->levels[l]);
    }
    out += "],\"domains\":[";
    for (size_t k = 0; k < a->domains.size(); k++) {
      if (k) out += ",";
      out += "{\"values\":[";
      for (size_t j = 0; j < a->domains[k].first.size(); j++) {
        if (j) out += ",";
        kjson::write_string(out, a->domains[k].first[j]);
      }
      out += "],\"count\":" + std::to_string(a->domains[k].second) + "}";
    }
    out += "]}";
  }
  out += ",\"reason\":";
  kjson::write_string(out, reason);
  out += "}";
}

// FindTopologyAssignmentsForFlavor with a workload in node replacement
// (HasUnhealthyNodes, :546-562): per group, per PodSet with an existing
// assignment, findReplacementAssignment (:614-656) — deleteDomain,
// IsTopologyAssignmentStale, requiredReplacementDomain, the slice
// adjustment, one device evaluation of the replacement pods with the
// required domain's leaf range and the replacements so far as assumed
// usage, mergeTopologyAssignments.
static int find_replacement(kueue_tas_host* h, std::vector<TASPodSetRequests>& podsets,
                            const std::string& unhealthy, const std::map<std::string, ExplicitAssignment>& psa,
                            std::string* out) {
  FlavorSnapshot& s = *h->snap;
  Replacement R{h, s};
  Workload wl;
  wl.podsets = podsets;
  make_groups(wl);
  s.ensure_columns_for(wl.podsets);  // assumed usage is kept per column
  std::map<std::pair<int32_t, int32_t>, int64_t> assumed;  // (leaf, column) -> addAssumedUsage
  std::vector<std::string> results;
  auto finish = [&]() {
    *out = "{\"results\":[";
    for (size_t i = 0; i < results.size(); i++) *out += (i ? "," : "") + results[i];
    *out += "]}";
    return 0;
  };
  for (auto& g : wl.groups) {
    for (const TASPodSetRequests* m : g.members) {
      auto p = psa.find(m->name);
      if (p == psa.end()) continue;
      ExplicitAssignment existing = p->second;
      TASPodSetRequests tr = *m;
      std::string reason;
      std::optional<ExplicitAssignment> merged, replacement;
      try {
        // deleteDomain (:746-758)
        int32_t affected = 0;
        std::vector<std::pair<std::vector<std::string>, int32_t>> kept;
        for (auto& d : existing.domains) {
          if (!d.first.empty() && d.first.back() == unhealthy) affected = d.second;
          else kept.push_back(d);
        }
        existing.domains = kept;
        tr.count = affected;
        for (auto& d : existing.domains)  // IsTopologyAssignmentStale (:733-743)
          if (!s.has_domain(join_values(d.first))) {
            reason = "Cannot replace the node, because the existing topologyAssignment is invalid, as it contains the "
                     "stale domain " + (d.first.empty() ? std::string() : d.first[0]);
            break;
          }
        if (reason.empty()) {
          const std::string reqDomain = R.required_domain(tr, existing);
          TASPodSetRequests trCopy = tr;
          if (Replacement::slices_requested(tr.topologyRequest) && !reqDomain.empty() &&
              Replacement::go_mod32(tr.count, Replacement::slice_size(tr.topologyRequest)) != 0) {
            int32_t effSize = 1;
            std::optional<std::string> effTopo;
            const auto& cs = tr.topologyRequest->constraints;
            for (size_t i = cs.size(); i-- > 0;)
              if (Replacement::go_mod32(tr.count, cs[i].size) == 0) {
                effSize = cs[i].size;
                effTopo = cs[i].topology;
                break;
              }
            trCopy.topologyRequest->constraints.clear();
            trCopy.topologyRequest->sliceRequiredTopology = effTopo;
            trCopy.topologyRequest->sliceSize = effSize;
          }
          // findTopologyAssignment(trCopy, nil, assumedUsage, false, requiredReplacementDomain)
          std::vector<Workload> one(1);
          one[0].podsets.push_back(trCopy);
          make_groups(one[0]);
          s.ensure_columns_for(one[0].podsets);
          GroupEval& ge = one[0].groups[0];
          s.compile_group(ge, false);
          if (!reqDomain.empty() && ge.early_reason.empty()) {
            ge.req.flags |= KUEUE_TAS_F_DOMAIN;
            R.domain_range(reqDomain, &ge.req.domain_begin, &ge.req.domain_end);
          }
          std::vector<Evaluator::Overlay> base(1);
          for (auto& kv : assumed) base[0].push_back({kv.first.first, kv.first.second, kv.second});
          Evaluator ev{&s};
          std::vector<std::vector<PodSetResult>> res;
          int rc = ev.run(one, false, &res, /*precompiled=*/true, base[0].empty() ? nullptr : &base);
          if (rc) {
            h->err = s.err;
            return rc;
          }
          const PodSetResult& r = res[0][0];
          if (!r.reason.empty()) {
            reason = r.reason;
          } else if (!r.has_assignment || r.domains.empty()) {
            reason = "cannot find replacement assignment for unhealthy node: " + unhealthy;
          } else {
            ExplicitAssignment rep;
            const int L = s.L();
            const size_t levelIdx = s.lowestIsHostname ? size_t(L - 1) : 0;
            rep.levels.assign(s.levelKeys.begin() + int64_t(levelIdx), s.levelKeys.end());
            for (auto& d : r.domains) {
              const auto& lv = s.values[size_t(L - 1)][size_t(d.leaf)];
              std::vector<std::string> vals(lv.begin() + int64_t(levelIdx), lv.end());
              if (s.lowestIsHostname) vals.back() = s.leafId[size_t(d.leaf)];
              rep.domains.emplace_back(std::move(vals), d.count);
            }
            merged = R.merge(rep, existing);
            replacement = rep;
          }
        }
      } catch (const std::runtime_error& e) {
        const std::string w = e.what();
        if (w.rfind("panic: ", 0) != 0) throw;
        reason = w;
      }
      std::string one_out;
      emit_explicit(one_out, m->name, reason.empty() ? merged : std::nullopt, reason);
      results.push_back(one_out);
      if (!reason.empty()) return finish();
      for (auto& d : replacement->domains) {  // addAssumedUsage (:658-666): single x count, no pods
        const int32_t leaf = R.leaf_of(d.first);
        for (auto& kv : m->requestIds) {
          const int32_t c = s.col_of(kv.first);
          int64_t& slot = assumed[{leaf, c}];
          slot = int64_t(uint64_t(slot) + uint64_t(kv.second) * uint64_t(int64_t(d.second)));
        }
      }
    }
  }
  return finish();
}

// FindTopologyAssignmentsForFlavor with ElasticJobsViaWorkloadSlicesWithTAS
// (:563-577, tas_elastic_workloads.go:35-127): groups in order, one device
// evaluation per group with the assumed usage so far as the overlay; a
// workers PodSet with a (non-stale) previous assignment is placed delta-only
// (scale up: the previous pods' usage incl. pods:count assumed, only the new
// pods evaluated, merged with the previous assignment; scale down:
// TruncateAssignment; same count: the previous assignment).
static int find_sequential(kueue_tas_host* h, std::vector<TASPodSetRequests>& podsets, bool sim, std::string* out) {
  FlavorSnapshot& s = *h->snap;
  Replacement R{h, s};
  Workload wl;
  wl.podsets = podsets;
  make_groups(wl);
  s.ensure_columns_for(wl.podsets);  // assumed usage is kept per column
  std::map<std::pair<int32_t, int32_t>, int64_t> assumed;  // (leaf, column) -> usage
  std::vector<std::pair<std::string, std::string>> results;  // (name, JSON) in set order
  auto set_result = [&](const std::string& name, const std::optional<ExplicitAssignment>& a, const std::string& reason) {
    std::string js;
    emit_explicit(js, name, a, reason);
    for (auto& r : results)
      if (r.first == name) {
        r.second = js;
        return;
      }
    results.emplace_back(name, js);
  };
  auto finish = [&]() {
    *out = "{\"results\":[";
    for (size_t i = 0; i < results.size(); i++) *out += (i ? "," : "") + results[i].second;
    *out += "]}";
    return 0;
  };
  auto add_usage = [&](const ExplicitAssignment& a, const TASPodSetRequests& tr, bool pods) {
    for (auto& d : a.domains) {
      const int32_t leaf = R.leaf_of(d.first);  // assumed usage of other domains is never read (:1620)
      if (leaf < 0) continue;
      for (auto& kv : tr.requestIds) {
        int64_t& slot = assumed[{leaf, s.col_of(kv.first)}];
        slot = int64_t(uint64_t(slot) + uint64_t(kv.second) * uint64_t(int64_t(d.second)));
      }
      if (pods) {
        int64_t& slot = assumed[{leaf, s.podsCol}];
        slot = int64_t(uint64_t(slot) + uint64_t(int64_t(d.second)));
      }
    }
  };
  const int L = s.L();
  const size_t levelIdx = s.lowestIsHostname ? size_t(L - 1) : 0;
  auto explicit_of = [&](const PodSetResult& r) {
    ExplicitAssignment a;
    a.levels.assign(s.levelKeys.begin() + int64_t(levelIdx), s.levelKeys.end());
    for (auto& d : r.domains) {
      const auto& lv = s.values[size_t(L - 1)][size_t(d.leaf)];
      std::vector<std::string> vals(lv.begin() + int64_t(levelIdx), lv.end());
      if (s.lowestIsHostname) vals.back() = s.leafId[size_t(d.leaf)];
      a.domains.emplace_back(std::move(vals), d.count);
    }
    return a;
  };
  // findTopologyAssignment(workers, leader, assumedUsage, simulateEmpty, "") on the device
  auto evaluate = [&](const TASPodSetRequests& workers, const TASPodSetRequests* leader,
                      std::vector<PodSetResult>* res) -> int {
    std::vector<Workload> one(1);
    one[0].podsets.push_back(workers);
    if (leader) one[0].podsets.push_back(*leader);
    s.ensure_columns_for(one[0].podsets);
    one[0].groups.resize(1);
    GroupEval& g = one[0].groups[0];
    g.workers = &one[0].podsets[0];
    g.leader = leader ? &one[0].podsets[1] : nullptr;
    g.members = {g.workers};
    if (leader) g.members.push_back(g.leader);
    s.compile_group(g, sim);
    std::vector<Evaluator::Overlay> base(1);
    for (auto& kv : assumed) base[0].push_back({kv.first.first, kv.first.second, kv.second});
    Evaluator ev{&s};
    std::vector<std::vector<PodSetResult>> rs;
    const int rc = ev.run(one, sim, &rs, /*precompiled=*/true, base[0].empty() ? nullptr : &base);
    if (rc) {
      h->err = s.err;
      return rc;
    }
    *res = rs[0];
    return 0;
  };
  auto find_in = [](const std::vector<PodSetResult>& rs, const std::string& name) -> const PodSetResult* {
    for (auto& r : rs)
      if (r.name == name) return &r;
    return nullptr;
  };
  for (auto& g : wl.groups) {
    const TASPodSetRequests& workers = *g.workers;
    const TASPodSetRequests* leader = g.leader;
    if (s.gates.elastic && workers.previousAssignment) {  // handleElasticWorkload (:35-69)
      const ExplicitAssignment& prev = *workers.previousAssignment;
      bool stale = false;
      for (auto& d : prev.domains) stale = stale || !s.has_domain(join_values(d.first));
      if (!stale) {
        int32_t prevCount = 0;
        for (auto& d : prev.domains) prevCount = int32_t(uint32_t(prevCount) + uint32_t(d.second));
        if (workers.count > prevCount) {  // handleScaleUp (:72-112)
          TASPodSetRequests delta = workers;
          delta.count = int32_t(uint32_t(workers.count) - uint32_t(prevCount));
          delta.previousAssignment.reset();
          {  // ComputeUsagePerDomain: per DomainID the last domain's single x count + pods:count
            std::map<std::string, std::pair<const std::vector<std::string>*, int32_t>> per;
            for (auto& d : prev.domains) per[join_values(d.first)] = {&d.first, d.second};
            for (auto& kv : per) {
              ExplicitAssignment one;
              one.domains.emplace_back(*kv.second.first, kv.second.second);
              add_usage(one, workers, true);
            }
          }
          std::vector<PodSetResult> rs;
          if (int rc = evaluate(delta, leader, &rs)) return rc;
          const PodSetResult* wr = find_in(rs, workers.name);
          if (!wr->reason.empty()) {
            set_result(workers.name, std::nullopt, wr->reason);
            return finish();
          }
          try {
            set_result(workers.name, R.merge(explicit_of(*wr), prev), "");
          } catch (const std::runtime_error& e) {
            set_result(workers.name, std::nullopt, e.what());
            return finish();
          }
          if (leader) {
            const ExplicitAssignment la = explicit_of(*find_in(rs, leader->name));
            set_result(leader->name, la, "");
            add_usage(la, *leader, false);
          }
          add_usage(explicit_of(*wr), workers, false);
        } else if (workers.count < prevCount) {  // handleScaleDown: TruncateAssignment
          ExplicitAssignment t;
          t.levels = prev.levels;
          int32_t remaining = workers.count;
          for (auto& d : prev.domains) {
            if (remaining <= 0) break;
            if (d.second <= remaining) {
              t.domains.push_back(d);
              remaining -= d.second;
            } else {
              t.domains.emplace_back(d.first, remaining);
              remaining = 0;
            }
          }
          set_result(workers.name, t, "");
          add_usage(t, workers, false);
        } else {
          set_result(workers.name, prev, "");
          add_usage(prev, workers, false);
        }
        continue;
      }
    }
    std::vector<PodSetResult> rs;
    if (int rc = evaluate(workers, leader, &rs)) return rc;
    const std::string reason = find_in(rs, workers.name)->reason;
    for (const TASPodSetRequests* m : g.members) {
      const PodSetResult* r = find_in(rs, m->name);
      if (r && r->has_assignment) set_result(m->name, explicit_of(*r), reason);
      else set_result(m->name, std::nullopt, reason);
    }
    if (!reason.empty()) return finish();
    for (const TASPodSetRequests* m : g.members) {
      const PodSetResult* r = find_in(rs, m->name);
      if (r && r->has_assignment) add_usage(explicit_of(*r), *m, false);
    }
  }
  return finish();
}

static int run_workloads(kueue_tas_host* h, std::vector<Workload>& wls, bool sim, std::string* out, bool nested) {
  Evaluator ev{h->snap.get()};
  std::vector<std::vector<PodSetResult>> results;
  int rc = ev.run(wls, sim, &results);
  if (rc) {
    h->err = h->snap->err;
    return rc;
  }
  *out = "{\"results\":";
  if (nested) {
    *out += "[";
    for (size_t i = 0; i < results.size(); i++) {
      if (i) *out += ",";
      emit_results(*out, *h->snap, results[i]);
    }
    *out += "]";
  } else {
    emit_results(*out, *h->snap, results[0]);
  }
  *out += "}";
  return 0;
}

int kueue_tas_host_find(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty, char** out_json) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  try {
    std::vector<Workload> wls(1);
    wls[0].podsets = parse_podsets(kjson::parse(podsets_json));
    std::string out;
    int rc = h->snap->gates.elastic ? find_sequential(h, wls[0].podsets, simulate_empty != 0, &out)
                                    : run_workloads(h, wls, simulate_empty != 0, &out, false);
    if (rc) return rc;
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_find_workload(kueue_tas_host* h, const char* workload_json, int32_t simulate_empty, char** out_json) {
  if (!h || !h->snap || !h->err.empty() || !workload_json || !out_json) return KUEUE_TAS_EINVAL;
  try {
    kjson::Node doc = kjson::parse(workload_json);
    std::vector<TASPodSetRequests> podsets = parse_podsets(doc["podSets"]);
    std::vector<std::string> unhealthy;
    for (auto& n : doc["unhealthyNodes"].items) unhealthy.push_back(n.s());
    std::string out;
    if (!unhealthy.empty()) {
      std::map<std::string, ExplicitAssignment> psa;
      for (auto& p : doc["podSetAssignments"].items)
        if (!p["topologyAssignment"].null()) psa[p["name"].s()] = parse_explicit(p["topologyAssignment"]);
      int rc = find_replacement(h, podsets, unhealthy[0], psa, &out);
      if (rc) return rc;
      *out_json = dup(out);
      return 0;
    }
    if (h->snap->gates.elastic) {
      int rc = find_sequential(h, podsets, simulate_empty != 0, &out);
      if (rc) return rc;
      *out_json = dup(out);
      return 0;
    }
    std::vector<Workload> wls(1);
    wls[0].podsets = std::move(podsets);
    int rc = run_workloads(h, wls, simulate_empty != 0, &out, false);
    if (rc) return rc;
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_find_batch(kueue_tas_host* h, const char* workloads_json, char** out_json) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  try {
    kjson::Node doc = kjson::parse(workloads_json);
    std::vector<Workload> wls(doc["workloads"].items.size());
    for (size_t i = 0; i < wls.size(); i++) wls[i].podsets = parse_podsets(doc["workloads"].items[i]);
    std::string out;
    if (h->snap->gates.elastic) {  // delta placement per workload (find_sequential)
      out = "{\"results\":[";
      for (size_t i = 0; i < wls.size(); i++) {
        std::string one;
        if (int rc = find_sequential(h, wls[i].podsets, false, &one)) return rc;
        // {"results":[...]} -> [...]
        out += (i ? "," : "") + one.substr(11, one.size() - 12);
      }
      *out_json = dup(out + "]}");
      return 0;
    }
    int rc = run_workloads(h, wls, false, &out, true);
    if (rc) return rc;
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_v1beta2_from(kueue_tas_host* h, const char* assignments_json, char** out_json) {
  if (!h || !h->snap || !h->err.empty() || !out_json) return KUEUE_TAS_EINVAL;
  try {
    int rc = h->snap->upload();  // the device context
    if (rc) {
      h->err = h->snap->err;
      return rc;
    }
    std::string out;
    rc = v1beta2_from_json(h->snap->ctx, kjson::parse(assignments_json), &out, &h->err);
    if (rc) return rc;
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_internal_from(kueue_tas_host* h, const char* v1beta2_json, char** out_json) {
  if (!h || !out_json) return KUEUE_TAS_EINVAL;
  try {
    std::string out;
    internal_from_json(kjson::parse(v1beta2_json), &out);
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_find_v1beta2(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty, char** out_json) {
  if (!h || !h->snap || !h->err.empty() || !out_json) return KUEUE_TAS_EINVAL;
  try {
    std::vector<Workload> wls(1);
    wls[0].podsets = parse_podsets(kjson::parse(podsets_json));
    Evaluator ev{h->snap.get()};
    std::vector<std::vector<PodSetResult>> results;
    int rc = ev.run(wls, simulate_empty != 0, &results);
    if (rc) {
      h->err = h->snap->err;
      return rc;
    }
    std::vector<const PodSetResult*> rs;
    for (auto& r : results[0]) rs.push_back(&r);
    std::vector<std::string> enc;
    rc = encode_results(*h->snap, rs, &enc);
    if (rc) {
      h->err = h->snap->err;
      return rc;
    }
    std::string out = "{\"results\":[";
    for (size_t i = 0; i < rs.size(); i++) {
      if (i) out += ",";
      out += "{\"name\":";
      kjson::write_string(out, rs[i]->name);
      out += ",\"topologyAssignment\":" + enc[i] + ",\"reason\":";
      kjson::write_string(out, rs[i]->reason);
      out += "}";
    }
    out += "]}";
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_v1beta2_last(kueue_tas_host* h, char** out_json) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  try {
    std::vector<const PodSetResult*> rs;
    std::vector<size_t> per;
    for (auto& w : h->last) {
      per.push_back(w.size());
      for (auto& r : w) rs.push_back(&r);
    }
    std::vector<std::string> enc;
    int rc = encode_results(*h->snap, rs, &enc);
    if (rc) {
      h->err = h->snap->err;
      return rc;
    }
    if (!out_json) return 0;
    std::string out = "[";
    size_t q = 0;
    for (size_t w = 0; w < per.size(); w++) {
      out += w ? ",[" : "[";
      for (size_t i = 0; i < per[w]; i++, q++) out += (i ? "," : "") + enc[q];
      out += "]";
    }
    out += "]";
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_update_usage(kueue_tas_host* h, const char* usage_json, int32_t add) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  try {
    auto us = FlavorSnapshot::parse_usage(kjson::parse(usage_json));
    int rc = h->snap->update_usage(us, add != 0);
    if (rc) h->err = h->snap->err;
    return rc;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

// Rebuild after a structural node event (a node added, removed, NotReady,
// cordoned, moved in the topology, or with a new taint profile / label):
// the reference rebuilds its snapshot every cycle (Cache.Snapshot,
// snapshot.go:186-191); here a new host mirror is assembled from the current
// cache state (nodesCache with the batch's events applied, non-TAS pods, TAS
// usage per domain), the device context is kept, and the compiled
// workloads are recompiled against the new columns.
static int rebuild(kueue_tas_host* h, const kjson::Node& node_events) {
  auto ns = h->snap->fork_state();
  for (auto& n : node_events.items) ns->sync_node(n);
  ns->assemble();
  ns->ctx = h->snap->ctx;  // keep the device context (and its buffers)
  h->snap->ctx = nullptr;
  h->snap = std::move(ns);
  h->ev.reset();
  h->last.clear();
  h->recompile_all();
  return h->snap->upload();
}

int kueue_tas_host_update_nodes(kueue_tas_host* h, const char* nodes_json, int32_t* rebuilt) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  try {
    double* um = h->upd_ms;
    for (double& x : h->upd_ms) x = 0;
    const double t0 = now_ms();
    kjson::Node arr = kjson::parse(nodes_json);
    const double t1 = now_ms();
    // every event's node parsed on the host pool, then applied in order
    const size_t ne = arr.items.size();
    std::vector<NodeInfo> parsed(ne);
    std::vector<char> ready(ne), unsched(ne);
    auto parse_range = [&](size_t b, size_t e) {
      for (size_t q = b; q < e; q++) {
        bool r, u;
        parsed[q] = FlavorSnapshot::parse_node(arr.items[q], &r, &u);
        ready[q] = r;
        unsched[q] = u;
      }
    };
    if (ne >= 16) ktas_pool::HostPool::get().run(ne, 4, parse_range);
    else parse_range(0, ne);
    std::set<int32_t> touched, liveChanged;
    size_t k = 0;
    for (; k < ne; k++)
      if (!h->snap->node_event_in_place(std::move(parsed[k]), ready[k] != 0, unsched[k] != 0, &touched, &liveChanged))
        break;
    const bool structural = k < arr.items.size();
    const double t2 = now_ms();
    if (structural) {  // rebuilt from the cache state, which holds the pending joins
      h->snap->joins.clear();
      h->snap->joinIds.clear();
    } else {
      h->snap->flush_joins(&touched, &liveChanged);
    }
    const double t3 = now_ms();
    int rc0 = 0;
    const bool splice = !structural && h->snap->splicePending;
    if (splice) rc0 = h->snap->upload();  // the pushes below use the new numbering
    if (rc0) {
      h->err = h->snap->err;
      return rc0;
    }
    const double t4 = now_ms();
    um[0] = t1 - t0;
    um[1] = t2 - t1;
    um[2] = t3 - t2;
    if (splice)
      for (int q = 0; q < 3; q++) um[3 + q] = h->snap->splice_ms[q];
    for (int q = 0; q < 4; q++) um[9 + q] = h->snap->flush_ms[q];
    if (rebuilt) *rebuilt = structural ? 1 : 0;
    int rc;
    if (structural) {  // the events applied so far are in the cache state; the rest replay on it
      kjson::Node rest;
      rest.type = kjson::Node::kArray;
      rest.items.assign(arr.items.begin() + int64_t(k), arr.items.end());
      rc = rebuild(h, rest);
    } else {
      if (h->snap->spliced) {  // leaf indices moved: results and the evaluator's caches refer to the old tree
        h->snap->spliced = false;
        h->ev.reset();
        h->last.clear();
      }
      um[6] = now_ms() - t4;
      rc = h->snap->push_liveness(liveChanged);
      if (!rc) rc = h->snap->push_leaves(touched, true);
      if (!rc && h->snap->dirty && h->snap->ctx) rc = h->snap->upload();  // joined leaves: the reload is this event's
    }
    const double t5 = now_ms();
    um[7] = t5 - t4 - um[6];
    um[8] = t5 - t0;
    if (rc) h->err = h->snap->err;
    return rc;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_update_pods(kueue_tas_host* h, const char* pods_json) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  try {
    int rc = h->snap->update_pods(kjson::parse(pods_json));
    if (rc) h->err = h->snap->err;
    return rc;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_fits(kueue_tas_host* h, const char* usage_json, int32_t* fits) {
  if (!h || !h->snap || !h->err.empty() || !fits) return KUEUE_TAS_EINVAL;
  try {
    bool f = false;
    int rc = h->snap->fits(FlavorSnapshot::parse_usage(kjson::parse(usage_json)), &f);
    if (rc) {
      h->err = h->snap->err;
      return rc;
    }
    *fits = f ? 1 : 0;
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

// Batched preemption search: the TAS part of `minimal` (pkg/scheduler/
// preemption/preemption.go:307-341) with workloadFits (:614-625) reduced to
// FindTopologyAssignmentsForWorkload(...).Failure() == nil.  Every candidate
// prefix is one evaluation of the same workload under a removal overlay, so
// the prefix scan is ONE device batch; fillBackWorkloads (:330-345) then runs
// its reverse add-back loop one evaluation per step (each step depends on the
// previous decision), keeping the reference's O(1) swap-delete target order.
static int preemption_search(kueue_tas_host* h, const kjson::Node& podsets, const kjson::Node& cands,
                             std::string* out) {
  FlavorSnapshot& s = *h->snap;
  std::vector<std::vector<FlavorSnapshot::DomainUsage>> cu;
  for (auto& c : cands.items) {
    cu.push_back(FlavorSnapshot::parse_usage(c));
    s.ensure_columns_for_usage(cu.back());  // a re-columned snapshot reloads inside Evaluator::run
  }
  const size_t k = cu.size();
  using Overlay = Evaluator::Overlay;
  auto fits_all = [](const std::vector<PodSetResult>& rs) {
    for (auto& r : rs)
      if (!r.reason.empty()) return false;  // TASAssignmentsResult.Failure() (:384-391)
    return true;
  };
  // settle the column set first (PodSets may add columns): overlays index columns
  {
    std::vector<Workload> probe(1);
    probe[0].podsets = parse_podsets(podsets);
    s.ensure_columns_for(probe[0].podsets);
  }
  std::vector<Overlay> rem(k);
  for (size_t c = 0; c < k; c++) rem[c] = s.removal(cu[c]);
  auto merge = [](const Overlay& x, const Overlay& y) {  // sorted (leaf, col) union, values added
    Overlay r;
    r.reserve(x.size() + y.size());
    size_t i = 0, j = 0;
    while (i < x.size() || j < y.size()) {
      if (j == y.size() || (i < x.size() && (x[i].leaf < y[j].leaf || (x[i].leaf == y[j].leaf && x[i].col < y[j].col)))) {
        r.push_back(x[i++]);
      } else if (i == x.size() || y[j].leaf < x[i].leaf || (y[j].leaf == x[i].leaf && y[j].col < x[i].col)) {
        r.push_back(y[j++]);
      } else {
        r.push_back({x[i].leaf, x[i].col, add64(x[i].value, y[j].value)});
        i++, j++;
      }
    }
    return r;
  };
  double eval_ms[4] = {}, dev_ms[6] = {};
  const double t0 = now_ms();
  // one evaluation per overlay; every Workload parses its own PodSets
  auto eval_overlays = [&](const std::vector<Overlay>& base, std::vector<char>* fit) -> int {
    std::vector<Workload> wls(base.size());
    for (auto& w : wls) w.podsets = parse_podsets(podsets);
    Evaluator ev{&s};
    std::vector<std::vector<PodSetResult>> results;
    int rc = ev.run(wls, false, &results, false, &base);
    if (rc) return rc;
    for (int q = 0; q < 4; q++) eval_ms[q] += ev.host_ms[q];
    for (int q = 0; q < 6; q++) dev_ms[q] += ev.dev_host_ms[q];
    fit->resize(base.size());
    for (size_t i = 0; i < base.size(); i++) (*fit)[i] = fits_all(results[i]) ? 1 : 0;
    return 0;
  };
  std::vector<Overlay> prefixes(k);
  for (size_t i = 0; i < k; i++) prefixes[i] = i ? merge(prefixes[i - 1], rem[i]) : rem[0];
  std::vector<char> pfit;
  int rc = k ? eval_overlays(prefixes, &pfit) : 0;
  if (rc) return rc;
  prefixes.clear();
  long first = -1;
  for (size_t i = 0; i < k; i++)
    if (pfit[i]) {
      first = long(i);
      break;
    }
  std::vector<size_t> targets;
  int64_t fill_evals = 0;
  if (first >= 0) {
    for (size_t c = 0; c <= size_t(first); c++) targets.push_back(c);
    for (long i = long(targets.size()) - 2; i >= 0; i--) {
      // AddWorkload(targets[i]): the removal set is every other target
      Overlay set;
      for (size_t j = 0; j < targets.size(); j++)
        if (long(j) != i) set = merge(set, rem[targets[j]]);
      std::vector<char> f;
      rc = eval_overlays({set}, &f);
      if (rc) return rc;
      fill_evals++;
      if (f[0]) {
        targets[size_t(i)] = targets.back();
        targets.pop_back();
      }
    }
  }
  *out = "{\"prefixFits\":[";
  for (size_t i = 0; i < k; i++) *out += std::string(i ? "," : "") + (pfit[i] ? "true" : "false");
  *out += "],\"firstFit\":" + std::to_string(first) + ",\"targets\":";
  if (first < 0) {
    *out += "null";
  } else {
    *out += "[";
    for (size_t j = 0; j < targets.size(); j++) *out += (j ? "," : "") + std::to_string(targets[j]);
    *out += "]";
  }
  *out += ",\"fillBackEvals\":" + std::to_string(fill_evals);
  // host profile: [prepare, eval calls, decode, total] of the Evaluator runs,
  // the device layer's [compile, classes, enqueue, wait, pack, copy], and the whole search
  *out += ",\"profileMs\":{\"evaluator\":[";
  for (int q = 0; q < 4; q++) *out += (q ? "," : "") + std::to_string(eval_ms[q]);
  *out += "],\"device\":[";
  for (int q = 0; q < 6; q++) *out += (q ? "," : "") + std::to_string(dev_ms[q]);
  *out += "],\"search\":" + std::to_string(now_ms() - t0) + "}}";
  return 0;
}

int kueue_tas_host_preemption_search(kueue_tas_host* h, const char* podsets_json, const char* candidates_json,
                                     char** out_json) {
  if (!h || !h->snap || !h->err.empty() || !out_json) return KUEUE_TAS_EINVAL;
  try {
    std::string out;
    int rc = preemption_search(h, kjson::parse(podsets_json), kjson::parse(candidates_json), &out);
    if (rc) {
      h->err = h->snap->err;
      return rc;
    }
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

// Batched partial-admission search: PodSetReducer.Search
// (pkg/scheduler/flavorassigner/podset_reducer.go:37-86, driven by
// Scheduler.getInitialAssignments, scheduler.go:720-739) with the fits closure
// reduced to its TAS part — Assign(nextCounts) scales each PodSet to its
// count (flavorassigner.go:599-609), a count-0 PodSet sends no TAS request
// (tas_flavorassigner.go:52-55), and the counts fit when
// FindTopologyAssignmentsForWorkload reports no failure (:734-747).
// sort.Search's decision tree is evaluated speculatively: from the current
// interval [i, j) every probe of its next `depth` levels (at most `cap`
// distinct counts vectors, each a workload evaluation against the same
// snapshot) goes into ONE device batch, then the search walks those levels
// on the results — the probes and the answer are exactly sort.Search's, for
// any fits predicate, in ceil(log2(totalDelta + 1) / depth) batches.
static int partial_admission_search(kueue_tas_host* h, const kjson::Node& podsets_doc, bool simulate_empty,
                                    int32_t cap, std::string* out) {
  FlavorSnapshot& s = *h->snap;
  const std::vector<TASPodSetRequests> podsets = parse_podsets(podsets_doc);
  const size_t n = podsets.size();
  std::vector<int32_t> full(n), delta(n);
  std::vector<char> tas(n, 1);
  int32_t total = 0;
  for (size_t i = 0; i < n; i++) {  // NewPodSetReducer (:37-53)
    const kjson::Node& p = podsets_doc.items[i];
    full[i] = podsets[i].count;
    const kjson::Node* m = p.find("minCount");
    delta[i] = full[i] - (m && !m->null() ? int32_t(m->i64()) : full[i]);
    total += delta[i];
    if (const kjson::Node* t = p.find("tas")) tas[i] = t->null() || t->b();
  }
  auto fill = [&](int64_t up) {  // fillPodSetSizesForSearchIndex (:55-62)
    std::vector<int32_t> c(n);
    for (size_t i = 0; i < n; i++) c[i] = full[i] - int32_t(int64_t(delta[i]) * up / int64_t(total));
    return c;
  };
  int depth = 1;
  while (depth < 20 && (int64_t(1) << (depth + 1)) - 1 <= int64_t(std::max(cap, 1))) depth++;
  // index -> (fits, results); a batch's results view the device's entry
  // regions, valid until the next batch: the walk after each batch emits them
  std::unordered_map<int64_t, std::pair<bool, std::vector<PodSetResult>>> probed;
  int64_t evals = 0, batches = 0, probes = 0;
  double eval_ms = 0;
  const double t0 = now_ms();
  int64_t i = 0, j = int64_t(total) + 1, lastGood = 0;
  std::string lastR;  // the last fitting probe's results, emitted
  bool any = total != 0;  // totalDelta == 0: (nil, false) without a probe (:71-73)
  while (any && i < j) {
    // the next `depth` levels of sort.Search's decision tree from [i, j)
    std::vector<int64_t> want;
    std::vector<std::pair<int64_t, int64_t>> lvl{{i, j}};
    for (int d = 0; d < depth && !lvl.empty(); d++) {
      std::vector<std::pair<int64_t, int64_t>> next;
      for (auto [a, b] : lvl) {
        if (a >= b) continue;
        const int64_t hh = int64_t(uint64_t(a + b) >> 1);
        if (!probed.count(hh)) want.push_back(hh);
        next.push_back({hh + 1, b});  // !f(h)
        next.push_back({a, hh});      // f(h)
      }
      lvl = std::move(next);
    }
    std::vector<Workload> wls;
    std::vector<int64_t> of;
    for (int64_t hh : want) {
      const std::vector<int32_t> cur = fill(hh);
      Workload w;
      for (size_t k = 0; k < n; k++)
        if (tas[k] && cur[k] != 0) {
          w.podsets.push_back(podsets[k]);
          w.podsets.back().count = cur[k];
        }
      if (w.podsets.empty()) {  // nothing for TAS to place: the TAS part fits
        probed[hh] = {true, {}};
        continue;
      }
      wls.push_back(std::move(w));
      of.push_back(hh);
    }
    if (!wls.empty()) {
      Evaluator ev{&s};
      std::vector<std::vector<PodSetResult>> results;
      const double te = now_ms();
      int rc = ev.run(wls, simulate_empty, &results);
      if (rc) return rc;
      eval_ms += now_ms() - te;
      batches++;
      evals += int64_t(wls.size());
      for (size_t q = 0; q < wls.size(); q++) {
        bool f = true;
        for (auto& r : results[q]) f = f && r.reason.empty();  // TASAssignmentsResult.Failure() (:384-391)
        probed[of[q]] = {f, std::move(results[q])};
      }
    }
    // sort.Search over the probed levels (:76-84)
    while (i < j) {
      const int64_t hh = int64_t(uint64_t(i + j) >> 1);
      auto it = probed.find(hh);
      if (it == probed.end()) break;  // beyond this batch's levels
      probes++;
      if (it->second.first) {
        lastGood = hh;
        lastR.clear();
        emit_results(lastR, s, it->second.second);
        j = hh;
      } else {
        i = hh + 1;
      }
    }
  }
  const bool found = any && i == lastGood;  // (:85)
  *out = std::string("{\"found\":") + (found ? "true" : "false") + ",\"counts\":";
  if (!found) {
    *out += "null,\"results\":null";
  } else {
    const std::vector<int32_t> c = fill(lastGood);
    *out += "[";
    for (size_t k = 0; k < n; k++) *out += (k ? "," : "") + std::to_string(c[k]);
    *out += "],\"results\":" + lastR;
  }
  *out += ",\"probes\":" + std::to_string(probes) + ",\"evaluations\":" + std::to_string(evals) +
          ",\"batches\":" + std::to_string(batches) + ",\"profileMs\":{\"evaluate\":" + std::to_string(eval_ms) +
          ",\"search\":" + std::to_string(now_ms() - t0) + "}}";
  return 0;
}

int kueue_tas_host_partial_admission_search(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty,
                                            int32_t max_batch, char** out_json) {
  if (!h || !h->snap || !h->err.empty() || !out_json || !podsets_json) return KUEUE_TAS_EINVAL;
  try {
    std::string out;
    int rc = partial_admission_search(h, kjson::parse(podsets_json), simulate_empty != 0,
                                      max_batch > 0 ? max_batch : 1023, &out);
    if (rc) {
      h->err = h->snap->err;
      return rc;
    }
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_compile(kueue_tas_host* h, const char* workloads_json) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  try {
    kjson::Node doc = kjson::parse(workloads_json);
    h->shard_ids.clear();
    h->shard.clear();
    h->compiled.assign(doc["workloads"].items.size(), Workload{});
    h->compiled_gen++;
    for (size_t i = 0; i < h->compiled.size(); i++) {
      h->compiled[i].podsets = parse_podsets(doc["workloads"].items[i]);
      make_groups(h->compiled[i]);
      h->snap->ensure_columns_for(h->compiled[i].podsets);
    }
    for (auto& wl : h->compiled)
      for (auto& g : wl.groups) h->snap->compile_group(g, false);
    h->compiled_cols = h->snap->col_gen;
    return h->snap->upload();
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

// One timed "step": every compiled workload evaluated against the resident
// snapshot, results decoded to (leaf, count) lists; FNV-1a over all results.
// KUEUE_TAS_RUN_COMPILE redoes FindTopologyAssignmentsForFlavor's grouping
// and findTopologyAssignment's prelude (make_groups, compile_group) for every
// workload inside the call, from its TASPodSetRequests; KUEUE_TAS_RUN_VALUES
// builds every result's TopologyAssignment domains (Values, Count).
int kueue_tas_host_run(kueue_tas_host* h, uint32_t flags, uint64_t* result_hash) {
  if (!h || !h->snap || !h->err.empty()) return KUEUE_TAS_EINVAL;
  if (h->compiled_cols != h->snap->col_gen) {  // a pod / usage event re-columned the snapshot since compile
    try {
      h->recompile_all();
    } catch (const std::exception& e) {
      h->err = e.what();
      return KUEUE_TAS_EINVAL;
    }
  }
  if (!h->ev) h->ev = std::make_unique<Evaluator>(Evaluator{h->snap.get()});
  Evaluator& ev = *h->ev;
  std::vector<std::vector<PodSetResult>>& results = h->last;
  const bool compile = (flags & KUEUE_TAS_RUN_COMPILE) != 0;
  int rc = ev.run(h->active(), false, &results, /*precompiled=*/!compile, nullptr, /*regroup=*/compile);
  if (rc) {
    h->err = h->snap->err;
    return rc;
  }
  const FlavorSnapshot& snap = *h->snap;
  const int32_t nlev = snap.lowestIsHostname ? 1 : snap.L();  // Values per domain
  if (flags & KUEUE_TAS_RUN_VALUES) {
    // Values of the domains still viewing the last batch's entries: the tags
    // the device wrote beside them (the leaf's Values address, uploaded per
    // snapshot by FlavorSnapshot::upload); the rest (earlier passes'
    // materialized results, balanced placements) on the host
    const double t0 = now_ms();
    size_t npairs = 0;
    const DomainAssignment* e0 =
        reinterpret_cast<const DomainAssignment*>(kueue_tas_last_entries(snap.ctx, &npairs));
    const uint64_t* tags = kueue_tas_last_entry_tags(snap.ctx);
    std::vector<PodSetResult*>& rest = h->values_rest;
    rest.clear();
    // without device tags: the same per-entry Values pointers built by the
    // host pool in one array laid out like the entry view (no per-result
    // allocation), each domain the leaf's levelValues from the leaf table
    std::vector<PodSetResult*> inview;
    for (auto& rs : results)
      for (auto& r : rs) {
        const size_t nd = r.domains.size();
        if (!nd) continue;
        const bool in = r.domains.p >= e0 && r.domains.p + nd <= e0 + npairs;
        if (tags && in)
          r.values = reinterpret_cast<const std::string* const*>(tags + (r.domains.p - e0));
        else if (in)
          inview.push_back(&r);
        else
          rest.push_back(&r);
      }
    if (!inview.empty()) {
      if (h->values_flat.size() < npairs) h->values_flat.resize(npairs);
      const std::string** vf = h->values_flat.data();
      const int32_t lvl = snap.L() - nlev;
      const std::string* const* lv = snap.leaf_values();
      HostPool::get().run_static(inview.size(), [&](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) {
          PodSetResult& r = *inview[i];
          const size_t o = size_t(r.domains.p - e0), nd = r.domains.size();
          for (size_t k = 0; k < nd; k++) vf[o + k] = lv[r.domains[k].leaf] + lvl;
          r.values = vf + o;
        }
      });
    }
    if (!rest.empty()) {
      const int32_t lvl = snap.L() - nlev;
      const std::string* const* lv = snap.leaf_values();
      HostPool::get().run(rest.size(), 16, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) {
          PodSetResult& r = *rest[i];
          const size_t nd = r.domains.size();
          r.own_values.resize(nd);
          for (size_t k = 0; k < nd; k++) r.own_values[k] = lv[r.domains[k].leaf] + lvl;
          r.values = r.own_values.data();
        }
      });
    }
    ev.host_ms[2] += now_ms() - t0;
    ev.host_ms[3] += now_ms() - t0;
    ev.detail_ms[3] += now_ms() - t0;
  }
  for (int k = 0; k < KUEUE_TAS_NUM_STAGES; k++) h->stage_accum[k] += ev.stage_ms[k];
  h->accum_runs++;
  h->accum_fills += ev.stats[2];
  memcpy(h->ms, ev.ms, sizeof h->ms);
  memcpy(h->counts, ev.counts, sizeof h->counts);
  memcpy(h->stats, ev.stats, sizeof h->stats);
  if (result_hash) {
    uint64_t x = 1469598103934665603ull;
    auto mix = [&](uint64_t v) {  // word-wise FNV-1a variant
      x ^= v;
      x *= 1099511628211ull;
      x ^= x >> 29;
    };
    for (auto& rs : results)
      for (auto& r : rs) {
        mix(r.has_assignment);
        mix(r.domains.size());
        for (auto& d : r.domains) {
          mix(uint64_t(uint32_t(d.leaf)));
          mix(uint64_t(uint32_t(d.count)));
        }
        if (r.values)
          for (size_t d = 0; d < r.domains.size(); d++)
            for (int32_t k = 0; k < nlev; k++) mix(std::hash<std::string>()(r.value(d, nlev).values[k]));
        mix(std::hash<std::string>()(r.reason));
      }
    *result_hash = x;
  }
  return 0;
}

int kueue_tas_host_run_compiled(kueue_tas_host* h, uint64_t* result_hash) { return kueue_tas_host_run(h, 0, result_hash); }

int kueue_tas_host_last_device_host_times(kueue_tas_host* h, double* ms, int n) {
  if (!h || !h->ev || !ms || n < 0) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < 8; k++) ms[k] = h->ev->dev_host_ms[k];
  return 0;
}

int kueue_tas_host_last_stage_times(kueue_tas_host* h, float* ms, int n) {
  if (!h || !h->ev || !ms || n < 0) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < KUEUE_TAS_NUM_STAGES; k++) ms[k] = h->ev->stage_ms[k];
  return 0;
}

int kueue_tas_host_last_eval_ticks(kueue_tas_host* h, int32_t* ticks, size_t n) {
  if (!h || !h->snap) return KUEUE_TAS_EINVAL;
  return kueue_tas_last_eval_ticks(h->snap->ctx, ticks, n);
}

int kueue_tas_host_last_eval_profile(kueue_tas_host* h, int32_t* ticks, size_t n) {
  if (!h || !h->snap) return KUEUE_TAS_EINVAL;
  return kueue_tas_last_eval_profile(h->snap->ctx, ticks, n);
}

int kueue_tas_host_last_profile(kueue_tas_host* h, double* ms4) {
  if (!h || !h->ev) return KUEUE_TAS_EINVAL;
  memcpy(ms4, h->ev->host_ms, sizeof h->ev->host_ms);
  return 0;
}

int kueue_tas_host_set_stage_timing(kueue_tas_host* h, int32_t on) {
  if (!h || !h->snap) return KUEUE_TAS_EINVAL;
  h->snap->stageTiming = on != 0;
  return h->snap->ctx ? kueue_tas_set_stage_timing(h->snap->ctx, on) : 0;
}

int kueue_tas_host_stage_accum(kueue_tas_host* h, float* ms, int n, int64_t* runs, int64_t* fill_launches,
                               int32_t reset) {
  if (!h || n < 0 || (n && !ms)) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < KUEUE_TAS_NUM_STAGES; k++) ms[k] = h->stage_accum[k];
  if (runs) *runs = h->accum_runs;
  if (fill_launches) *fill_launches = h->accum_fills;
  if (reset) {
    for (auto& v : h->stage_accum) v = 0;
    h->accum_runs = h->accum_fills = 0;
  }
  return 0;
}

int kueue_tas_host_last_update_detail(kueue_tas_host* h, double* ms, int n) {
  if (!h || !ms) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < 13; k++) ms[k] = h->upd_ms[k];
  return KUEUE_TAS_OK;
}

int kueue_tas_host_last_host_detail(kueue_tas_host* h, double* ms, int n) {
  if (!h || !h->ev || !ms || n < 0) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < 4; k++) ms[k] = h->ev->detail_ms[k];
  return 0;
}

int kueue_tas_host_last_timings(kueue_tas_host* h, float* ms4, int64_t* counts3) {
  if (!h) return KUEUE_TAS_EINVAL;
  if (ms4) memcpy(ms4, h->ms, sizeof h->ms);
  if (counts3) memcpy(counts3, h->counts, sizeof h->counts);
  return 0;
}

int kueue_tas_host_last_stats(kueue_tas_host* h, int64_t* stats8) {
  if (!h || !stats8) return KUEUE_TAS_EINVAL;
  stats8[0] = h->counts[0];
  stats8[1] = h->counts[1];
  stats8[2] = h->counts[2];
  for (int k = 0; k < 5; k++) stats8[3 + k] = h->stats[k];
  return 0;
}

int kueue_tas_host_last_stats_ext(kueue_tas_host* h, int64_t* out, int32_t n) {
  if (!h || !out || n < 0) return KUEUE_TAS_EINVAL;
  int64_t all[9];
  kueue_tas_host_last_stats(h, all);
  all[8] = h->stats[5];
  for (int k = 0; k < n && k < 9; k++) out[k] = all[k];
  return 0;
}

int kueue_tas_host_set_shard(kueue_tas_host* h, const int32_t* ids, size_t n) {
  if (!h || !h->snap || !h->err.empty() || (n && !ids)) return KUEUE_TAS_EINVAL;
  try {
    h->shard_ids.assign(ids, ids + n);
    h->shard.assign(n, Workload{});
    for (size_t k = 0; k < n; k++) {
      if (ids[k] < 0 || size_t(ids[k]) >= h->compiled.size()) throw std::runtime_error("shard index out of range");
      h->shard[k].podsets = h->compiled[size_t(ids[k])].podsets;
      make_groups(h->shard[k]);
      for (auto& g : h->shard[k].groups) h->snap->compile_group(g, false);
    }
    h->ev.reset();
    h->last.clear();
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_last_assignments(kueue_tas_host* h, int32_t* buf, size_t cap, size_t* len) {
  if (!h || !h->snap || !len) return KUEUE_TAS_EINVAL;
  std::vector<Workload>& wls = h->active();
  size_t need = 0;
  for (size_t i = 0; i < h->last.size(); i++) {
    need += 4;
    for (auto& r : h->last[i]) need += 4 * r.domains.size();
  }
  *len = need;
  if (need > cap || (need && !buf)) return KUEUE_TAS_EOVERFLOW;
  size_t o = 0;
  for (size_t i = 0; i < h->last.size() && i < wls.size(); i++) {
    const int32_t g = h->shard_ids.empty() ? int32_t(i) : h->shard_ids[i];
    bool fail = false;
    int32_t nd = 0;
    for (auto& r : h->last[i]) {
      fail |= !r.reason.empty();
      nd += int32_t(r.domains.size());
    }
    int32_t* hd = buf + o;
    hd[0] = g;
    hd[1] = -1;
    hd[2] = fail ? 1 : 0;
    hd[3] = nd;
    o += 4;
    for (auto& r : h->last[i]) {
      int32_t p = 0;
      while (size_t(p) < wls[i].podsets.size() && wls[i].podsets[size_t(p)].name != r.name) p++;
      for (auto& d : r.domains) {
        buf[o] = g;
        buf[o + 1] = p;
        buf[o + 2] = d.leaf;
        buf[o + 3] = d.count;
        o += 4;
      }
    }
  }
  return 0;
}

// Admission over the gathered records of a nominate batch: workloads in
// ascending id order (the iteration order of processEntry,
// pkg/scheduler/scheduler.go:337-339), each admitted when its assignments
// all exist and Fits, then AddUsage -> updateTASUsage (usage records as
// ComputeTASNetUsage builds them, flavorassigner.go:94-130: per assigned
// domain, the PodSet's single-pod requests and the domain's count).  The
// device applies the usage (kueue_tas_admit); the host mirror follows.
int kueue_tas_host_admit(kueue_tas_host* h, const int32_t* recs, size_t len, int32_t* admitted, size_t admitted_cap,
                         size_t* n_workloads, size_t* n_deltas) {
  if (!h || !h->snap || !h->err.empty() || (len && !recs) || len % 4 || !n_workloads) return KUEUE_TAS_EINVAL;
  try {
    // workloads in ascending id (the gathered quads of every rank; a
    // workload's quads are contiguous per rank), capacity checked first:
    // nothing is admitted when the caller's buffer is short
    const size_t W = h->compiled.size();
    std::vector<int32_t>& seen = h->admit_seen;  // per id: 0 absent, 1 present, 2 failed evaluation
    // the records in the host pool's static parts: per part and workload, the
    // presence mark and the record count (pass 1), then each part scatters its
    // records behind the earlier parts' (pass 2) — the order of one serial pass
    const size_t R = len / 4;
    auto& pool = ktas_pool::HostPool::get();
    const size_t T = pool.parts();
    auto part_of = [&](size_t b) {
      size_t t = 0;
      while (t + 1 < T && ktas_pool::HostPool::part_begin(R, t + 1, T) <= b) t++;
      return t;
    };
    const int64_t Nleaf = h->snap->N();
    std::vector<int32_t>& pseen = h->admit_pseen;
    std::vector<int64_t>& pcnt = h->admit_pcnt;
    pseen.assign(T * W, 0);
    pcnt.assign(T * W, 0);
    std::atomic<bool> bad_g{false}, bad_r{false};
    pool.run_static(R, [&](size_t b, size_t e) {
      if (b >= e) return;
      const size_t t = part_of(b);
      int32_t* sn = pseen.data() + t * W;
      int64_t* cnt = pcnt.data() + t * W;
      for (size_t q = b; q < e; q++) {
        const int32_t* r = recs + 4 * q;
        const int32_t g = r[0];
        if (g < 0 || size_t(g) >= W) {
          bad_g = true;
          return;
        }
        if (r[1] < 0) {
          sn[g] = r[2] != 0 ? 2 : std::max(sn[g], 1);
        } else {
          sn[g] = std::max(sn[g], 1);
          if (size_t(r[1]) >= h->compiled[size_t(g)].podsets.size() || r[2] < 0 || r[2] >= Nleaf) bad_r = true;
          else cnt[g]++;
        }
      }
    });
    if (bad_g) throw std::runtime_error("admit: workload id out of range");
    seen.assign(W, 0);
    size_t nwl = 0;
    for (size_t t = 0; t < T; t++)
      for (size_t g = 0; g < W; g++) seen[g] = std::max(seen[g], pseen[t * W + g]);
    for (size_t g = 0; g < W; g++) nwl += seen[g] != 0;
    *n_workloads = nwl;
    if (!admitted || admitted_cap < 2 * nwl) return KUEUE_TAS_EOVERFLOW;
    h->last_deltas.clear();
    const double t0 = now_ms();
    FlavorSnapshot& s = *h->snap;
    int rc = s.upload();
    if (rc) {
      h->err = s.err;
      return rc;
    }
    if (bad_r) throw std::runtime_error("admit: record out of range");
    // records of each workload, grouped by id (a counting sort over the parts)
    std::vector<int64_t>& start = h->admit_start;
    start.assign(W + 1, 0);
    for (size_t g = 0; g < W; g++) {
      int64_t c = start[g];
      for (size_t t = 0; t < T; t++) {  // part t's first slot for workload g
        const int64_t k = pcnt[t * W + g];
        pcnt[t * W + g] = c;
        c += k;
      }
      start[g + 1] = c;
    }
    std::vector<std::array<int32_t, 3>>& doms = h->admit_doms;  // podset, leaf, count
    doms.resize(size_t(start[W]));
    pool.run_static(R, [&](size_t b, size_t e) {
      if (b >= e) return;
      int64_t* pos = pcnt.data() + part_of(b) * W;
      for (size_t q = b; q < e; q++) {
        const int32_t* r = recs + 4 * q;
        if (r[1] >= 0) doms[size_t(pos[size_t(r[0])]++)] = {r[1], r[2], r[3]};
      }
    });
    std::vector<kueue_tas_fits_req>& fr = h->admit_fr;
    std::vector<kueue_tas_fits_term>& terms = h->admit_terms;
    std::vector<int64_t>& off = h->admit_off;
    std::vector<int32_t>& ids = h->admit_ids;
    ids.clear();
    for (size_t g = 0; g < W; g++)
      if (seen[g]) ids.push_back(int32_t(g));
    // per workload in id order: its records (one per domain; a failed
    // evaluation one record that cannot fit) and its PodSets' single-pod
    // request terms (once per PodSet, shared by the PodSet's domains):
    // counted, offset, then written in place — both passes on the host pool
    const size_t nw = ids.size();
    std::vector<int64_t>& toff = h->admit_toff;
    off.assign(nw + 1, 0);
    toff.assign(nw + 1, 0);
    std::atomic<bool> bad_col{false};
    pool.run(nw, 64, [&](size_t k0, size_t k1) {
      std::vector<uint8_t> used;
      for (size_t k = k0; k < k1; k++) {
        const size_t g = size_t(ids[k]);
        if (seen[g] != 1) {
          off[k + 1] = 1;
          continue;
        }
        const Workload& wl = h->compiled[g];
        used.assign(wl.podsets.size(), 0);
        int64_t nt = 0;
        for (int64_t i = start[g]; i < start[g + 1]; i++) {
          const size_t ps = size_t(doms[size_t(i)][0]);
          if (!used[ps]) {
            used[ps] = 1;
            nt += int64_t(wl.podsets[ps].requestIds.size());
          }
        }
        off[k + 1] = start[g + 1] - start[g];
        toff[k + 1] = nt;
      }
    });
    for (size_t k = 0; k < nw; k++) {
      off[k + 1] += off[k];
      toff[k + 1] += toff[k];
    }
    fr.resize(size_t(off[nw]));
    terms.resize(size_t(toff[nw]));
    pool.run(nw, 64, [&](size_t k0, size_t k1) {
      std::vector<std::pair<int32_t, int32_t>> psTerms;
      for (size_t k = k0; k < k1; k++) {
        const size_t g = size_t(ids[k]);
        int64_t r = off[k], t = toff[k];
        if (seen[g] != 1) {  // a failed evaluation is never admitted: one record that cannot fit
          fr[size_t(r)] = {-1, 0, int32_t(t), 0};
          continue;
        }
        const Workload& wl = h->compiled[g];
        psTerms.assign(wl.podsets.size(), {-1, 0});
        for (int64_t i = start[g]; i < start[g + 1]; i++) {
          const auto& d = doms[size_t(i)];
          auto& pt = psTerms[size_t(d[0])];
          if (pt.first < 0) {
            pt.first = int32_t(t);
            for (auto& rq : wl.podsets[size_t(d[0])].requestIds) {
              const int32_t c = s.col_of(rq.first);
              if (c < 0) bad_col = true;
              terms[size_t(t++)] = {rq.second, c, 0};
              pt.second++;
            }
          }
          fr[size_t(r++)] = {d[1], d[2], pt.first, pt.second};
        }
      }
    });
    if (bad_col) throw std::runtime_error("admit: request resource without a column");
    std::vector<int32_t> adm(ids.size(), 0);
    const auto pods = s.colByName.find("pods");
    const int32_t pods_col = pods == s.colByName.end() ? -1 : pods->second;
    const double t1 = now_ms();
    rc = kueue_tas_admit(s.ctx, fr.data(), fr.size(), terms.data(), terms.size(), off.data(), ids.size(), pods_col,
                         adm.data());
    if (rc) {
      h->err = std::string("admit: ") + kueue_tas_last_error(s.ctx);
      return rc;
    }
    // the delta list the replicas apply (updateTASUsage per record); the
    // host mirror takes it deferred (already applied on the device)
    const double t2 = now_ms();
    std::vector<kueue_tas_delta>& deltas = h->last_deltas;
    for (size_t k = 0; k < ids.size(); k++) {
      admitted[2 * k] = ids[k];
      admitted[2 * k + 1] = adm[k];
      if (!adm[k]) continue;
      for (int64_t i = off[k]; i < off[k + 1]; i++) {
        const kueue_tas_fits_req& r = fr[size_t(i)];
        for (int q = 0; q < r.num_terms; q++) {
          const kueue_tas_fits_term& t = terms[size_t(r.term_begin + q)];
          deltas.push_back({r.leaf, t.col, mul64(t.value, r.count)});
        }
        if (pods_col >= 0) deltas.push_back({r.leaf, pods_col, int64_t(r.count)});
      }
    }
    if (n_deltas) *n_deltas = deltas.size();
    s.device_applied();
    h->admit_ms[0] = t1 - t0;
    h->admit_ms[1] = t2 - t1;
    h->admit_ms[2] = now_ms() - t2;
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_admit_block(kueue_tas_host* h, const int32_t* block, size_t row_words, const int64_t* lens,
                               int32_t world, int32_t* admitted, size_t admitted_cap, size_t* n_workloads,
                               size_t* n_deltas) {
  if (!h || !h->snap || !h->err.empty() || !block || !lens || world < 1 || !n_workloads) return KUEUE_TAS_EINVAL;
  try {
    FlavorSnapshot& s = *h->snap;
    const double t0 = now_ms();
    int rc = s.upload();
    if (rc) {
      h->err = s.err;
      return rc;
    }
    const size_t W = h->compiled.size();
    // the compiled workloads' per-PodSet request terms on the device, rebuilt
    // when the compiled set or the columns change
    const std::array<uint64_t, 3> key{h->compiled_gen, s.compile_gen, s.col_gen};
    if (h->admit_table_key != key) {
      std::vector<int32_t> base(W + 1, 0), pst;
      std::vector<kueue_tas_fits_term> terms;
      for (size_t g = 0; g < W; g++) {
        for (auto& ps : h->compiled[g].podsets) {
          pst.push_back(int32_t(terms.size()));
          pst.push_back(int32_t(ps.requestIds.size()));
          for (auto& rq : ps.requestIds) terms.push_back({rq.second, s.col_of(rq.first), 0});
        }
        base[g + 1] = int32_t(pst.size() / 2);
      }
      rc = kueue_tas_admit_table(s.ctx, base.data(), int32_t(W), pst.data(), terms.data(), terms.size());
      if (rc) {
        h->err = std::string("admit: ") + kueue_tas_last_error(s.ctx);
        return rc;
      }
      h->admit_table_key = key;
    }
    const auto pods = s.colByName.find("pods");
    const int32_t pods_col = pods == s.colByName.end() ? -1 : pods->second;
    std::vector<int32_t>& ids = h->admit_ids;
    std::vector<int32_t>& adm = h->admit_adm;
    ids.resize(std::max<size_t>(W, 1));
    adm.resize(std::max<size_t>(W, 1));
    const kueue_tas_delta* dl = nullptr;
    size_t nw = 0, nd = 0;
    const double t1 = now_ms();
    rc = kueue_tas_admit_block(s.ctx, block, row_words, lens, world, pods_col, ids.data(), adm.data(), W, &nw, &dl, &nd);
    if (rc == KUEUE_TAS_ELAYOUT || rc == KUEUE_TAS_EHOSTMEM) {  // the quads through the host path
      std::vector<int32_t> quads;
      for (int32_t r = 0; r < world; r++) {
        const size_t at = quads.size();
        quads.resize(at + size_t(lens[r]));
        const int32_t* row = block + size_t(r) * row_words + 1;
        if (rc == KUEUE_TAS_EHOSTMEM) {
          if (lens[r]) memcpy(quads.data() + at, row, size_t(lens[r]) * 4);
        } else if (lens[r] && kueue_tas_copy_to_host(s.ctx, quads.data() + at, row, size_t(lens[r]) * 4)) {
          throw std::runtime_error("admit: block copy");
        }
      }
      return kueue_tas_host_admit(h, quads.data(), quads.size(), admitted, admitted_cap, n_workloads, n_deltas);
    }
    if (rc && rc != KUEUE_TAS_EOVERFLOW) {
      h->err = std::string("admit: ") + kueue_tas_last_error(s.ctx);
      return rc;
    }
    *n_workloads = nw;
    if (rc == KUEUE_TAS_EOVERFLOW || !admitted || admitted_cap < 2 * nw) return KUEUE_TAS_EOVERFLOW;
    const double t2 = now_ms();
    for (size_t k = 0; k < nw; k++) {
      admitted[2 * k] = ids[k];
      admitted[2 * k + 1] = adm[k];
    }
    h->last_deltas.assign(dl, dl + nd);
    if (n_deltas) *n_deltas = nd;
    s.device_applied();
    h->admit_ms[0] = t1 - t0;
    h->admit_ms[1] = t2 - t1;
    h->admit_ms[2] = now_ms() - t2;
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_last_admit_stats(kueue_tas_host* h, int64_t* out3) {
  if (!h || !h->snap || !h->snap->ctx || !out3) return KUEUE_TAS_EINVAL;
  return kueue_tas_last_admit_stats(h->snap->ctx, out3);
}

int kueue_tas_host_last_admit_times(kueue_tas_host* h, double* ms3) {
  if (!h || !ms3) return KUEUE_TAS_EINVAL;
  memcpy(ms3, h->admit_ms, sizeof h->admit_ms);
  return 0;
}

int kueue_tas_host_last_deltas(kueue_tas_host* h, kueue_tas_delta* buf, size_t cap) {
  if (!h || (cap && !buf)) return KUEUE_TAS_EINVAL;
  if (cap < h->last_deltas.size()) return KUEUE_TAS_EOVERFLOW;
  std::copy(h->last_deltas.begin(), h->last_deltas.end(), buf);
  return 0;
}

// A replica applies the delta list another rank's admission produced
// (updateTASUsage on its own copy of the snapshot).
int kueue_tas_host_apply_deltas(kueue_tas_host* h, const kueue_tas_delta* d, size_t n) {
  if (!h || !h->snap || !h->err.empty() || (n && !d)) return KUEUE_TAS_EINVAL;
  try {
    FlavorSnapshot& s = *h->snap;
    if (s.dirty || !s.ctx) {  // no device copy to follow: the mirror takes the deltas, the upload the mirror
      for (size_t i = 0; i < n; i++)
        if (d[i].leaf < 0 || d[i].leaf >= s.N() || d[i].col < 0 || size_t(d[i].col) >= s.cols.size())
          throw std::runtime_error("delta out of range");
      s.apply_to_mirror(d, n);
      const int rc = s.upload();
      if (rc) h->err = s.err;  // sticky, as on the admit path
      return rc;
    }
    // (the device layer checks every record against the resident snapshot,
    // whose leaves and columns are the mirror's when it is not dirty)
    int rc = n ? kueue_tas_snapshot_apply_deltas(s.ctx, d, n, nullptr) : 0;
    if (rc == KUEUE_TAS_EINVAL) {
      h->err = "delta out of range";
      return KUEUE_TAS_EINVAL;
    }
    if (rc) h->err = std::string("apply deltas: ") + kueue_tas_last_error(s.ctx);
    else if (n) s.device_applied();  // the host mirror follows at its next read
    return rc;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_last_results(kueue_tas_host* h, char** out_json) {
  if (!h || !h->snap || !out_json) return KUEUE_TAS_EINVAL;
  try {
    std::string out = "{\"results\":[";
    for (size_t i = 0; i < h->last.size(); i++) {
      if (i) out += ",";
      emit_results(out, *h->snap, h->last[i]);
    }
    out += "]}";
    *out_json = dup(out);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

#ifndef KTAS_SOURCE_HASH
#define KTAS_SOURCE_HASH "unversioned"
#endif
int kueue_tas_resource_quantity_string(const char* name, int64_t value, char* buf, size_t cap, size_t* len) {
  if (!name || !len || (cap && !buf)) return KUEUE_TAS_EINVAL;
  const std::string q = resource_quantity_string(name, value);
  *len = q.size();
  if (cap < q.size() + 1) return KUEUE_TAS_EOVERFLOW;
  memcpy(buf, q.c_str(), q.size() + 1);
  return 0;
}

int kueue_tas_host_has_level(kueue_tas_host* h, const char* topology_request_json, int32_t* out) {
  if (!h || !h->snap || !topology_request_json || !out) return KUEUE_TAS_EINVAL;
  try {
    *out = h->snap->has_level(parse_topology_request(kjson::parse(topology_request_json))) ? 1 : 0;
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_assignment_stale(kueue_tas_host* h, const char* assignment_json, int32_t* stale, char** domain) {
  if (!h || !h->snap || !assignment_json || !stale) return KUEUE_TAS_EINVAL;
  try {
    std::string d;
    *stale = h->snap->assignment_stale(kjson::parse(assignment_json), &d) ? 1 : 0;
    if (domain) *domain = dup(d);
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

int kueue_tas_host_free_capacity_json(kueue_tas_host* h, char** out_json) {
  if (!h || !h->snap || !out_json) return KUEUE_TAS_EINVAL;
  try {
    *out_json = dup(h->snap->free_capacity_json());
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

kueue_tas_ctx* kueue_tas_host_ctx(kueue_tas_host* h) {
  if (!h || !h->snap || !h->err.empty()) return nullptr;
  return h->snap->upload() ? nullptr : h->snap->ctx;
}

int kueue_tas_host_leaf_ids(kueue_tas_host* h, char** out_json) {
  if (!h || !h->snap || !out_json) return KUEUE_TAS_EINVAL;
  std::string o = "[";
  for (size_t i = 0; i < h->snap->leafId.size(); i++) {
    if (i) o += ",";
    kjson::write_string(o, h->snap->leafId[i]);
  }
  *out_json = dup(o + "]");
  return 0;
}

int kueue_tas_host_compile_workload(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty,
                                    kueue_tas_eval_req* reqs, size_t reqs_cap, size_t* n_groups, int32_t* taint_table,
                                    size_t taint_cap, size_t* taint_len, int32_t* num_taints,
                                    kueue_tas_affinity_req* affinity, size_t affinity_cap, size_t* n_affinity,
                                    int32_t* affinity_values, size_t values_cap, size_t* n_values,
                                    char** early_reasons_json) {
  if (!h || !h->snap || !h->err.empty() || !podsets_json || !n_groups || !taint_len || !n_affinity || !n_values)
    return KUEUE_TAS_EINVAL;
  try {
    FlavorSnapshot& s = *h->snap;
    Workload wl;
    wl.podsets = parse_podsets(kjson::parse(podsets_json));
    make_groups(wl);
    s.ensure_columns_for(wl.podsets);
    for (auto& g : wl.groups) s.compile_group(g, simulate_empty != 0);
    int rc = s.upload();  // a new request resource re-columns the device snapshot
    if (rc) {
      h->err = s.err;
      return rc;
    }
    size_t na = 0, nv = 0;
    for (auto& g : wl.groups) {
      na += g.aff.size() + g.sel_ext.size();
      nv += g.aff_vals.size() + g.sel_vals.size();
    }
    const size_t P = s.profiles.size();
    *n_groups = wl.groups.size();
    *taint_len = P * wl.groups.size();
    *n_affinity = na;
    *n_values = nv;
    if (num_taints) *num_taints = int32_t(s.taintStrings.size());
    if (reqs_cap < wl.groups.size() || taint_cap < *taint_len || affinity_cap < na || values_cap < nv ||
        (wl.groups.size() && (!reqs || (P && !taint_table))) || (na && !affinity) || (nv && !affinity_values))
      return KUEUE_TAS_EOVERFLOW;
    std::string reasons = "[";
    size_t ka = 0, kv = 0;
    for (size_t i = 0; i < wl.groups.size(); i++) {
      const GroupEval& g = wl.groups[i];
      kueue_tas_eval_req q = g.req;
      q.taint_table = int32_t(i * P);
      std::copy(g.taint_row.begin(), g.taint_row.end(), taint_table + i * P);
      q.assumed_begin = q.assumed_end = 0;
      q.affinity_begin = int32_t(ka);
      for (auto r : g.aff) {
        r.begin += int32_t(kv);
        affinity[ka++] = r;
      }
      q.affinity_end = int32_t(ka);
      std::copy(g.aff_vals.begin(), g.aff_vals.end(), affinity_values + kv);
      kv += g.aff_vals.size();
      q.selector_begin = int32_t(ka);
      for (auto r : g.sel_ext) {
        r.begin += int32_t(kv);
        affinity[ka++] = r;
      }
      q.selector_end = int32_t(ka);
      std::copy(g.sel_vals.begin(), g.sel_vals.end(), affinity_values + kv);
      kv += g.sel_vals.size();
      reqs[i] = q;
      if (i) reasons += ",";
      kjson::write_string(reasons, g.early_reason);
    }
    if (early_reasons_json) *early_reasons_json = dup(reasons + "]");
    return 0;
  } catch (const std::exception& e) {
    h->err = e.what();
    return KUEUE_TAS_EINVAL;
  }
}

const char* kueue_tas_build_id(void) { return KTAS_SOURCE_HASH; }

void kueue_tas_free(char* p) { free(p); }

}  // extern "C"
