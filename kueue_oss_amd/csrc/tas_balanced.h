// tas_balanced.h — TASBalancedPlacement (Alpha, tas_flavor_snapshot.go:906-917,
// pkg/cache/scheduler/tas_balanced_placement.go) as a host path of the host
// layer over one evaluation's phase-1 counters, which the device computed
// (fill + roll-up; kueue_tas_last_counters).
//
// The reference runs it on clones of the requested level's sibling subtrees
// (cloneDomains :343-359), prunes the clones below a balance threshold and
// recomputes their counters (pruneDomainsBelowThreshold :361-382 ->
// fillInCountsHelper), picks a domain set with a small dynamic program
// (selectOptimalDomainSetToFit :81-147), spreads the slices evenly
// (placeSlicesOnDomainsBalanced :149-184) and then descends the clones the
// way findTopologyAssignment does (:928-996).  Here the clones are an arena
// of nodes cloned breadth-first from the CSR tree, so a node's children are
// a contiguous range in domain-index (= lexicographic levelValues) order.
//
// Tie rule where Go iterates a map (domainsPerLevel :243-246; the children
// slices, filled in s.leaves map order by initialize :210-241):
// lexicographic levelValues order; sortDomainsByCapacityAndEntropy (:211-231,
// pdqsort, comparator 0 on equal entropy) is a stable insertion sort.  The
// oracle (oracle/tas_oracle.cpp) restates the same rules.
// Parity unpinned: Go's slices.SortFunc is an insertion sort
// only up to 12 elements (pdqsort, not stable, above), so more than 12
// siblings whose keys tie may order differently; go_log restates Go's pure-Go
// math.Log, while Go on amd64 calls its assembly archLog.  No reference
// golden reaches either case.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <limits>
#include <map>
#include <optional>
#include <string>
#include <vector>

namespace ktas_balanced {

inline int32_t w_add(int32_t a, int32_t b) { return int32_t(uint32_t(a) + uint32_t(b)); }
inline int32_t w_sub(int32_t a, int32_t b) { return int32_t(uint32_t(a) - uint32_t(b)); }
inline int32_t w_mul(int32_t a, int32_t b) { return int32_t(uint32_t(a) * uint32_t(b)); }
inline int32_t go_div32(int32_t a, int32_t b) {  // b != 0 (checked by the callers' preludes)
  if (b == -1) return int32_t(0u - uint32_t(a));
  return a / b;
}

// One domain's counters (tas_flavor_snapshot.go:71-84).
struct Ctr {
  int32_t st = 0, ss = 0, swl = 0, sswl = 0, ls = 0;
};

// The snapshot's domain tree with one evaluation's phase-1 counters.
struct Tree {
  int L = 0;
  std::vector<int32_t> size;                   // D_l
  std::vector<const std::vector<int32_t>*> co; // l < L-1: [D_l + 1] child offsets into level l+1
  std::vector<std::vector<Ctr>> ctr;           // [l][i]
};

// The request's parameters (topologyAssignmentParameters, :447-464).
struct Params {
  int32_t count = 0, sliceSize = 1, leaderCount = 0;
  int requestedLevelIdx = 0, sliceLevelIdx = 0;
  const int32_t* sliceSizeAtLevel = nullptr;  // [L]: 0 = absent (buildSliceSizeAtLevel :1018-1063)
};

struct Result {
  bool used = false;           // useBalancedPlacement (:910): otherwise findLevelWithFitDomains decides
  std::string reason;          // failure text ("TAS Balanced Placement: ..." or a Go panic)
  std::vector<std::pair<int32_t, int32_t>> workers, leaders;  // (leaf, count) in leaf order (buildAssignment)
};

class Placement {
 public:
  Placement(const Tree& t, const Params& p) : t_(t), p_(p) {}

  Result run() {
    Result r;
    std::vector<int32_t> best;
    bool panic = false;
    const int32_t thr = find_best_domains(&best, &panic);
    if (panic) {  // balanceThresholdValue :67 divides by a zero domain count
      r.used = true;
      r.reason = "panic: runtime error: integer divide by zero";
      return r;
    }
    if (thr <= 0) return r;
    r.used = true;
    std::vector<int32_t> cur;
    int fitLevel = 0;
    r.reason = apply(thr, best, &cur, &fitLevel);
    if (!r.reason.empty()) return r;
    descend(cur, fitLevel, &r);
    return r;
  }

 private:
  struct Node {
    Ctr c;
    int32_t level, idx;          // original domain (idx: index in its level = lexicographic rank)
    int32_t kid_begin, kid_end;  // arena range of the children
  };
  const Tree& t_;
  const Params& p_;
  std::vector<Node> a_;  // clones (cloneDomain)

  bool lex_less(int32_t x, int32_t y) const { return a_[x].idx < a_[y].idx; }  // same level: slices.Compare

  // cloneDomains (:343-359) of domains `doms` of `level`: breadth first, so
  // every node's children are contiguous and in index order
  std::vector<int32_t> clone(int level, const std::vector<int32_t>& doms) {
    std::vector<int32_t> roots;
    size_t lo = a_.size();
    for (int32_t i : doms) {
      roots.push_back(int32_t(a_.size()));
      a_.push_back(Node{t_.ctr[size_t(level)][size_t(i)], level, i, 0, 0});
    }
    size_t hi = a_.size();
    for (int l = level; l + 1 < t_.L; l++) {
      const std::vector<int32_t>& co = *t_.co[size_t(l)];
      for (size_t n = lo; n < hi; n++) {
        const int32_t b = co[size_t(a_[n].idx)], e = co[size_t(a_[n].idx) + 1];
        a_[n].kid_begin = int32_t(a_.size());
        for (int32_t j = b; j < e; j++) a_.push_back(Node{t_.ctr[size_t(l + 1)][size_t(j)], l + 1, j, 0, 0});
        a_[n].kid_end = int32_t(a_.size());
      }
      lo = hi;
      hi = a_.size();
    }
    for (size_t n = lo; n < hi; n++) a_[n].kid_begin = a_[n].kid_end = int32_t(n);  // leaves of the clone
    return roots;
  }
  std::vector<int32_t> lower(const std::vector<int32_t>& ds) const {  // lowerLevelDomains (:1503-1509)
    std::vector<int32_t> out;
    for (int32_t d : ds)
      for (int32_t k = a_[d].kid_begin; k < a_[d].kid_end; k++) out.push_back(k);
    return out;
  }
  bool has_kids(int32_t d) const { return a_[d].kid_end > a_[d].kid_begin; }

  // sortedDomainsWithLeader / sortedDomains (:1511-1564), BestFit order
  // (balanced placement only runs for requests that are not unconstrained)
  std::vector<int32_t> sorted_wl(std::vector<int32_t> v) const {
    std::sort(v.begin(), v.end(), [&](int32_t x, int32_t y) {
      const Ctr &a = a_[x].c, &b = a_[y].c;
      if (a.ls != b.ls) return a.ls > b.ls;
      if (a.sswl != b.sswl) return a.sswl > b.sswl;
      if (a.swl != b.swl) return a.swl < b.swl;
      return lex_less(x, y);
    });
    return v;
  }
  std::vector<int32_t> sorted(std::vector<int32_t> v) const {
    std::sort(v.begin(), v.end(), [&](int32_t x, int32_t y) {
      const Ctr &a = a_[x].c, &b = a_[y].c;
      if (a.ss != b.ss) return a.ss > b.ss;
      if (a.st != b.st) return a.st < b.st;
      return lex_less(x, y);
    });
    return v;
  }

  struct Greedy {
    bool fit = false;
    int32_t count = 0;
    int32_t lastWL = -1, last = -1;
  };
  Greedy greedy(const std::vector<int32_t>& ds, int32_t sliceCount, int32_t leaderCount) const {  // :30-63
    Greedy g;
    int32_t remS = sliceCount, remL = leaderCount;
    std::vector<int32_t> rest;
    size_t idx = 0;
    if (leaderCount > 0) {
      const std::vector<int32_t> wl = sorted_wl(ds);
      for (; remL > 0 && idx < wl.size() && a_[wl[idx]].c.ls > 0; idx++) {
        g.count = w_add(g.count, 1);
        g.lastWL = wl[idx];
        remL = w_sub(remL, a_[wl[idx]].c.ls);
        remS = w_sub(remS, a_[wl[idx]].c.sswl);
      }
      rest = sorted(std::vector<int32_t>(wl.begin() + int64_t(idx), wl.end()));
    } else {
      rest = sorted(ds);
    }
    if (remL > 0) return Greedy{};
    for (idx = 0; remS > 0 && idx < rest.size() && a_[rest[idx]].c.ss > 0; idx++) {
      g.count = w_add(g.count, 1);
      g.last = rest[idx];
      remS = w_sub(remS, a_[rest[idx]].c.ss);
    }
    if (remS > 0) return Greedy{};
    g.fit = true;
    return g;
  }

  // fillInCountsHelper (:1658-1719) over a clone subtree, no inner slice
  // layers (pruneDomainsBelowThreshold passes a nil sliceSizeAtLevel, :379)
  void rollup(int32_t d, int level) {
    Node& n = a_[size_t(d)];
    if (!has_kids(d)) {
      if (level == p_.sliceLevelIdx) {
        n.c.ss = go_div32(n.c.st, p_.sliceSize);
        n.c.sswl = go_div32(n.c.swl, p_.sliceSize);
      }
      return;
    }
    const bool leaderReq = p_.leaderCount > 0;
    int32_t cap = 0, slc = 0, minD = INT32_MAX, minSD = INT32_MAX, lead = 0;
    bool has = false;
    for (int32_t k = a_[d].kid_begin; k < a_[d].kid_end; k++) {
      rollup(k, level + 1);
      const Ctr& c = a_[size_t(k)].c;
      cap = w_add(cap, c.st);
      slc = w_add(slc, c.ss);
      if (!leaderReq || c.ls > 0) {
        has = true;
        minD = std::min(w_sub(c.st, c.swl), minD);
        minSD = std::min(w_sub(c.ss, c.sswl), minSD);
      }
      lead = std::max(c.ls, lead);
    }
    Ctr& c = a_[size_t(d)].c;
    c.st = cap;
    int32_t sswl = 0;
    if (has) {
      c.swl = w_sub(cap, minD);
      sswl = w_sub(slc, minSD);
    } else {
      c.swl = 0;
    }
    c.ls = lead;
    if (level == p_.sliceLevelIdx) {
      slc = go_div32(c.st, p_.sliceSize);
      sswl = go_div32(c.swl, p_.sliceSize);
    }
    c.ss = slc;
    c.sswl = sswl;
  }
  void clear(int32_t d, bool leader_only) {  // clearState / clearLeaderCapacity (:323-341)
    Ctr& c = a_[size_t(d)].c;
    if (!leader_only) c.st = c.ss = 0;
    c.swl = c.sswl = c.ls = 0;
    for (int32_t k = a_[d].kid_begin; k < a_[d].kid_end; k++) clear(k, leader_only);
  }
  void prune_node(int32_t d, int32_t threshold) {  // :361-370
    const Ctr& c = a_[size_t(d)].c;
    if (c.ss < threshold) {
      clear(d, false);
      return;
    }
    if (p_.leaderCount > 0 && c.ls > 0 && c.sswl < threshold) clear(d, true);
  }
  void prune(const std::vector<int32_t>& ds, int32_t threshold) {  // :372-382
    for (int32_t d : ds)
      for (int32_t k = a_[d].kid_begin; k < a_[d].kid_end; k++) prune_node(k, threshold);
    for (int32_t d : ds) {
      rollup(d, p_.requestedLevelIdx);
      prune_node(d, threshold);
    }
  }

  // Go's math.Log / math.Log2 (FreeBSD e_log.c), so entropies round as in
  // the reference (built with -ffp-contract=off: no fused multiply-adds)
  static double go_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
    const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
                 L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    if (std::isnan(x) || std::isinf(x)) return x;
    if (x < 0) return std::nan("");
    if (x == 0) return -std::numeric_limits<double>::infinity();
    int ki;
    double f1 = std::frexp(x, &ki);
    if (f1 < M_SQRT2 / 2) {
      f1 *= 2;
      ki--;
    }
    const double f = f1 - 1, k = double(ki);
    const double s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
    const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    const double R = t1 + t2, hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
  }
  static double go_log2(double x) {
    int e;
    const double frac = std::frexp(x, &e);
    if (frac == 0.5) return double(e - 1);
    return go_log(frac) * (1 / 0.693147180559945309417232121458176568) + double(e);
  }
  double entropy(int32_t d) const {  // calculateEntropy (:186-209) of the children's states
    if (!has_kids(d)) return 0.0;
    int32_t total = 0;
    for (int32_t k = a_[d].kid_begin; k < a_[d].kid_end; k++) total = w_add(total, a_[size_t(k)].c.st);
    if (total == 0) return 0.0;
    double e = 0;
    const double tf = double(total);
    for (int32_t k = a_[d].kid_begin; k < a_[d].kid_end; k++)
      if (a_[size_t(k)].c.st > 0) {
        const double pi = double(a_[size_t(k)].c.st) / tf;
        e += -pi * go_log2(pi);
      }
    return e;
  }
  void sort_by_entropy(std::vector<int32_t>& ds) const {  // sortDomainsByCapacityAndEntropy (:211-231)
    auto cmp = [&](int32_t x, int32_t y) -> int {  // Go's int(b - a) on the int32 fields
      const Ctr &a = a_[x].c, &b = a_[y].c;
      if (const int32_t r = w_sub(b.ls, a.ls)) return r;
      if (const int32_t r = w_sub(b.sswl, a.sswl)) return r;
      const double ea = entropy(x), eb = entropy(y);
      return eb > ea ? 1 : (eb < ea ? -1 : 0);
    };
    for (size_t i = 1; i < ds.size(); i++)
      for (size_t j = i; j > 0 && cmp(ds[j - 1], ds[j]) > 0; j--) std::swap(ds[j - 1], ds[j]);
  }

  // selectOptimalDomainSetToFit (:81-147): nullopt = Go's nil
  std::optional<std::vector<int32_t>> select_optimal(std::vector<int32_t>& ds, int32_t sliceCount, bool byEntropy) {
    const Greedy g = greedy(ds, sliceCount, p_.leaderCount);
    if (!g.fit) return std::nullopt;
    if (byEntropy) sort_by_entropy(ds);
    const int32_t opt = std::max(g.count, 0);
    // [i][leadersLeft][stateLeft] -> the first domain list found with i domains
    std::vector<std::map<int32_t, std::map<int32_t, std::vector<int32_t>>>> pl(size_t(opt) + 1);
    pl[0][p_.leaderCount][w_mul(sliceCount, p_.sliceSize)] = {};
    for (int32_t d : ds) {
      const Ctr& c = a_[size_t(d)].c;
      for (int32_t i = opt; i > 0; i--)
        for (auto& lk : pl[size_t(i - 1)])
          for (auto& sk : lk.second) {
            const int32_t bl = lk.first, bs = sk.first;
            if (bl <= 0 && bs <= 0) continue;
            std::vector<int32_t> np = sk.second;
            np.push_back(d);
            if (bl > 0 && c.ls > 0) pl[size_t(i)][w_sub(bl, c.ls)].emplace(w_sub(bs, c.swl), np);  // with the leader
            if (c.ss > 0) pl[size_t(i)][bl].emplace(w_sub(bs, c.st), np);                         // without
          }
    }
    const auto it = pl[size_t(opt)].find(0);
    if (it == pl[size_t(opt)].end()) return std::nullopt;
    int32_t bestSlice = INT32_MIN;
    const std::vector<int32_t>* best = nullptr;
    for (auto& kv : it->second)
      if (kv.first > bestSlice && kv.first <= 0) {
        bestSlice = kv.first;
        best = &kv.second;
      }
    if (!best) return std::nullopt;
    return *best;
  }

  // findBestDomainsForBalancedPlacement (:236-290)
  int32_t find_best_domains(std::vector<int32_t>* best, bool* panic) {
    const int32_t sliceCount = go_div32(p_.count, p_.sliceSize);
    const int rl = p_.requestedLevelIdx;
    std::vector<std::vector<int32_t>> groups;  // sibling sets of the requested level, parents in index order
    if (rl == 0) {
      groups.emplace_back();
      for (int32_t i = 0; i < t_.size[0]; i++) groups.back().push_back(i);
    } else {
      const std::vector<int32_t>& co = *t_.co[size_t(rl - 1)];
      for (int32_t h = 0; h < t_.size[size_t(rl - 1)]; h++) {
        groups.emplace_back();
        for (int32_t i = co[size_t(h)]; i < co[size_t(h) + 1]; i++) groups.back().push_back(i);
      }
    }
    int32_t bestThreshold = 0, bestCount = 0;
    for (const auto& sib : groups) {
      std::vector<int32_t> cand = clone(rl, sib);
      const Greedy g = greedy(rl < p_.sliceLevelIdx ? lower(cand) : cand, sliceCount, p_.leaderCount);
      if (!g.fit) continue;
      if (g.count == 0) {
        *panic = true;
        return 0;
      }
      int32_t threshold = go_div32(sliceCount, g.count);  // balanceThresholdValue (:66-75)
      if (g.lastWL >= 0) threshold = std::min(threshold, a_[size_t(g.lastWL)].c.sswl);
      if (g.last >= 0) threshold = std::min(threshold, a_[size_t(g.last)].c.ss);
      int32_t thrWL = threshold;
      if (p_.leaderCount > 0 && g.last >= 0) thrWL = std::min(threshold, a_[size_t(g.last)].c.sswl);
      if (threshold < bestThreshold) continue;
      prune(cand, threshold);
      Greedy g2 = greedy(cand, sliceCount, p_.leaderCount);
      if (!g2.fit && thrWL < threshold) {  // retry reserving leader capacity
        if (thrWL <= 0 || thrWL < bestThreshold) continue;
        threshold = thrWL;
        cand = clone(rl, sib);
        prune(cand, threshold);
        g2 = greedy(cand, sliceCount, p_.leaderCount);
      }
      if (!g2.fit) continue;
      if (threshold > bestThreshold || (threshold == bestThreshold && g2.count < bestCount)) {
        bestThreshold = threshold;
        bestCount = g2.count;
        *best = cand;
      }
    }
    return bestThreshold;
  }

  // applyBalancedPlacementAlgorithm (:295-314) + placeSlicesOnDomainsBalanced (:149-184)
  std::string apply(int32_t threshold, std::vector<int32_t> cur, std::vector<int32_t>* out, int* fitLevel) {
    const int32_t sliceCount = go_div32(p_.count, p_.sliceSize);
    if (p_.requestedLevelIdx < p_.sliceLevelIdx) {
      auto res = select_optimal(cur, sliceCount, true);
      if (!res) return "TAS Balanced Placement: Cannot find optimal domain set to fit the request";
      cur = lower(*res);
      *fitLevel = p_.requestedLevelIdx + 1;
    } else {
      *fitLevel = p_.requestedLevelIdx;
    }
    auto res = select_optimal(cur, sliceCount, false);
    if (!res) return "TAS Balanced Placement: Cannot find optimal domain set to fit the request";
    if (sliceCount < w_mul(int32_t(res->size()), threshold)) return "TAS Balanced Placement: Not enough slices to meet the threshold";
    std::vector<int32_t> rd = sorted_wl(*res);
    int32_t extra = w_sub(sliceCount, w_mul(int32_t(rd.size()), threshold));
    int32_t leadersLeft = p_.leaderCount, take = 0;
    for (int32_t d : rd) {
      Ctr& c = a_[size_t(d)].c;
      if (leadersLeft > 0) {
        take = std::min(w_sub(c.sswl, threshold), extra);
        c.ls = 1;
        leadersLeft = w_sub(leadersLeft, 1);
      } else if (extra > 0) {
        take = std::min(w_sub(c.ss, threshold), extra);
        c.ls = 0;
      } else {
        c.ls = 0;
        take = 0;
      }
      c.st = w_mul(w_add(threshold, take), p_.sliceSize);
      c.ss = w_add(threshold, take);
      c.sswl = c.ss;
      c.swl = w_sub(c.st, c.ls);
      extra = w_sub(extra, take);
    }
    if (extra > 0 || leadersLeft > 0) return "TAS Balanced Placement: Not all slices or leaders could be placed";
    *out = rd;
    return "";
  }

  // ---- the descent over the clones (:928-996, balanced: no global level sort) ----
  enum F { F_ST, F_SS, F_SWL, F_SSWL };
  int32_t& fld(int32_t d, F f) {
    Ctr& c = a_[size_t(d)].c;
    return f == F_ST ? c.st : f == F_SS ? c.ss : f == F_SWL ? c.swl : c.sswl;
  }
  // findBestFitDomainBy (:1216-1231): first minimal value >= needed from `from`
  int32_t best_fit(const std::vector<int32_t>& ds, size_t from, int32_t needed, F f) {
    int32_t best = ds[from];
    int32_t bs = fld(best, f);
    for (size_t i = from; i < ds.size(); i++) {
      const int32_t v = fld(ds[i], f);
      if (v >= needed && v < bs) {
        best = ds[i];
        bs = v;
      }
    }
    return best;
  }
  // consumeWithLeadersGeneric (:1348-1403), BestFit
  int32_t consume(int32_t dom, const std::vector<int32_t>& ds, size_t from, int32_t* remP, int32_t* remL, F wl, F pr,
                  int32_t sliceSize, bool slices, bool* completed) {
    if (fld(dom, wl) >= *remP && a_[size_t(dom)].c.ls >= *remL) {
      if (slices) {
        dom = best_fit(ds, from, *remP, *remL > 0 ? F_SSWL : F_SS);
        wl = F_SSWL;
        pr = F_SS;
      } else {
        dom = best_fit(ds, from, *remP, *remL > 0 ? F_SWL : F_ST);
        wl = F_SWL;
        pr = F_ST;
      }
    }
    Ctr& c = a_[size_t(dom)].c;
    if (fld(dom, wl) >= *remP && c.ls >= *remL) {
      fld(dom, pr) = *remP;
      c.ls = *remL;
      c.st = w_mul(*remP, sliceSize);
      *completed = true;
      return dom;
    }
    if (slices) {
      if (fld(dom, wl) > *remP) fld(dom, wl) = *remP;
      if (c.ls > *remL) c.ls = *remL;
      c.st = w_mul(fld(dom, wl), sliceSize);
      *remL = w_sub(*remL, c.ls);
      *remP = w_sub(*remP, fld(dom, wl));
      *completed = false;
      return dom;
    }
    *remP = w_sub(*remP, fld(dom, wl));
    *remL = w_sub(*remL, c.ls);
    if (fld(dom, wl) > *remP) fld(dom, wl) = *remP;
    if (c.ls > *remL) c.ls = *remL;
    *completed = false;
    return dom;
  }
  // updateCountsToMinimumGeneric (:1405-1469), BestFit; false: Go's nil
  bool update_counts(const std::vector<int32_t>& ds, int32_t count, int32_t leaderCount, int32_t sliceSize, bool slices,
                     std::vector<int32_t>* out) {
    out->clear();
    int32_t remP = slices ? go_div32(count, sliceSize) : count, remL = leaderCount;
    for (size_t i = 0; i < ds.size(); i++) {
      int32_t dom = ds[i];
      if (remL > 0) {
        bool done = false;
        const int32_t d = slices ? consume(dom, ds, i, &remP, &remL, F_SSWL, F_SS, sliceSize, true, &done)
                                 : consume(dom, ds, i, &remP, &remL, F_SWL, F_ST, 1, false, &done);
        out->push_back(d);
        if (done) return true;
        continue;
      }
      Ctr* c = &a_[size_t(dom)].c;
      if (slices) {
        if (c->ss >= remP) dom = best_fit(ds, i, remP, F_SS);
        c = &a_[size_t(dom)].c;
        c->ls = 0;
        if (c->ss >= remP) {
          c->st = w_mul(remP, sliceSize);
          c->ss = remP;
          out->push_back(dom);
          return true;
        }
        c->st = w_mul(c->ss, sliceSize);
        remP = w_sub(remP, c->ss);
        out->push_back(dom);
        continue;
      }
      if (c->st >= remP) dom = best_fit(ds, i, remP, F_ST);
      c = &a_[size_t(dom)].c;
      c->ls = 0;
      if (c->st >= remP) {
        c->st = remP;
        out->push_back(dom);
        return true;
      }
      remP = w_sub(remP, c->st);
      out->push_back(dom);
    }
    out->clear();
    return false;
  }
  void descend(std::vector<int32_t> cur, int fitLevel, Result* r) {
    std::vector<int32_t> next;
    if (!update_counts(cur, p_.count, p_.leaderCount, p_.sliceSize, true, &next)) next.clear();  // :928
    cur = next;
    for (int level = fitLevel; level < t_.L - 1; level++) {  // :937-971 (the :930 loop is skipped)
      int32_t sol = p_.sliceSize;
      if (level >= p_.sliceLevelIdx) {
        sol = 1;
        if (p_.sliceSizeAtLevel && p_.sliceSizeAtLevel[level + 1] != 0) sol = p_.sliceSizeAtLevel[level + 1];
      }
      std::vector<int32_t> nc, add;
      for (int32_t d : cur) {
        std::vector<int32_t> kids;
        for (int32_t k = a_[d].kid_begin; k < a_[d].kid_end; k++) kids.push_back(k);
        kids = sorted(kids);
        if (sol > 1)
          for (int32_t k : kids) {
            Ctr& c = a_[size_t(k)].c;
            c.ss = go_div32(c.st, sol);
            c.sswl = go_div32(c.swl, sol);
          }
        const Ctr& pc = a_[size_t(d)].c;
        if (!update_counts(kids, pc.st, pc.ls, sol, sol > 1, &add)) add.clear();
        nc.insert(nc.end(), add.begin(), add.end());
      }
      cur = nc;
    }
    // buildAssignment (:1472-1501): leaf order, zero counts dropped; leaders
    // are copies with state = leaderState (:975-994)
    std::sort(cur.begin(), cur.end(), [&](int32_t x, int32_t y) { return lex_less(x, y); });
    for (int32_t d : cur) {
      const Ctr& c = a_[size_t(d)].c;
      if (p_.leaderCount > 0 && c.ls > 0) r->leaders.emplace_back(a_[size_t(d)].idx, c.ls);
      if (c.st != 0 && (p_.leaderCount == 0 || c.st > 0)) r->workers.emplace_back(a_[size_t(d)].idx, c.st);
    }
  }
};

}  // namespace ktas_balanced
