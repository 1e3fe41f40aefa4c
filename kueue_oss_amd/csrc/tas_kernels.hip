// tas_kernels.hip — CDNA4 (gfx950) kernels for Kueue's TAS evaluation path.
//
// Three stages per batch of PodSet-group evaluations ("evals"), all integer,
// all HBM/latency bound (no MFMA: there is no matrix-shaped work here):
//
//  K1 fill_leaves   — fillInCounts leaf loop (tas_flavor_snapshot.go:1578-1643):
//                     per (leaf, eval) taint/selector masks, remaining capacity
//                     and Requests.CountInWithLimitingResource (requests.go:183-217)
//                     with exact int64 magic-number division, leader split,
//                     wave-aggregated ExclusionStats.  One block = 256 leaves x
//                     kEvalsPerBlock evals so the SoA snapshot columns are read
//                     from HBM once per block and re-served from L1/L2.
//  K2 rollup_level  — fillInCountsHelper (:1658-1719) bottom-up, one launch per
//                     level, one thread per parent domain over its CSR children.
//  K3 select        — phase 2 (findLevelWithFitDomains :1236-1321,
//                     updateCountsToMinimumGeneric :1405-1469, the descent
//                     :925-971, buildAssignment :1490-1501): one 64-lane wave per
//                     eval executing the reference's sequential greedy with
//                     wave-parallel primitives (arg-min reductions, LDS bitonic
//                     sort, lazy sorted iteration, histogram threshold select).
//
// Every scalar of the greedy is held redundantly by all 64 lanes and every
// mutation of a domain counter is stored by all lanes (so each lane reads back
// its own store: no cross-lane global-memory hazards).  LDS traffic between
// lanes is ordered with wave_sync().
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "tas_internal.h"

namespace ktas {

// ----------------------------------------------------------------------------
// Go integer helpers
// ----------------------------------------------------------------------------
__device__ __forceinline__ int32_t w_add(int32_t a, int32_t b) { return int32_t(uint32_t(a) + uint32_t(b)); }
__device__ __forceinline__ int32_t w_sub(int32_t a, int32_t b) { return int32_t(uint32_t(a) - uint32_t(b)); }
__device__ __forceinline__ int32_t w_mul(int32_t a, int32_t b) { return int32_t(uint32_t(a) * uint32_t(b)); }
// ---- lane exchange without LDS ----
// bfly<M>(v): the partner value of step M of an ASCENDING butterfly (M = 1,
// 2, 4, ..., 32) in one VALU op: DPP quad_perm for 1 and 2, the half-row and
// row mirrors for 4 and 8 (after the steps below M every lane of an aligned
// M-group holds the same partial, so the mirror reads the partner group's),
// and the gfx950 permlane swaps across rows for 16 and 32 (exact xor: the
// swap returns the lane's own row value and its partner row's).  No ds_bpermute /
// ds_swizzle, so no LDS round trip and no lgkmcnt wait per step.
__device__ __forceinline__ int lane_id();
template <int M>
__device__ __forceinline__ uint32_t bfly(uint32_t v) {
  if constexpr (M == 1) return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  else if constexpr (M == 2) return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  else if constexpr (M == 4) return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  else if constexpr (M == 8) return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x140, 0xF, 0xF, false));  // row_mirror
  else if constexpr (M == 16) {  // {r0, r1} = {own, partner} in some order; equal values are interchangeable
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return uint32_t(r[0]) == v ? uint32_t(r[1]) : uint32_t(r[0]);
  } else {
    static_assert(M == 32, "butterfly steps are 1..32");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return uint32_t(r[0]) == v ? uint32_t(r[1]) : uint32_t(r[0]);
  }
}
template <int M>
__device__ __forceinline__ uint64_t bfly64(uint64_t v) {
  return (uint64_t(bfly<M>(uint32_t(v >> 32))) << 32) | bfly<M>(uint32_t(v));
}
template <int M>
__device__ __forceinline__ int32_t bfly_i(int32_t v) { return int32_t(bfly<M>(uint32_t(v))); }
// Ascending butterfly over the aligned groups of F lanes (F = 1..64):
// step(integral_constant<M>) folds the partner of step M into the lane's
// partial; a commutative, associative fold leaves every lane of a group
// holding the group's result.
template <class Step>
__device__ __forceinline__ void butterfly(int F, Step step) {
  if (F >= 2) step(std::integral_constant<int, 1>());
  if (F >= 4) step(std::integral_constant<int, 2>());
  if (F >= 8) step(std::integral_constant<int, 4>());
  if (F >= 16) step(std::integral_constant<int, 8>());
  if (F >= 32) step(std::integral_constant<int, 16>());
  if (F >= 64) step(std::integral_constant<int, 32>());
}
// step m of an ascending butterfly (m = 1, 2, 4, ..., 32; see bfly) for
// reduction loops `for (m = 1; m <= 32; m <<= 1)` (unrolled: m is a constant)
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int m) {
  switch (m) {
    case 1: return bfly<1>(v);
    case 2: return bfly<2>(v);
    case 4: return bfly<4>(v);
    case 8: return bfly<8>(v);
    case 16: return bfly<16>(v);
    default: return bfly<32>(v);
  }
}
__device__ __forceinline__ int32_t xor_lane(int32_t v, int m) { return int32_t(xor_lane(uint32_t(v), m)); }
template <class Op>
__device__ __forceinline__ int32_t group_reduce(int32_t v, int F, Op op) {
  butterfly(F, [&](auto m) { v = op(v, bfly_i<decltype(m)::value>(v)); });
  return v;
}
struct OpWAdd {
  __device__ int32_t operator()(int32_t a, int32_t b) const { return int32_t(uint32_t(a) + uint32_t(b)); }
};
struct OpMin {
  __device__ int32_t operator()(int32_t a, int32_t b) const { return a < b ? a : b; }
};
struct OpMax {
  __device__ int32_t operator()(int32_t a, int32_t b) const { return a > b ? a : b; }
};

// Go int32 division (truncating; MinInt32 / -1 == MinInt32).  b == 0 is
// rejected on the host (Go panics).
__device__ __forceinline__ int32_t go_div32(int32_t a, int32_t b) {
  if (b == -1) return int32_t(0u - uint32_t(a));
  return b == 0 ? 0 : a / b;
}

// Exact unsigned 64-bit division by an invariant divisor (host-computed magic).
__device__ __forceinline__ uint64_t udiv_magic(uint64_t n, const DevTerm& t) {
  if (t.pow2) return n >> t.shift;
  uint64_t q = __umul64hi(t.magic, n);
  if (t.add) {
    uint64_t x = ((n - q) >> 1) + q;
    return x >> t.shift;
  }
  return q >> t.shift;
}

// max(int32(cap / val), 0) with Go's truncating int64 division (val != 0).
__device__ __forceinline__ int32_t count_term(int64_t cap, const DevTerm& t) {
  uint64_t ucap = cap < 0 ? (0ull - uint64_t(cap)) : uint64_t(cap);
  uint64_t q = udiv_magic(ucap, t);
  bool negq = (cap < 0) != (t.neg != 0);
  uint64_t sq = negq ? (0ull - q) : q;
  int32_t c = int32_t(uint32_t(sq));
  return c > 0 ? c : 0;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Orders one wave's own LDS / global accesses across its lanes.  Wavefront
// scope: a wave's vector memory and LDS operations complete in issue order
// (LLVM AMDGPU memory model, GFX942/950: a wavefront-scope fence emits no
// wait), so this is a compiler barrier only.  A workgroup-scope fence would
// wait for every outstanding store (s_waitcnt vmcnt(0)): one memory round
// trip per call, a PCIe round trip after stores to pinned host memory.  The
// select path's lists in global scratch are wave-private (one wave per
// workgroup), so their cross-lane ordering needs wavefront scope only.
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }
__device__ __forceinline__ void wave_sync() {
  wave_fence();
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// value of lane `src` (wave-uniform: a ballot's first set bit, 0, 63) by
// v_readlane into an SGPR, no LDS round trip
template <class T>
__device__ __forceinline__ T bcast(T v, int src) {
  static_assert(sizeof(T) == 4, "32-bit lane values");
  return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}
__device__ __forceinline__ uint64_t bcast64(uint64_t v, int src) {
  return (uint64_t(bcast(uint32_t(v >> 32), src)) << 32) | bcast(uint32_t(v), src);
}
// per-lane source (scans, gathers): ds_bpermute
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
  lo = __shfl(lo, src, 64);
  hi = __shfl(hi, src, 64);
  return (uint64_t(hi) << 32) | lo;
}

__device__ __forceinline__ bool key_lt(const Key& a, const Key& b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
__device__ __forceinline__ bool key_le(const Key& a, const Key& b) { return !key_lt(b, a); }
__device__ __forceinline__ Key key_max() { return Key{~0ull, ~0ull}; }
__device__ __forceinline__ Key wave_min_key(Key k) {
  butterfly(64, [&](auto m) {
    constexpr int M = decltype(m)::value;
    const Key o{bfly64<M>(k.hi), bfly64<M>(k.lo)};
    if (key_lt(o, k)) k = o;
  });
  return k;
}
// Wave arg-min / arg-max over (value, index) pairs: ties keep the smaller
// (arg-min) or larger (arg-max) index (lexicographic, so the butterfly's
// order does not matter).
__device__ __forceinline__ void wave_argmin(uint64_t& v, int32_t& i) {
  butterfly(64, [&](auto m) {
    constexpr int M = decltype(m)::value;
    const uint64_t ov = bfly64<M>(v);
    const int32_t oi = bfly_i<M>(i);
    if (ov < v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  });
}
__device__ __forceinline__ void wave_argmax(uint64_t& v, int32_t& i) {
  butterfly(64, [&](auto m) {
    constexpr int M = decltype(m)::value;
    const uint64_t ov = bfly64<M>(v);
    const int32_t oi = bfly_i<M>(i);
    if (ov > v || (ov == v && oi > i)) {
      v = ov;
      i = oi;
    }
  });
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  butterfly(64, [&](auto m) {
    const uint64_t o = bfly64<decltype(m)::value>(v);
    v = o < v ? o : v;
  });
  return v;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
  butterfly(64, [&](auto m) { v += int64_t(bfly64<decltype(m)::value>(uint64_t(v))); });
  return v;
}
// Exclusive wave scan (int add) with DPP, no LDS: row_shr 1/2/4/8 scan each
// row of 16, row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry the
// row totals; the total is lane 63's inclusive sum (v_readlane).
__device__ __forceinline__ int wave_incl_scan(int x) {  // wrapping int add
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}
// Segmented inclusive wave scan: lane gets op over lanes [max(seg0, ...), lane]
// of its segment (seg0: the lane's segment start; segments are contiguous).
// The same DPP steps as wave_incl_scan, each applied only where its source
// lane lies in the lane's segment.
template <class Op>
__device__ __forceinline__ int32_t seg_incl_scan(int32_t x, int lane, int seg0, Op op) {
  const int r = lane & 15;
  int32_t t;
  t = __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  if (r >= 1 && lane - 1 >= seg0) x = op(x, t);
  t = __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  if (r >= 2 && lane - 2 >= seg0) x = op(x, t);
  t = __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  if (r >= 4 && lane - 4 >= seg0) x = op(x, t);
  t = __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  if (r >= 8 && lane - 8 >= seg0) x = op(x, t);
  t = __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 (rows 1, 3)
  if (((lane >> 4) & 1) && seg0 <= (lane & ~15) - 1) x = op(x, t);
  t = __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 (rows 2, 3)
  if (lane >= 32 && seg0 <= 31) x = op(x, t);
  return x;
}
__device__ __forceinline__ int wave_excl_scan(int v, int* total) {
  const int x = wave_incl_scan(v);
  *total = __builtin_amdgcn_readlane(x, 63);
  return x - v;
}

__device__ __forceinline__ int32_t wave_sum_wrap32(int32_t v) { return group_reduce(v, 64, OpWAdd()); }

__device__ __forceinline__ uint32_t s_asc(int32_t x) { return uint32_t(x) ^ 0x80000000u; }
__device__ __forceinline__ uint32_t s_desc(int32_t x) { return ~(uint32_t(x) ^ 0x80000000u); }

// sortedDomains comparator (:1544-1564): sliceState desc (asc if LFC), state asc, levelValues asc.
__device__ __forceinline__ Key key_plain(bool lfc, int32_t ss, int32_t s, int32_t idx) {
  uint64_t k0 = lfc ? s_asc(ss) : s_desc(ss);
  return Key{(k0 << 32) | s_asc(s), uint64_t(uint32_t(idx))};
}
// sortedDomainsWithLeader comparator (:1511-1535): leaderState desc,
// sliceStateWithLeader desc (asc if LFC), stateWithLeader asc, levelValues asc.
__device__ __forceinline__ Key key_wl(bool lfc, int32_t ls, int32_t sswl, int32_t swl, int32_t idx) {
  uint64_t k1 = lfc ? s_asc(sswl) : s_desc(sswl);
  return Key{(uint64_t(s_desc(ls)) << 32) | k1, (uint64_t(s_asc(swl)) << 32) | uint32_t(idx)};
}

// ----------------------------------------------------------------------------
// K1: fillInCounts leaf loop
// ----------------------------------------------------------------------------
constexpr int kFillThreads = 256;
constexpr int kEvalsPerBlock = 16;

enum ExclKind : int { EX_NONE = 0, EX_TAINT = 1, EX_SELECTOR = 2, EX_RESOURCE = 3, EX_AFFINITY = 4, EX_TOPOLOGY = 5,
                      EX_DEAD = 6 };  // EX_DEAD: the leaf is out of the snapshot (counted nowhere)
__device__ __forceinline__ bool leaf_out(const DevSnap& s, int leaf) { return s.leaf_dead && s.leaf_dead[leaf]; }
// ExclusionStats slots of the LDS / per-block partials: [0] nodeSelector,
// [1] affinity, [2] topologyDomain, then one per taint string, then one per
// resource column.
constexpr int kStatFixed = 3;
// belongsToRequiredDomain (:1649-1656) on every leaf, after the hostname-only
// filters (:1613-1617): the host turns the required domain's DomainID prefix
// into the leaf range [db, de) (db < 0: no required domain).
__device__ __forceinline__ bool outside_domain(int db, int de, int leaf) { return db >= 0 && (leaf < db || leaf >= de); }

__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(uint64_t(v)));
  uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(uint64_t(v) >> 32));
  return int64_t((uint64_t(hi) << 32) | lo);
}
// A request term with every field in scalar registers (wave-uniform).
__device__ __forceinline__ DevTerm uni_term(const DevTerm& t) {
  DevTerm u;
  u.val = uni64(t.val);
  u.magic = uint64_t(uni64(int64_t(t.magic)));
  u.col = uni(t.col);
  u.shift = uint8_t(uni(t.shift));
  u.add = uint8_t(uni(t.add));
  u.pow2 = uint8_t(uni(t.pow2));
  u.neg = uint8_t(uni(t.neg));
  return u;
}

// CountInWithLimitingResource (requests.go:190-215) over the staged columns
// in ascending column order, as selects: the column tests, the term fields
// and the division variant are wave-uniform (scalar branches), the per-leaf
// parts — a missing resource, the running minimum, the limiting column —
// are v_cndmask, so no divergent branch (no exec-mask bookkeeping on the
// CU's one scalar unit per term).  Counts are >= 0 (count_term), a zero
// request counts MaxInt32 and never lowers the minimum; the first missing
// resource (capacity absent, request non-zero) returns 0 with that column.
template <int NS>
__device__ __forceinline__ int32_t count_slots_sel(const int (&scol)[NS], const int64_t (&cap)[NS], const DevTerm* terms,
                                                   uint32_t mask, const DevTerm* lterms, uint32_t lmask, uint32_t presm,
                                                   bool sub_leader, int* lim_out) {
  int32_t result = 0;
  bool any = false, done = false;
  int lim = -1;
#pragma unroll
  for (int k = 0; k < NS; k++) {
    const int col = scol[k];
    if (col >= 0 && ((mask >> col) & 1u)) {  // wave-uniform
      const DevTerm t = uni_term(terms[__popc(mask & ((1u << col) - 1u))]);
      int64_t c = cap[k];
      if (sub_leader && ((lmask >> col) & 1u)) {
        const DevTerm lt = uni_term(lterms[__popc(lmask & ((1u << col) - 1u))]);
        c = int64_t(uint64_t(c) - uint64_t(lt.val));
      }
      const int32_t cnt = t.val == 0 ? 0x7fffffff : count_term(c, t);
      const bool miss = t.val != 0 && !((presm >> col) & 1u);
      const bool upd = !done && (miss || !any || cnt < result);
      result = upd ? (miss ? 0 : cnt) : result;
      lim = upd ? col : lim;
      done = done || miss;
      any = true;
    }
  }
  *lim_out = lim;
  return any ? result : 0;
}

// Sorted-set membership of a per-lane id in a wave-uniform id list.
__device__ __forceinline__ bool sorted_contains(const int32_t* v, int len, int32_t x) {
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < len && v[lo] == x;
}

// Required node affinity of one leaf (fillInCounts :1605-1610):
// nodeaffinity.NodeSelector.Match (nodeaffinity.go:84-103, :190-201) with
// the terms ORed and each term's requirements ANDed; a compiled requirement
// (host: labels.Requirement / fields selector folded against the snapshot's
// label dictionaries) is "the leaf's id is in a sorted set" XOR negate.
// [rb, re) is wave-uniform; an empty range matches no leaf (no terms).
// Label value id of `leaf` in column `col` (wave-uniform): one of the first
// kStagedLabels columns held in registers (l0..l3), else a load.
__device__ __forceinline__ int32_t staged_label(const DevSnap& s, int leaf, int col, int32_t l0, int32_t l1, int32_t l2,
                                                int32_t l3) {
  if (col == 0) return l0;
  if (col == 1) return l1;
  if (col == 2) return l2;
  if (col == 3) return l3;
  return s.label_values[int64_t(col) * s.N + leaf];
}
template <class LabelAt>
__device__ __forceinline__ bool affinity_match(const DevBatch& b, int rb, int re, int leaf, LabelAt label_at) {
  if (rb >= re) return false;
  bool any = false, cur = true;
  int term = uni(b.aff[rb].term);
  for (int r = rb; r < re; r++) {
    const int t = uni(b.aff[r].term);
    if (t != term) {
      any = any || cur;
      cur = true;
      term = t;
    }
    if (cur) {
      const int col = uni(b.aff[r].col);
      const int32_t v = col < 0 ? int32_t(leaf) : label_at(col);
      const bool in = sorted_contains(b.aff_vals + uni(b.aff[r].begin), uni(b.aff[r].len), v);
      cur = in != (uni(b.aff[r].negate) != 0);
    }
  }
  return any || cur;
}

// nodeSelector pairs beyond the inline ones (KUEUE_TAS_F_SELECTOR_EXT): one
// Equals requirement per key (labels.ValidatedSelectorFromSet, selector.go:
// 954-968), each compiled to "the leaf's value id is in a sorted set" XOR
// negate like an affinity requirement; every one must match (:1599-1603).
template <class LabelAt>
__device__ __forceinline__ bool selector_ext_match(const DevBatch& b, int rb, int re, int leaf, LabelAt label_at) {
  for (int r = rb; r < re; r++) {
    const int col = uni(b.aff[r].col);
    const int32_t v = col < 0 ? int32_t(leaf) : label_at(col);
    if (sorted_contains(b.aff_vals + uni(b.aff[r].begin), uni(b.aff[r].len), v) == (uni(b.aff[r].negate) != 0))
      return false;
  }
  return true;
}

// Requests.CountIn / CountInWithLimitingResource over up to MAXT terms held in
// registers (fully unrolled: no runtime-indexed private arrays).  Terms are in
// ascending column (= resource name) order, so the first missing key and the
// first minimum are Go's limiting resource with the alphabetical tie-break.
template <int MAXT>
__device__ __forceinline__ int32_t count_in_regs(const DevTerm* terms, int nt, uint32_t pres, const int64_t (&caps)[MAXT],
                                                 int* lim_out) {
  int32_t result = 0;
  bool any = false, done = false;
  int lim = -1;
#pragma unroll
  for (int i = 0; i < MAXT; i++) {
    if (i < nt && !done) {
      const DevTerm t = uni_term(terms[i]);
      if (!((pres >> t.col) & 1u) && t.val != 0) {
        lim = t.col;
        result = 0;
        any = true;
        done = true;
      } else {
        int32_t c = t.val == 0 ? 0x7fffffff : count_term(caps[i], t);
        if (!any || c < result) {
          result = c;
          lim = t.col;
          any = true;
        }
      }
    }
  }
  *lim_out = lim;
  return any ? result : 0;
}

__device__ __forceinline__ Key key_min2(const Key& a, const Key& b) { return key_lt(b, a) ? b : a; }
__device__ __forceinline__ Key key_max2(const Key& a, const Key& b) { return key_lt(a, b) ? b : a; }

// Per-eval parameters of a fill chunk, staged in LDS once per block so the
// per-eval loop has no dependent global loads (eval record -> taint row).
// The fields the per-eval loop reads come first, in 16-byte groups: the loop
// fetches them with three ds_read_b128 and one wait (not one LDS round trip
// per field), the selector pairs with four more when the eval has selectors.
struct alignas(16) FillEvalParams {
  int32_t eid, nsel, slice_size, slice_level;
  int32_t inner, sel_far, aff_begin, aff_end;  // inner: ssal of the leaf level; sel_far: a nodeSelector
                                               // column beyond the kStagedLabels held in registers;
                                               // aff_begin < 0: no required node affinity
  int32_t dom_begin, dom_end, taint_off, sig_new;  // replacement domain leaf range (dom_begin < 0: none);
                                                   // sig_new 1: first position of its signature run
  int32_t run, rmask, lmask, sx_begin;  // signature run (DevBatch::fill_run); the run's worker / leader column
                                        // masks; nodeSelector requirements beyond the inline pairs (-1: none)
  int32_t sel_col[KUEUE_TAS_MAX_SELECTORS], sel_val[KUEUE_TAS_MAX_SELECTORS];
  int32_t sx_end, pad[3];
  // the nodeSelector as one masked compare of the leaf's packed staged label
  // ids (fill_pair_kernel): column c < kStagedLabels is the 16-bit field c of
  // the 64-bit key; sel_fast 1 when every pair is a staged column and every
  // staged column's ids fit 16 bits (kueue_tas_ctx::labels16), else the loop
  // over sel_col / sel_val.  A pair whose value id no leaf has, or two pairs
  // on one column with different values, set a want bit outside the mask
  // (never equal: every leaf mismatches, as labels.SelectorFromSet does).
  uint32_t sel_mlo, sel_mhi, sel_wlo, sel_whi;
  int32_t sel_fast;
  // 1: the class is simple (no leader, one-pod slices at the leaf level, no
  // inner slice rounding), so its sliceState equals its state at every level
  // and the class row's sliceState field is not stored: every reader takes
  // the state field instead (ss_off)
  int32_t ss_alias;
  int32_t lfc_slot;  // the class's fast-LFC table slot, -1: none
  int32_t ctr_row;   // the class row's offset in DevBatch::counters, in units of SD int32s: rows
                     // hold 1 field (simple), 2 (state, sliceState) or 5 (and the leader fields)
};
static_assert(KUEUE_TAS_MAX_SELECTORS == 8, "selector pairs are fetched as two int4 each");
constexpr int kFillTilesPerBlock = 1;  // leaf tiles of one staged-fill block
constexpr int kStagedProfiles = 32;  // taint-profile rows staged in LDS (more: read from global)

// Everything fill_pair_kernel needs about one fill position, built by the
// host in fill order (DevBatch::fill_pos): the parameters (pad[0] = the
// chunk's base flags, pad[1..2] = its assumed-usage range), the eval's
// taint-profile row and its run's worker | leader terms.  A block copies its
// chunk's records into LDS with one coalesced pass: one memory round trip
// instead of the chain chunk -> eval ids -> eval records -> rows / terms.
constexpr int kPosTerms = 16;  // 2 * the largest staged column count
struct alignas(16) FillPos {
  FillEvalParams p;
  int32_t taint[kStagedProfiles];
  DevTerm term[kPosTerms];
};
static_assert(sizeof(FillPos) % 16 == 0, "FillPos is copied as int4");
// Offset of the sliceState field in a class row (counters[row]): SD, or 0
// for a simple class whose sliceState is its state (FillEvalParams::ss_alias).
__device__ __forceinline__ int64_t ss_off(const DevBatch& b, int row, int64_t SD) {
  return b.fill_pos[row].p.ss_alias ? 0 : SD;
}
// The class row of fill position `row` (FillEvalParams::ctr_row).
__device__ __forceinline__ int32_t* ctr_base(const DevBatch& b, int row) {
  return b.counters + int64_t(b.fill_pos[row].p.ctr_row) * b.ctr_sd;
}

template <int MAXT>
__global__ __launch_bounds__(kFillThreads) void fill_leaves_kernel(DevSnap s, DevBatch b) {

  __shared__ DevEval sh_ev[kEvalsPerBlock];
  __shared__ DevTerm sh_terms[kEvalsPerBlock][2 * MAXT];
  __shared__ int64_t sh_wlead[kEvalsPerBlock][MAXT];  // leader value on each worker term's column

  const int e0 = b.fill_chunks[2 * blockIdx.y];
  const int ne = b.fill_chunks[2 * blockIdx.y + 1];
  if (threadIdx.x < ne) sh_ev[threadIdx.x] = b.evals[b.fill_ids[e0 + threadIdx.x]];
  __syncthreads();
  for (int e = 0; e < ne; e++) {
    const DevEval& ev = sh_ev[e];
    if (threadIdx.x < ev.nreq) sh_terms[e][threadIdx.x] = b.terms[ev.term_begin + threadIdx.x];
    if (threadIdx.x < ev.nlead) sh_terms[e][MAXT + threadIdx.x] = b.terms[ev.lead_begin + threadIdx.x];
  }
  __syncthreads();
  for (int e = 0; e < ne; e++) {
    const DevEval& ev = sh_ev[e];
    if (threadIdx.x < ev.nreq) {
      int col = sh_terms[e][threadIdx.x].col;
      int64_t v = 0;
      for (int j = 0; j < ev.nlead; j++)
        if (sh_terms[e][MAXT + j].col == col) v = sh_terms[e][MAXT + j].val;
      sh_wlead[e][threadIdx.x] = v;
    }
  }
  __syncthreads();

  const int leaf = blockIdx.x * kFillThreads + threadIdx.x;
  const bool valid = leaf < s.N;
  const int N = s.N;
  const int gleaf = s.level_off[s.L - 1] + leaf;
  const uint32_t fp = valid ? s.free_present[leaf] : 0u;
  const uint32_t up = valid ? s.usage_present[leaf] : 0u;
  const int prof = (valid && s.taint_profile) ? s.taint_profile[leaf] : 0;
  const int lane = lane_id();

  for (int e = 0; e < ne; e++) {
    const DevEval& ev = sh_ev[e];
    const int eid = b.fill_ids[e0 + e];
    const DevTerm* wt = sh_terms[e];
    const DevTerm* lt = sh_terms[e] + MAXT;
    // wave-uniform copies (scalar registers: uniform branches below)
    const uint32_t flags = uint32_t(uni(int32_t(ev.flags)));
    const int nreq = uni(ev.nreq), nlead = uni(ev.nlead), nsel = uni(ev.nsel);
    const int abeg = uni(ev.assumed_begin), aend = uni(ev.assumed_end);
    const bool leader = (flags & KUEUE_TAS_F_LEADER) != 0;
    int32_t state = 0, swl = 0, ls = 0;
    int kind = (valid && leaf_out(s, leaf)) ? EX_DEAD : EX_NONE, id = -1;
    if (valid && kind == EX_NONE) {
      if (s.lowest_is_hostname) {
        if (s.taint_profile) {
          int t = b.taint_table[ev.taint_table + prof];
          if (t >= 0) {
            kind = EX_TAINT;
            id = t;
          }
        }
        if (kind == EX_NONE) {
          for (int k = 0; k < nsel; k++) {
            if (s.label_values[int64_t(ev.sel_col[k]) * N + leaf] != ev.sel_val[k]) {
              kind = EX_SELECTOR;
              break;
            }
          }
        }
        if (kind == EX_NONE && uni(ev.sx_begin) >= 0 &&
            !selector_ext_match(b, uni(ev.sx_begin), uni(ev.sx_end), leaf,
                                [&](int col) { return s.label_values[int64_t(col) * N + leaf]; }))
          kind = EX_SELECTOR;
        if (kind == EX_NONE && (flags & KUEUE_TAS_F_AFFINITY) &&
            !affinity_match(b, uni(ev.aff_begin), uni(ev.aff_end), leaf,
                            [&](int col) { return s.label_values[int64_t(col) * N + leaf]; }))
          kind = EX_AFFINITY;
      }
      if (kind == EX_NONE && outside_domain(uni(ev.dom_begin), uni(ev.dom_end), leaf)) kind = EX_TOPOLOGY;
      if (kind == EX_NONE) {
        const bool sim = (flags & KUEUE_TAS_F_SIMULATE_EMPTY) != 0;
        uint32_t pres = fp | (sim ? 0u : up);
        int a_lo = 0, a_hi = 0;
        if (aend > abeg) {
          int lo = abeg, hi = aend;
          while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (b.assumed[mid].leaf < leaf) lo = mid + 1;
            else hi = mid;
          }
          a_lo = lo;
          a_hi = lo;
          while (a_hi < aend && b.assumed[a_hi].leaf == leaf) {
            pres |= 1u << b.assumed[a_hi].col;
            a_hi++;
          }
        }
        // remaining capacity: free - used - assumed (Requests.Sub, requests.go:90-94)
        int64_t wcap[MAXT], lcap[MAXT];
#pragma unroll
        for (int i = 0; i < MAXT; i++) {
          wcap[i] = 0;
          lcap[i] = 0;
          if (i < nreq) {
            const int col = wt[i].col;
            int64_t c = s.free_cap[int64_t(col) * N + leaf];
            if (!sim) c = int64_t(uint64_t(c) - uint64_t(s.tas_usage[int64_t(col) * N + leaf]));
            for (int a = a_lo; a < a_hi; a++)
              if (b.assumed[a].col == col) c = int64_t(uint64_t(c) - uint64_t(b.assumed[a].value));
            wcap[i] = c;
          }
          if (leader && i < nlead) {
            const int col = lt[i].col;
            int64_t c = s.free_cap[int64_t(col) * N + leaf];
            if (!sim) c = int64_t(uint64_t(c) - uint64_t(s.tas_usage[int64_t(col) * N + leaf]));
            for (int a = a_lo; a < a_hi; a++)
              if (b.assumed[a].col == col) c = int64_t(uint64_t(c) - uint64_t(b.assumed[a].value));
            lcap[i] = c;
          }
        }
        int lim = -1;
        state = count_in_regs<MAXT>(wt, nreq, pres, wcap, &lim);
        if (state == 0 && lim >= 0) {
          kind = EX_RESOURCE;
          id = lim;
        }
        swl = state;
        if (leader) {
          int dummy;
          int32_t lc = count_in_regs<MAXT>(lt, nlead, pres, lcap, &dummy);
          if (lc > 0) {
            ls = 1;
#pragma unroll
            for (int i = 0; i < MAXT; i++) wcap[i] = int64_t(uint64_t(wcap[i]) - uint64_t(sh_wlead[e][i]));
            swl = count_in_regs<MAXT>(wt, nreq, pres | uint32_t(uni(int32_t(ev.lead_mask))), wcap, &dummy);
          }
        }
      }
    }
    if (valid) {
      int32_t* base = ctr_base(b, e0 + e);  // the class's row: its fill position
      const int64_t SD = s.SD;
      int32_t ss = 0, sswl = 0;
      if (s.L - 1 == ev.slice_level) {
        ss = go_div32(state, ev.slice_size);
        sswl = go_div32(swl, ev.slice_size);
      }
      base[gleaf] = state;
      if (b.fill_pos[e0 + e].p.ss_alias == 0) base[SD + gleaf] = ss;
      if (leader) {
        base[2 * SD + gleaf] = swl;
        base[3 * SD + gleaf] = sswl;
        base[4 * SD + gleaf] = ls;
      }
    }
    // ExclusionStats (:1579-1634), aggregated per wave before the atomics.
    uint64_t selm = ballot(kind == EX_SELECTOR);
    if (lane == 0 && selm) atomicAdd(&b.sel_counts[eid], __popcll(selm));
    const uint64_t affm = ballot(kind == EX_AFFINITY);
    if (lane == 0 && affm) atomicAdd(&b.aff_counts[eid], __popcll(affm));
    const uint64_t domm = ballot(kind == EX_TOPOLOGY);
    if (lane == 0 && domm) atomicAdd(&b.dom_counts[eid], __popcll(domm));
    uint64_t tm = ballot(kind == EX_TAINT);
    while (tm) {
      int src = __ffsll((unsigned long long)tm) - 1;
      int tid = bcast(id, src);
      uint64_t mm = ballot(kind == EX_TAINT && id == tid);
      if (lane == 0) atomicAdd(&b.taint_counts[int64_t(eid) * b.num_taints + tid], __popcll(mm));
      tm &= ~mm;
    }
    uint64_t rm = ballot(kind == EX_RESOURCE);
    while (rm) {
      int src = __ffsll((unsigned long long)rm) - 1;
      int rid = bcast(id, src);
      uint64_t mm = ballot(kind == EX_RESOURCE && id == rid);
      if (lane == 0) atomicAdd(&b.res_counts[int64_t(eid) * s.R + rid], __popcll(mm));
      rm &= ~mm;
    }
  }
}






// Staged variant (the batch requests at most NS distinct resource columns):
// every thread loads its leaf's free/used words of those columns ONCE into
// registers (static slots, ascending column order).  A block handles one
// fill chunk: up to kEvalsPerBlock phase-1 classes with the same request
// signature (worker/leader terms, overlay, simulateEmpty; the host groups
// them), so CountInWithLimitingResource runs once per leaf and only the
// per-eval masks (taints, nodeSelector) and slice parameters differ.
// Semantics identical to fill_leaves_kernel.
constexpr int kStagedLabels = 4;     // label columns held in registers (more: read from global)

// ExclusionStats of a fill block are counted in LDS and written as per-block
// partials (DevBatch::fill_stats), summed by fill_stats_reduce_kernel: no
// global atomics on a handful of hot addresses from every wave of the grid
// (device-scope atomics from all XCDs serialize at the memory side).
constexpr int kMaxFillStats = 64;  // kStatFixed + taints + resource columns; more: global atomics

// TS: the batch's taint-profile rows fit LDS (b.num_profiles <= kStagedProfiles).
// A template parameter, not a runtime select: a select between the LDS row and
// the global table compiles to a flat load whose vmcnt wait also drains every
// store the loop issued before it.
// MR: the launch's chunks hold several signature runs (CountIn per run inside
// the eval loop); otherwise one run per chunk, counted before the loop (fewer
// live registers: higher occupancy).  chunk_base: first chunk of the launch.
// GL: some eval of the launch needs global lookups in the eval loop (a
// nodeSelector column beyond the staged ones, required node affinity).
// Without it the loop holds no global load at all: on gfx9 vmcnt counts
// stores too, so a load's wait inside the loop would drain every store of
// the earlier evals.
// The five-column variants without global lookups fit 96 VGPRs without
// spilling when asked to: 5 waves per SIMD instead of 4 (C3J's multi-run fill).
#ifndef KTAS_WAVES_PER_EU  // (tests/emu's CPU build defines it empty)
#define KTAS_WAVES_PER_EU(n) __attribute__((amdgpu_waves_per_eu(n)))
#endif
template <int NS, bool TS, bool MR, bool GL>
__global__ __launch_bounds__(kFillThreads) KTAS_WAVES_PER_EU(NS == 5 && !GL ? 5 : 1) void fill_leaves_staged_kernel(DevSnap s, DevBatch b, uint32_t stage_mask,
                                                                          int chunk_base) {
  __shared__ FillEvalParams sh_p[kEvalsPerBlock];
  __shared__ DevTerm sh_term[kEvalsPerBlock][2 * NS];  // a run's worker | leader terms (at its first position)
  __shared__ int32_t sh_taint[kEvalsPerBlock][kStagedProfiles];
  __shared__ int32_t sh_stats[kEvalsPerBlock][kMaxFillStats];
  const bool split = b.stats_split != 0;  // ExclusionStats counted by fill_exclusion_kernel
  const bool lds_stats = !split && b.nstat > 0;
  if (lds_stats)
    for (int i = threadIdx.x; i < kEvalsPerBlock * kMaxFillStats; i += kFillThreads) (&sh_stats[0][0])[i] = 0;
  // XCD-aware (tile, chunk) order: consecutive workgroups go round-robin to
  // the 8 XCDs, so the chunks of one leaf tile are laid out 8 workgroups apart
  // and land on the same XCD back to back, where the tile's snapshot columns
  // are still in that XCD's L2 (each chunk re-reads them).  A bijection of
  // the 2-D grid; identity when the tile count is not a multiple of 8.
  int tgroup = blockIdx.x, chunk = blockIdx.y;
  if ((gridDim.x & 7u) == 0 && gridDim.y > 1) {
    const uint32_t lin = blockIdx.y * gridDim.x + blockIdx.x;
    const uint32_t g = lin >> 3;
    chunk = int(g % gridDim.y);
    tgroup = int((g / gridDim.y) * 8u + (lin & 7u));
  }
  chunk += chunk_base;
  const int e0 = b.fill_chunks[2 * chunk];
  const int ne = b.fill_chunks[2 * chunk + 1];
  constexpr bool stage_taints = TS;
  if (int(threadIdx.x) < ne) {
    const int eid = b.fill_ids[e0 + threadIdx.x];
    const DevEval& ev = b.evals[eid];
    FillEvalParams& P = sh_p[threadIdx.x];
    P.eid = eid;
    P.taint_off = ev.taint_table;
    P.nsel = ev.nsel;
    P.slice_size = ev.slice_size;
    P.slice_level = ev.slice_level;
    P.inner = ev.ssal[s.L - 1];
    const bool aff = (ev.flags & KUEUE_TAS_F_AFFINITY) != 0;
    P.aff_begin = aff ? ev.aff_begin : -1;
    P.aff_end = aff ? ev.aff_end : -1;
    P.dom_begin = ev.dom_begin;
    P.dom_end = ev.dom_end;
    P.sel_far = 0;
    for (int k = 0; k < KUEUE_TAS_MAX_SELECTORS; k++) {
      P.sel_col[k] = ev.sel_col[k];
      P.sel_val[k] = ev.sel_val[k];
      if (k < ev.nsel && ev.sel_col[k] >= kStagedLabels) P.sel_far = 1;
    }
    P.sx_begin = ev.sx_begin;
    P.sx_end = ev.sx_end;
    if (ev.sx_begin >= 0) P.sel_far = 1;  // the requirements are read from global memory (GL launch)
    P.run = b.fill_run[e0 + threadIdx.x];
    P.sig_new = threadIdx.x == 0 || b.fill_run[e0 + threadIdx.x - 1] != P.run;
    P.rmask = int32_t(ev.req_mask);
    P.lmask = int32_t(ev.lead_mask);
  }
  __syncthreads();
  if (s.taint_profile && stage_taints) {
    for (int i = threadIdx.x; i < ne * kStagedProfiles; i += kFillThreads) {
      const int e = i / kStagedProfiles, p = i % kStagedProfiles;
      sh_taint[e][p] = p < b.num_profiles ? b.taint_table[sh_p[e].taint_off + p] : -1;
    }
  }
  for (int i = threadIdx.x; i < ne * 2 * NS; i += kFillThreads) {
    const int e = i / (2 * NS), j = i % (2 * NS);
    if (!sh_p[e].sig_new) continue;
    const DevEval& ev = b.evals[sh_p[e].eid];
    if (j < NS && j < ev.nreq) sh_term[e][j] = b.terms[ev.term_begin + j];
    if (j >= NS && j - NS < ev.nlead) sh_term[e][j] = b.terms[ev.lead_begin + (j - NS)];
  }
  __syncthreads();
  // kFillTilesPerBlock consecutive leaf tiles per block: the setup above
  // (chunk parameters, terms, taint rows: dependent global loads) is paid
  // once per block, and the grid fits one residency round
  // ragged parents (rack_fanout < 0): a tile is 4 wave slots of whole parents
  const bool packed = b.rack_fanout < 0;
  const int ntiles = packed ? (s.n_wave_slots + 3) / 4 : (s.N + kFillThreads - 1) / kFillThreads;
  for (int tile = tgroup * kFillTilesPerBlock; tile < min(ntiles, (tgroup + 1) * kFillTilesPerBlock); tile++) {
  const int lane = lane_id();
  int leaf;
  bool valid;
  if (packed) {
    const int slot = tile * 4 + int(threadIdx.x >> 6);
    const int2 wt = slot < s.n_wave_slots ? s.wave_tab[slot] : make_int2(0, 0);
    leaf = wt.x + lane;
    valid = lane < wt.y;
  } else {
    leaf = tile * kFillThreads + int(threadIdx.x);
    valid = leaf < s.N;
  }
  const int N = s.N;
  const int gleaf = s.level_off[s.L - 1] + leaf;
  // ragged parents: this lane's parent, its segment's first lane, and
  // whether it is the segment's last lane (which writes the parent)
  int rparent = -1, seg0 = 0;
  bool seg_tail = false;
  if (packed) {
    rparent = valid ? s.leaf_parent[leaf] : -1;
    const int prevp = __shfl(rparent, lane > 0 ? lane - 1 : 0);
    const uint64_t H = ballot(valid && (lane == 0 || prevp != rparent));
    const uint64_t V = ballot(valid);
    const uint64_t upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1ull);
    seg0 = 63 - __builtin_clzll((H & upto) | 1ull);
    seg_tail = valid && (lane == kWave - 1 || ((H >> (lane + 1)) & 1ull) || !((V >> (lane + 1)) & 1ull));
  }
  int scol[NS];
  int64_t fr[NS], us[NS];
  {
    uint32_t m = stage_mask;
#pragma unroll
    for (int k = 0; k < NS; k++) {
      scol[k] = m ? __builtin_ctz(m) : -1;
      if (m) m &= m - 1;
      fr[k] = 0;
      us[k] = 0;
      if (valid && scol[k] >= 0) {
        fr[k] = s.free_cap[int64_t(scol[k]) * N + leaf];
        us[k] = s.tas_usage[int64_t(scol[k]) * N + leaf];
      }
    }
  }
  const uint32_t fp = valid ? s.free_present[leaf] : 0u;
  const uint32_t up = valid ? s.usage_present[leaf] : 0u;
  const int prof = (valid && s.taint_profile) ? s.taint_profile[leaf] : 0;
  int32_t lab[kStagedLabels];
#pragma unroll
  for (int k = 0; k < kStagedLabels; k++) lab[k] = (valid && s.label_values && k < s.K) ? s.label_values[int64_t(k) * N + leaf] : 0;
  static_assert(kStagedLabels == 4, "staged_label takes four staged columns");
  const int32_t lab0 = lab[0], lab1 = lab[1], lab2 = lab[2], lab3 = lab[3];
  auto label_at = [s, leaf, lab0, lab1, lab2, lab3](int col) {  // by value: nothing escapes to scratch
    return staged_label(s, leaf, col, lab0, lab1, lab2, lab3);
  };

  // ---- the chunk's base signature (leader / simulateEmpty, assumed usage):
  // the leaf's remaining capacity, once per leaf ----
  bool leader, live;
  uint32_t pres = 0;
  int64_t cap[NS];
  {
    const DevEval& ev = b.evals[uni(b.fill_ids[e0])];
    const uint32_t flags = uint32_t(uni(int32_t(ev.flags)));
    const int abeg = uni(ev.assumed_begin), aend = uni(ev.assumed_end);
    leader = (flags & KUEUE_TAS_F_LEADER) != 0;
    const bool sim = (flags & KUEUE_TAS_F_SIMULATE_EMPTY) != 0;
    live = valid && !leaf_out(s, leaf);
    pres = fp | (sim ? 0u : up);
    int a_lo = 0, a_hi = 0;
    if (live && aend > abeg) {
      int lo = abeg, hi = aend;
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (b.assumed[mid].leaf < leaf) lo = mid + 1;
        else hi = mid;
      }
      a_lo = lo;
      a_hi = lo;
      while (a_hi < aend && b.assumed[a_hi].leaf == leaf) {
        pres |= 1u << b.assumed[a_hi].col;
        a_hi++;
      }
    }
#pragma unroll
    for (int k = 0; k < NS; k++) {
      int64_t c = sim ? fr[k] : int64_t(uint64_t(fr[k]) - uint64_t(us[k]));
      for (int a = a_lo; a < a_hi; a++)
        if (b.assumed[a].col == scol[k]) c = int64_t(uint64_t(c) - uint64_t(b.assumed[a].value));
      cap[k] = c;
    }
  }
  // CountInWithLimitingResource over a run's terms (LDS), ascending column order
  auto count_slots = [&](const DevTerm* terms, uint32_t mask, const DevTerm* lterms, uint32_t lmask, uint32_t presm,
                         bool sub_leader, int* lim_out) -> int32_t {
    return count_slots_sel<NS>(scol, cap, terms, mask, lterms, lmask, presm, sub_leader, lim_out);
  };
  int32_t state0 = 0, swl0 = 0, ls0 = 0;
  int lim0 = -1;
  auto count_run = [&](int e) {  // CountIn of the run starting at chunk position e
    state0 = swl0 = ls0 = 0;
    lim0 = -1;
    const FillEvalParams& P = sh_p[e];
    if (live) {
      const uint32_t rmask = uint32_t(uni(P.rmask)), lmask = uint32_t(uni(P.lmask));
      const DevTerm* wt = sh_term[e];
      const DevTerm* lt = sh_term[e] + NS;
      state0 = count_slots(wt, rmask, lt, lmask, pres, false, &lim0);
      if (split) b.fill_lim[int64_t(uni(P.run)) * N + leaf] = int8_t(state0 == 0 ? lim0 : -1);
      swl0 = state0;
      if (leader) {
        int dummy;
        int32_t lc = count_slots(lt, lmask, lt, lmask, pres, false, &dummy);
        if (lc > 0) {
          ls0 = 1;
          swl0 = count_slots(wt, rmask, lt, lmask, pres | lmask, true, &dummy);
        }
      }
    } else if (split && valid) {
      b.fill_lim[int64_t(uni(P.run)) * N + leaf] = int8_t(-1);
    }
  };
  if constexpr (!MR) count_run(0);

  // loads the per-eval loop needs, hoisted: a global load inside the loop
  // waits (vmcnt) for every store of the earlier evals
  const bool dead = valid && !live;
  const int rack_f = b.rack_fanout;
  for (int e = 0; e < ne; e++) {
    const int4* pq = reinterpret_cast<const int4*>(&sh_p[e]);
    const int4 q0 = pq[0], q1 = pq[1], q2 = pq[2];
    if constexpr (MR) {
      if (uni(q2.w)) count_run(e);  // sig_new: a new signature run, CountIn once per leaf for the run
    }
    const int eid = uni(q0.x);
    const int nsel = uni(q0.y);
    const int32_t slice_size = uni(q0.z), slice_level = uni(q0.w);
    const int32_t p_inner = uni(q1.x), sel_far = uni(q1.y), aff_begin = uni(q1.z), aff_end = uni(q1.w);
    const int32_t dom_begin = uni(q2.x), dom_end = uni(q2.y);
    int32_t state = 0, swl = 0, ls = 0;
    int kind = dead ? EX_DEAD : EX_NONE, id = -1;
    if (valid && kind == EX_NONE) {
      if (s.lowest_is_hostname) {
        if (s.taint_profile) {
          int t;
          if constexpr (TS) t = sh_taint[e][prof];
          else t = b.taint_table[uni(q2.z) + prof];
          if (t >= 0) {
            kind = EX_TAINT;
            id = t;
          }
        }
        if (kind == EX_NONE && nsel > 0) {
          // two loops: with every column in registers the loop holds no global
          // load, so no vmcnt wait (which would also drain the earlier stores)
          const int4 c0 = pq[4], c1 = pq[5], v0 = pq[6], v1 = pq[7];  // sel_col[8], sel_val[8]
          const int32_t scol[KUEUE_TAS_MAX_SELECTORS] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
          const int32_t sval[KUEUE_TAS_MAX_SELECTORS] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
          if (!GL || !sel_far) {
#pragma unroll
            for (int k = 0; k < KUEUE_TAS_MAX_SELECTORS; k++) {
              if (k < nsel && kind == EX_NONE) {
                const int col = uni(scol[k]);
                int32_t v = lab[0];
#pragma unroll
                for (int q = 1; q < kStagedLabels; q++) v = col == q ? lab[q] : v;
                if (v != uni(sval[k])) kind = EX_SELECTOR;
              }
            }
          } else {
#pragma unroll
            for (int k = 0; k < KUEUE_TAS_MAX_SELECTORS; k++)
              if (k < nsel && kind == EX_NONE && label_at(uni(scol[k])) != uni(sval[k])) kind = EX_SELECTOR;
            if constexpr (GL) {
              const int32_t sxb = uni(pq[3].w);  // (the host fills the inline pairs first: nsel == 8)
              if (kind == EX_NONE && sxb >= 0 && !selector_ext_match(b, sxb, uni(pq[8].x), leaf, label_at))
                kind = EX_SELECTOR;
            }
          }
        }
        if constexpr (GL) {
          if (kind == EX_NONE && aff_begin >= 0 && !affinity_match(b, aff_begin, aff_end, leaf, label_at)) kind = EX_AFFINITY;
        }
      }
      if (kind == EX_NONE && outside_domain(dom_begin, dom_end, leaf)) kind = EX_TOPOLOGY;
      if (kind == EX_NONE) {
        state = state0;
        swl = swl0;
        ls = ls0;
        if (state == 0 && lim0 >= 0) {
          kind = EX_RESOURCE;
          id = lim0;
        }
      }
    }
    int32_t ss = 0, sswl = 0;
    if (s.L - 1 == slice_level) {
      if (slice_size == 1) {  // wave-uniform: no integer division
        ss = state;
        sswl = swl;
      } else {
        ss = go_div32(state, slice_size);
        sswl = leader ? go_div32(swl, slice_size) : ss;
      }
    }
    int32_t* base = ctr_base(b, e0 + e);  // the class's row: its fill position
    const int64_t SD = s.SD;
    if (valid) {
      base[gleaf] = state;
      if (b.fill_pos[e0 + e].p.ss_alias == 0) base[SD + gleaf] = ss;
      if (leader) {
        base[2 * SD + gleaf] = swl;
        base[3 * SD + gleaf] = sswl;
        base[4 * SD + gleaf] = ls;
      }
    }
    // fused fillInCountsHelper (:1658-1719) of the leaves' parents: uniform
    // power-of-two fan-out F <= 64, parent p owns leaves [p*F, (p+1)*F), so
    // a parent's children are F aligned lanes of one wave (butterfly
    // reductions).  F = 32 / 64 compile-time: no per-step fan-out tests.
    auto rack_rollup = [&](auto FC) {
      const int F = decltype(FC)::value > 0 ? int(decltype(FC)::value) : b.rack_fanout;
      const int32_t inner = p_inner;
      int32_t cs = state, csw = swl;
      if (inner != 0 && inner != 1) {  // wave-uniform; x / 1 * 1 == x
        cs = w_mul(go_div32(cs, inner), inner);
        csw = w_mul(go_div32(csw, inner), inner);
      }
      int32_t cap = cs, slc = ss, lead = ls, minD = 0x7fffffff, minSD = 0x7fffffff;
      int has = 0;
      if (!leader || ls > 0) {
        has = 1;
        minD = w_sub(cs, csw);
        minSD = w_sub(ss, sswl);
      }
      cap = group_reduce(cap, F, OpWAdd());
      if (s.L - 1 != slice_level) {  // wave-uniform: the leaves' sliceState is 0
      } else if (inner == 1 && slice_size == 1) {  // wave-uniform: sliceState == state
        slc = cap;
      } else {
        slc = group_reduce(slc, F, OpWAdd());
      }
      if (leader) {  // leader fields only matter for leader evals (parents of others keep state, sliceState)
        minD = group_reduce(minD, F, OpMin());
        minSD = group_reduce(minSD, F, OpMin());
        lead = group_reduce(lead, F, OpMax());
        has = group_reduce(has, F, OpMax());
      }
      const int parent = leaf / F;
      const uint64_t posm = ballot(valid && ss > 0);  // positive children, for the BestFit descent
      if ((lane & (F - 1)) == 0 && parent < s.level_size[s.L - 2]) {
        const uint64_t seg = F == kWave ? posm : (posm >> lane) & ((1ull << (F & 63)) - 1ull);
        b.rack_pos[int64_t(e0 + e) * s.level_size[s.L - 2] + parent] = seg;
        const int32_t pswl = has ? w_sub(cap, minD) : 0;
        int32_t psswl = has ? w_sub(slc, minSD) : 0;
        if (s.L - 2 == slice_level) {
          slc = go_div32(cap, slice_size);
          psswl = go_div32(pswl, slice_size);
        }
        const int g = s.level_off[s.L - 2] + parent;
        base[g] = cap;
        if (b.fill_pos[e0 + e].p.ss_alias == 0) base[SD + g] = slc;
        if (leader) {
          base[2 * SD + g] = pswl;
          base[3 * SD + g] = psswl;
          base[4 * SD + g] = lead;
        }
      }
    };
    // the same over ragged parents: segmented scans, the segment's last lane writes
    auto ragged_rollup = [&]() {
      const int32_t inner = p_inner;
      int32_t cs = state, csw = swl;
      if (inner != 0 && inner != 1) {
        cs = w_mul(go_div32(cs, inner), inner);
        csw = w_mul(go_div32(csw, inner), inner);
      }
      int32_t cap = cs, slc = ss, lead = ls, minD = 0x7fffffff, minSD = 0x7fffffff;
      int has = 0;
      if (!leader || ls > 0) {
        has = 1;
        minD = w_sub(cs, csw);
        minSD = w_sub(ss, sswl);
      }
      cap = seg_incl_scan(cap, lane, seg0, OpWAdd());
      if (s.L - 1 != slice_level) {
      } else if (inner == 1 && slice_size == 1) {
        slc = cap;
      } else {
        slc = seg_incl_scan(slc, lane, seg0, OpWAdd());
      }
      if (leader) {
        minD = seg_incl_scan(minD, lane, seg0, OpMin());
        minSD = seg_incl_scan(minSD, lane, seg0, OpMin());
        lead = seg_incl_scan(lead, lane, seg0, OpMax());
        has = seg_incl_scan(has, lane, seg0, OpMax());
      }
      const uint64_t posm = ballot(valid && ss > 0);
      if (seg_tail) {
        const int len = lane - seg0 + 1;
        const uint64_t seg = len == kWave ? posm : (posm >> seg0) & ((1ull << len) - 1ull);
        b.rack_pos[int64_t(e0 + e) * s.level_size[s.L - 2] + rparent] = seg;
        const int32_t pswl = has ? w_sub(cap, minD) : 0;
        int32_t psswl = has ? w_sub(slc, minSD) : 0;
        if (s.L - 2 == slice_level) {
          slc = go_div32(cap, slice_size);
          psswl = go_div32(pswl, slice_size);
        }
        const int g = s.level_off[s.L - 2] + rparent;
        base[g] = cap;
        if (b.fill_pos[e0 + e].p.ss_alias == 0) base[SD + g] = slc;
        if (leader) {
          base[2 * SD + g] = pswl;
          base[3 * SD + g] = psswl;
          base[4 * SD + g] = lead;
        }
      }
    };
    if (rack_f < 0) ragged_rollup();
    else if (rack_f == 32) rack_rollup(std::integral_constant<int, 32>());
    else if (rack_f == 64) rack_rollup(std::integral_constant<int, 64>());
    else if (rack_f) rack_rollup(std::integral_constant<int, 0>());
    if (split) continue;
    // wave-uniform skips: a wave with every leaf counted nowhere, and the
    // kinds this eval cannot produce (no selector / affinity / domain)
    if (ballot(valid && kind != EX_NONE && kind != EX_DEAD) == 0) continue;
    if (nsel > 0) {
      const uint64_t selm = ballot(kind == EX_SELECTOR);
      if (lane == 0 && selm) {
        if (lds_stats) atomicAdd(&sh_stats[e][0], __popcll(selm));
        else atomicAdd(&b.sel_counts[eid], __popcll(selm));
      }
    }
    if (aff_begin >= 0) {
      const uint64_t affm = ballot(kind == EX_AFFINITY);
      if (lane == 0 && affm) {
        if (lds_stats) atomicAdd(&sh_stats[e][1], __popcll(affm));
        else atomicAdd(&b.aff_counts[eid], __popcll(affm));
      }
    }
    if (dom_begin >= 0) {
      const uint64_t domm = ballot(kind == EX_TOPOLOGY);
      if (lane == 0 && domm) {
        if (lds_stats) atomicAdd(&sh_stats[e][2], __popcll(domm));
        else atomicAdd(&b.dom_counts[eid], __popcll(domm));
      }
    }
    uint64_t tm = ballot(kind == EX_TAINT);
    while (tm) {
      int src = __ffsll((unsigned long long)tm) - 1;
      int tid = bcast(id, src);
      uint64_t mm = ballot(kind == EX_TAINT && id == tid);
      if (lane == 0) {
        if (lds_stats) atomicAdd(&sh_stats[e][kStatFixed + tid], __popcll(mm));
        else atomicAdd(&b.taint_counts[int64_t(eid) * b.num_taints + tid], __popcll(mm));
      }
      tm &= ~mm;
    }
    uint64_t rm = ballot(kind == EX_RESOURCE);
    while (rm) {
      int src = __ffsll((unsigned long long)rm) - 1;
      int rid = bcast(id, src);
      uint64_t mm = ballot(kind == EX_RESOURCE && id == rid);
      if (lane == 0) {
        if (lds_stats) atomicAdd(&sh_stats[e][kStatFixed + b.num_taints + rid], __popcll(mm));
        else atomicAdd(&b.res_counts[int64_t(eid) * s.R + rid], __popcll(mm));
      }
      rm &= ~mm;
    }
  }
  }  // tiles
  if (lds_stats) {  // per-block partials [fill position][block][stat]
    __syncthreads();
    for (int i = threadIdx.x; i < ne * b.nstat; i += kFillThreads) {
      const int e = i / b.nstat, k = i % b.nstat;
      b.fill_stats[(int64_t(e0 + e) * b.nstat_blocks + tgroup) * b.nstat + k] = sh_stats[e][k];
    }
  }
}

// ---- the staged fill with kPairLP adjacent leaves per thread ----
// Same semantics as fill_leaves_staged_kernel<NS, TS, MR, GL> on a snapshot
// whose leaf parents are uniform power-of-two fan-out F >= kPairLP (or not
// rolled up, F = 0), with the ExclusionStats counted in the loop.  A thread
// holds leaves kPairLP*t .. kPairLP*t + kPairLP - 1 of a kPairTile-leaf tile,
// so every per-class cost that does not depend on the leaf — the parameter
// reads, the wave-uniform branches (scalar instructions: the CU's one scalar
// unit is this kernel's tightest issue port), the counter row addresses, a
// ballot, a butterfly step — is paid once per 64 * kPairLP leaves instead of
// 64: the parent sums start with the in-lane group and take log2(kPairLP)
// butterfly steps fewer, the counter words go out as one wide store, the
// ExclusionStats ballots cover kPairLP leaves each.  Two leaves measured
// faster than four on C3 (84 us vs 117 us per launch, profiles/r03_lp4): at
// four the register footprint halves the waves per SIMD and the grid (128
// tiles x classes / 8) leaves too few waves to hide the column loads.
constexpr int kPairLP = 2;                     // leaves per thread (adjacent)
constexpr int kCatSlots = 2 * 64;              // leaf-category table of a fill_pair_kernel block (CAT)
constexpr int kPairTile = kPairLP * kFillThreads;  // leaves per block

// Profiling build: fill_pair_kernel's block phase stamps (DevBatch::fill_prof)
#ifndef KTAS_PROFILE
#define KTAS_PROFILE 0
#endif
#define KTAS_FILL_STAMP(k)                                                                       \
  do {                                                                                          \
    if (KTAS_PROFILE && b.fill_prof && threadIdx.x == 0) {                                      \
      const uint32_t blk = blockIdx.y * gridDim.x + blockIdx.x;                                 \
      if (blk < (1u << 15)) b.fill_prof[blk * 8 + (k)] = int32_t(uint32_t(wall_clock64()));       \
    }                                                                                           \
  } while (0)

// The fast-LFC chunk tables from the fill (DevBatch::lfc_fill; what
// lfc_hist_kernel computes from the written rows): a slot class's leaf values
// as counts per (slot, 2048-leaf chunk, value bin), the overflow bin's value
// sum, and the byte copy of the values for lfc_emit_kernel.  Generic per-wave
// form (any leaf layout, one ballot round per distinct value): the fill's
// non-lean blocks.  The tables start at zero (lfc_total's stream zeroes them
// after the batch's emit).
__device__ void lfc_fill_accum(const DevBatch& b, int slot, const int32_t* vals, const int* leaves, const bool* act,
                               int n) {
  const int lane = lane_id();
  for (int j = 0; j < n; j++) {
    uint64_t pending = ballot(act[j]);
    const int32_t x = act[j] ? vals[j] : 0;
    const int bin = x >= kLfcBins - 1 ? kLfcBins - 1 : (x < 0 ? 0 : x);
    const int ch = leaves[j] / kLfcChunk;
    if (act[j]) {
      b.lfc_u8[int64_t(slot) * b.lfc_nchunks * kLfcChunk + leaves[j]] = uint8_t(x < 0 ? 0 : x > 255 ? 255 : x);
    }
    while (pending) {
      const int src = __ffsll((unsigned long long)pending) - 1;
      const int key = bcast(ch * kLfcBins + bin, src);
      const uint64_t m = ballot(act[j] && ch * kLfcBins + bin == key);
      if (lane == src) atomicAdd(&b.lfc_ch[int64_t(slot) * b.lfc_nchunks * kLfcBins + key], uint32_t(__popcll(m)));
      pending &= ~m;
    }
    // the overflow sums per chunk: a wave's leaves span at most two chunks
    uint64_t om = ballot(act[j] && x >= kLfcBins - 1);
    while (om) {
      const int src = __ffsll((unsigned long long)om) - 1;
      const int c0 = bcast(ch, src);
      const uint64_t m = ballot(act[j] && x >= kLfcBins - 1 && ch == c0);
      unsigned long long v = (act[j] && x >= kLfcBins - 1 && ch == c0) ? (unsigned long long)int64_t(x) : 0ull;
      v = (unsigned long long)wave_sum_i64(int64_t(v));
      if (lane == src) atomicAdd(reinterpret_cast<unsigned long long*>(&b.lfc_ovs[int64_t(slot) * b.lfc_nchunks + c0]), v);
      om &= ~m;
    }
  }
}

// Or-fold: the positive-children masks
struct OpOr {
  __device__ int32_t operator()(int32_t a, int32_t b) const { return a | b; }
};

// MR: chunks of several signature runs (CountIn again at each run's first
// position, the leaves' remaining capacity kept in registers), as the
// staged kernel's MR.
// CAT: leaf categories (below); single-run chunks only (!MR), every filter on
// staged data (!GL), taint rows in LDS (TS), ExclusionStats in LDS.
// FC: 32 compile-time fan-out, 0: b.rack_fanout.  LF: the lean loop may
// accumulate the fast-LFC tables (DevBatch::lfc_fill); its per-wave pair
// lists cost 4 KB of LDS, which without LF lets 8 blocks share a CU
template <int NS, bool TS, bool MR, bool GL, int FC, bool CAT = false, bool LF = false>
                                                      // (or none), -1: ragged parents in 128-leaf slots (DevSnap::wave_tab2)
// (75-79 VGPRs: 6 waves per SIMD.  Forcing 8 — the whole C3 grid resident —
// spilled ~20 prologue values: 37.8 -> 36.4 us but 61 -> 113 MB of HBM
// traffic per launch, profiles/r05/waves8 and final2/pmc_summary.json)
__global__ __launch_bounds__(kFillThreads) void fill_pair_kernel(DevSnap s, DevBatch b, uint32_t stage_mask,
                                                                 int chunk_base) {
  static_assert(!CAT || (!MR && !GL && TS), "leaf categories: single-run chunks, staged filters, LDS taint rows");
  __shared__ FillPos sh_pos[kEvalsPerBlock];  // the chunk's host-built position records
  __shared__ int32_t sh_stats[kEvalsPerBlock][kMaxFillStats];
  // multi-run chunks: each leaf's remaining capacity waits in LDS for the
  // next run's CountIn ([column][leaf of the lane][thread]), not in 4 * NS
  // VGPRs live across the whole class loop
  __shared__ int64_t sh_cap[MR ? NS * kPairLP * kFillThreads : 1];
  // CAT: the block's leaf-category table (key | 1 << 63, 0: empty), leaf
  // counts per category, the overflow flag, each class's pass mask
  __shared__ unsigned long long sh_ckey[CAT ? kCatSlots : 1];
  __shared__ int32_t sh_ccnt[CAT ? kCatSlots : 1];
  __shared__ int32_t sh_cflag;
  __shared__ uint64_t sh_passd[CAT ? 2 * kEvalsPerBlock : 1];  // pass masks over dense category ids (two words)
  __shared__ unsigned long long sh_dkey[CAT ? kCatSlots : 1];  // the categories' keys by dense id
  __shared__ int32_t sh_dcnt[CAT ? kCatSlots : 1];             // and their leaf counts
  // lean blocks with fast-LFC slot classes (DevBatch::lfc_fill): the distinct
  // (dense category, state0 > 0) pairs of each wave's leaves and their counts
  constexpr int kTri = 2 * kWave;  // at most one pair per leaf of the wave
  __shared__ int32_t sh_tv[CAT && LF ? 4 * kTri : 1];
  __shared__ int32_t sh_tc[CAT && LF ? 4 * kTri : 1];  // count << 8 | dense category
  __shared__ int32_t sh_tn[CAT && LF ? 4 : 1];
  static_assert(2 * NS <= kPosTerms, "a position holds 2 * NS terms");
  const bool lds_stats = b.nstat > 0;
  KTAS_FILL_STAMP(0);
  if (lds_stats)
    for (int i = threadIdx.x; i < kEvalsPerBlock * kMaxFillStats; i += kFillThreads) (&sh_stats[0][0])[i] = 0;
  if constexpr (CAT) {
    for (int i = threadIdx.x; i < kCatSlots; i += kFillThreads) {
      sh_ckey[i] = 0ull;
      sh_ccnt[i] = 0;
    }
    if (threadIdx.x == 0) sh_cflag = 0;
  }
  int tile = blockIdx.x, chunk = blockIdx.y;  // XCD-aware (tile, chunk) order as in the staged kernel
  if ((gridDim.x & 7u) == 0 && gridDim.y > 1) {
    const uint32_t lin = blockIdx.y * gridDim.x + blockIdx.x;
    const uint32_t g = lin >> 3;
    chunk = int(g % gridDim.y);
    tile = int((g / gridDim.y) * 8u + (lin & 7u));
  }
  // the leaves' snapshot columns first (they do not depend on the chunk),
  // then the chunk's records: both sets of loads in flight together
  const int lane = lane_id();
  const int N = s.N;
  int leaf0 = tile * kPairTile + kPairLP * int(threadIdx.x);
  int slot_len = N - tile * kPairTile;  // leaves of this lane's window from the window's first
  bool wide_slot = false;               // FC < 0: the slot is a 128-leaf piece of a wider parent
  if constexpr (FC < 0) {  // this wave's 128-leaf slot of whole parents
    const int slot = tile * 4 + int(threadIdx.x >> 6);
    const int2 wt = slot < s.n_wave_slots2 ? s.wave_tab2[slot] : make_int2(0, 0);
    leaf0 = wt.x + kPairLP * lane;
    slot_len = wt.y & 0xffff;
    wide_slot = (wt.y >> 16) != 0;
  }
  const int gleaf0 = s.level_off[s.L - 1] + leaf0;
  bool valid[kPairLP];
  int scol[NS];
  int64_t cap[kPairLP][NS], used[kPairLP][NS];
  uint32_t fp[kPairLP], up[kPairLP];
  int prof[kPairLP];
  int32_t lab[kPairLP][kStagedLabels];
#pragma unroll
  for (int j = 0; j < kPairLP; j++) {
    const int leaf = leaf0 + j;
    if constexpr (FC < 0) valid[j] = kPairLP * lane + j < slot_len;
    else valid[j] = leaf < N;
    fp[j] = valid[j] ? s.free_present[leaf] : 0u;
    up[j] = valid[j] ? s.usage_present[leaf] : 0u;
    prof[j] = (valid[j] && s.taint_profile) ? s.taint_profile[leaf] : 0;
#pragma unroll
    for (int k = 0; k < kStagedLabels; k++)
      lab[j][k] = (valid[j] && s.label_values && k < s.K) ? s.label_values[int64_t(k) * N + leaf] : 0;
  }
  uint32_t pk_lo[kPairLP], pk_hi[kPairLP];  // the staged label ids as one 64-bit key (FillEvalParams::sel_fast)
#pragma unroll
  for (int j = 0; j < kPairLP; j++) {
    pk_lo[j] = (uint32_t(lab[j][0]) & 0xffffu) | (uint32_t(lab[j][1]) << 16);
    pk_hi[j] = (uint32_t(lab[j][2]) & 0xffffu) | (uint32_t(lab[j][3]) << 16);
  }
  {
    uint32_t m = stage_mask;
#pragma unroll
    for (int k = 0; k < NS; k++) {
      scol[k] = m ? __builtin_ctz(m) : -1;
      if (m) m &= m - 1;
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        cap[j][k] = used[j][k] = 0;
        if (valid[j] && scol[k] >= 0) {
          cap[j][k] = s.free_cap[int64_t(scol[k]) * N + leaf0 + j];
          used[j][k] = s.tas_usage[int64_t(scol[k]) * N + leaf0 + j];
        }
      }
    }
  }
  chunk += chunk_base;
  const int e0 = b.fill_chunks[2 * chunk];
  const int ne = b.fill_chunks[2 * chunk + 1];
  {
    const int4* src = reinterpret_cast<const int4*>(b.fill_pos + e0);
    int4* dst = reinterpret_cast<int4*>(sh_pos);
    const int words = ne * int(sizeof(FillPos) / 16);
    for (int i = threadIdx.x; i < words; i += kFillThreads) dst[i] = src[i];
  }
  __syncthreads();
  // ---- base signature: remaining capacity per leaf ----
  bool leader, live[kPairLP];
  uint32_t pres[kPairLP];
  {
    const uint32_t flags = uint32_t(uni(sh_pos[0].p.pad[0]));
    const int abeg = uni(sh_pos[0].p.pad[1]), aend = uni(sh_pos[0].p.pad[2]);
    leader = (flags & KUEUE_TAS_F_LEADER) != 0;
    const bool sim = (flags & KUEUE_TAS_F_SIMULATE_EMPTY) != 0;
#pragma unroll
    for (int j = 0; j < kPairLP; j++) {
      const int leaf = leaf0 + j;
      live[j] = valid[j] && !leaf_out(s, leaf);
      pres[j] = fp[j] | (sim ? 0u : up[j]);
      int a_lo = 0, a_hi = 0;
      if (live[j] && aend > abeg) {
        int lo = abeg, hi = aend;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (b.assumed[mid].leaf < leaf) lo = mid + 1;
          else hi = mid;
        }
        a_lo = lo;
        a_hi = lo;
        while (a_hi < aend && b.assumed[a_hi].leaf == leaf) {
          pres[j] |= 1u << b.assumed[a_hi].col;
          a_hi++;
        }
      }
#pragma unroll
      for (int k = 0; k < NS; k++) {
        int64_t c = sim ? cap[j][k] : int64_t(uint64_t(cap[j][k]) - uint64_t(used[j][k]));
        for (int a = a_lo; a < a_hi; a++)
          if (b.assumed[a].col == scol[k]) c = int64_t(uint64_t(c) - uint64_t(b.assumed[a].value));
        cap[j][k] = c;
        if constexpr (MR) sh_cap[(k * kPairLP + j) * kFillThreads + threadIdx.x] = c;
      }
    }
  }
  // CountInWithLimitingResource over the run's terms (LDS), ascending column order
  auto count_slots = [&](const int64_t (&cp)[NS], const DevTerm* terms, uint32_t mask, const DevTerm* lterms,
                         uint32_t lmask, uint32_t presm, bool sub_leader, int* lim_out) -> int32_t {
    return count_slots_sel<NS>(scol, cp, terms, mask, lterms, lmask, presm, sub_leader, lim_out);
  };
  int32_t state0[kPairLP] = {}, swl0[kPairLP] = {}, ls0[kPairLP] = {};
  int lim0[kPairLP];
#pragma unroll
  for (int j = 0; j < kPairLP; j++) lim0[j] = -1;
  auto count_run = [&](int e) {  // CountIn of the run starting at chunk position e, both leaves
    const uint32_t rmask = uint32_t(uni(sh_pos[e].p.rmask)), lmask = uint32_t(uni(sh_pos[e].p.lmask));
    const DevTerm* wt = sh_pos[e].term;
    const DevTerm* lt = wt + NS;
#pragma unroll
    for (int j = 0; j < kPairLP; j++) {
      state0[j] = swl0[j] = ls0[j] = 0;
      lim0[j] = -1;
      if (!live[j]) continue;
      int64_t cj[NS];
#pragma unroll
      for (int k = 0; k < NS; k++) {
        if constexpr (MR) cj[k] = sh_cap[(k * kPairLP + j) * kFillThreads + threadIdx.x];
        else cj[k] = cap[j][k];
      }
      state0[j] = count_slots(cj, wt, rmask, lt, lmask, pres[j], false, &lim0[j]);
      swl0[j] = state0[j];
      if (leader) {
        int dummy;
        const int32_t lc = count_slots(cj, lt, lmask, lt, lmask, pres[j], false, &dummy);
        if (lc > 0) {
          ls0[j] = 1;
          swl0[j] = count_slots(cj, wt, rmask, lt, lmask, pres[j] | lmask, true, &dummy);
        }
      }
    }
  };
  KTAS_FILL_STAMP(1);
  if constexpr (!MR) count_run(0);
  KTAS_FILL_STAMP(2);
  // ---- CAT: leaf categories.  In a single-run chunk every filter of
  // fillInCounts (:1578-1634) sees a leaf only through its category: out of
  // the snapshot or not, taint profile, the label ids the chunk's
  // nodeSelectors test, and the run's limiting column when CountIn gives 0
  // (the resource exclusion).  The block's 512 leaves fall into few
  // categories (C3: 3 profiles x 4 gpu-type ids x a few limiting columns),
  // numbered by an LDS hash table (64-bit keys, compare-and-swap, linear
  // probing) that also counts each category's leaves.  Every class then
  // decides its verdict once per category (a lane per category, the classes
  // spread over the block's waves) and adds its ExclusionStats as one LDS
  // add per excluded category; the wave's pass mask goes to LDS.  In the
  // class loop a leaf takes its category's bit: no per-leaf classification,
  // no per-class stats ballots (the SALU / VALU issue that bounded the
  // round-4 fill).  A block whose categories overflow the table, or one of
  // whose classes filters on something else (a required domain, a selector
  // outside the packed compare), keeps the per-leaf path.
  int cslot[kPairLP], did[kPairLP];  // the leaves' table slots and dense category ids
  int ncat = 0;
  bool cat_ok = false;
  if constexpr (CAT) {
    // the chunk's selected label fields (16-bit fields of the packed key)
    uint32_t kmlo = 0u, kmhi = 0u;
    bool catable = lds_stats;  // (the host launches CAT with LDS stats only)
    for (int e = 0; e < ne; e++) {
      const FillEvalParams& P = sh_pos[e].p;
      kmlo |= uint32_t(P.sel_mlo);
      kmhi |= uint32_t(P.sel_mhi);
      catable = catable && P.dom_begin < 0 && (P.nsel == 0 || P.sel_fast != 0 || !s.lowest_is_hostname);
    }
    int fld[3] = {0, 0, 0}, nf = 0;
#pragma unroll
    for (int f = 0; f < kStagedLabels; f++) {
      const uint32_t m = ((f < 2 ? kmlo : kmhi) >> (16 * (f & 1))) & 0xffffu;
      if (m) {
        if (nf < 3) fld[nf] = f;
        nf++;
      }
    }
    cat_ok = catable && nf <= 3;  // block-uniform
    if (cat_ok) {
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        cslot[j] = -1;
        if (!valid[j]) continue;
        const int zl = (live[j] && state0[j] == 0) ? lim0[j] : -1;
        uint64_t key = (1ull << 63) | (uint64_t(uint32_t(!live[j]) | (uint32_t(prof[j]) << 1) | (uint32_t(zl + 1) << 6)) << 48);
#pragma unroll
        for (int q = 0; q < 3; q++) {
          if (q < nf) {
            const int f = fld[q];
            const uint32_t v = ((f < 2 ? pk_lo[j] : pk_hi[j]) >> (16 * (f & 1))) & 0xffffu;
            key |= uint64_t(v) << (16 * q);
          }
        }
        uint32_t h = uint32_t(key ^ (key >> 29) ^ (key >> 48)) * 0x9e3779b1u;
        h >>= 25;  // 7 bits: kCatSlots
        for (int probe = 0; probe < kCatSlots; probe++) {
          const unsigned long long old = atomicCAS(&sh_ckey[h], 0ull, (unsigned long long)key);
          if (old == 0ull || old == key) {
            cslot[j] = int(h);
            break;
          }
          h = (h + 1) & (kCatSlots - 1);
        }
        if (cslot[j] < 0) atomicOr(&sh_cflag, 1);
        else atomicAdd(&sh_ccnt[cslot[j]], 1);
      }
      __syncthreads();
      cat_ok = sh_cflag == 0;  // block-uniform
    }
    KTAS_FILL_STAMP(3);
    uint64_t U0 = 0, U1 = 0;  // the table's used slots: dense id = rank among them
    if (cat_ok) {
      U0 = ballot(sh_ckey[lane] != 0ull);
      U1 = ballot(sh_ckey[kWave + lane] != 0ull);
      ncat = __popcll(U0) + __popcll(U1);
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        const int sl = cslot[j];
        did[j] = sl < 0 ? 0
                 : sl < kWave ? __popcll(U0 & ((1ull << sl) - 1ull))
                              : __popcll(U0) + __popcll(U1 & ((1ull << (sl - kWave)) - 1ull));
      }
      if (threadIdx.x < kCatSlots) {  // the dense table (threads of waves 0 and 1: a slot each)
        const int sl = int(threadIdx.x);
        const uint64_t Uh = sl < kWave ? U0 : U1;
        if ((Uh >> (sl & 63)) & 1ull) {
          const int d = (sl < kWave ? 0 : __popcll(U0)) + __popcll(Uh & ((1ull << (sl & 63)) - 1ull));
          sh_dkey[d] = sh_ckey[sl];
          sh_dcnt[d] = sh_ccnt[sl];
        }
      }
      __syncthreads();
    }
    if (cat_ok) {
      // the classes' verdicts per category: wave w takes classes w, w + 4, ...;
      // a lane per dense category id (a second half past 64 categories)
      const int wave = int(threadIdx.x >> 6);
      const bool hn = s.lowest_is_hostname != 0;
      const int halves = ncat > kWave ? 2 : 1;
      for (int e = wave; e < ne; e += kFillThreads / kWave) {
        const FillEvalParams& P = sh_pos[e].p;
        const int nsel = P.nsel;
        const uint32_t mlo = uint32_t(P.sel_mlo), mhi = uint32_t(P.sel_mhi), wlo = uint32_t(P.sel_wlo),
                       whi = uint32_t(P.sel_whi);
        if (halves == 1 && lane == 0) sh_passd[2 * e + 1] = 0ull;
        for (int half = 0; half < halves; half++) {
          const int dd = half * kWave + lane;
          const bool used = dd < ncat;
          const uint64_t key = used ? sh_dkey[dd] : 0ull;
          const uint32_t small = uint32_t(key >> 48);
          const bool dead = (small & 1u) != 0;
          const int pf = int((small >> 1) & 31u);
          const int zl = int((small >> 6) & 63u) - 1;
          uint32_t lo = 0u, hi = 0u;
#pragma unroll
          for (int q = 0; q < 3; q++) {
            if (q < nf) {
              const int f = fld[q];
              const uint32_t v = uint32_t(key >> (16 * q)) & 0xffffu;
              if (f < 2) lo |= v << (16 * (f & 1));
              else hi |= v << (16 * (f & 1));
            }
          }
          bool ok = used && !dead;
          int x = -1;
          if (hn && s.taint_profile) {
            const int t = sh_pos[e].taint[pf];
            x = (ok && t >= 0) ? kStatFixed + t : x;
            ok = ok && t < 0;
          }
          if (hn && nsel > 0) {
            const bool mis = ((lo & mlo) != wlo) | ((hi & mhi) != whi);
            x = (ok && mis) ? 0 : x;
            ok = ok && !mis;
          }
          x = (ok && zl >= 0) ? kStatFixed + b.num_taints + zl : x;
          if (x >= 0) atomicAdd(&sh_stats[e][x], sh_dcnt[dd]);
          const uint64_t pass = ballot(ok);
          if (lane == 0) sh_passd[2 * e + half] = pass;
        }
      }
      __syncthreads();
      KTAS_FILL_STAMP(4);
    }
  }
  // ragged slots: the parents of the lane's two leaves, which of them start
  // (head) or end (tail) a parent, and the lane holding the start of its
  // second leaf's parent (the segmented scans' bound)
  int rp[kPairLP] = {}, seg0 = 0, st0 = 0, st1 = 0;
  bool head0 = false, head1 = false, tail0 = false, tail1 = false;
  if constexpr (FC < 0) {
    rp[0] = valid[0] ? s.leaf_parent[leaf0] : -1;
    rp[1] = valid[1] ? s.leaf_parent[leaf0 + 1] : -2;
    const int pprev = __shfl(rp[1], lane > 0 ? lane - 1 : 0);
    const int pnext = __shfl(rp[0], lane < kWave - 1 ? lane + 1 : lane);
    head0 = valid[0] && (lane == 0 || pprev != rp[0]);
    head1 = valid[1] && rp[1] != rp[0];
    tail0 = valid[0] && (!valid[1] || rp[1] != rp[0]);
    tail1 = valid[1] && (lane == kWave - 1 || pnext != rp[1]);
    const uint64_t H = ballot(head0 || head1);
    const uint64_t upto = lane == kWave - 1 ? ~0ull : ((2ull << lane) - 1ull);
    seg0 = 63 - __builtin_clzll((H & upto) | 1ull);
    // slot positions (2 * lane + j) where the leaves' parents start
    const int hpos = head1 ? kPairLP * lane + 1 : kPairLP * lane;
    st1 = __shfl(hpos, seg0);
    const int st1_prev = __shfl(st1, lane > 0 ? lane - 1 : 0);
    st0 = head0 ? kPairLP * lane : st1_prev;
  }
  const int rack_f = FC > 0 ? FC : FC < 0 ? -1 : b.rack_fanout;  // fan-out of the fused parents (0: none, -1: ragged)
  const int half = rack_f / kPairLP;                    // lanes per parent
  const int parent = rack_f > 0 ? leaf0 / rack_f : 0;
  const int gpos = rack_f > 0 ? (lane & (half - 1)) : 0;  // this lane's group within its parent
  // every leaf of the block's tile exists and its counter words are
  // kPairLP-aligned (level offsets are multiples of 4): block-uniform, so the
  // stores below take a scalar branch, not a per-lane exec mask
  const bool full_tile = FC >= 0 && (tile + 1) * kPairTile <= N && (s.level_off[s.L - 1] & (kPairLP - 1)) == 0;
  const int64_t SD = s.SD;
  // CAT, every class of the chunk simple (no leader, one-pod slices at the
  // leaf level, no inner rounding: sliceState is state at the leaves and the
  // parents) and uniform parents: the lean loop — per class a pass-mask
  // lookup per leaf, the counter stores and the fused parents, nothing else
  bool lean = false;
  if constexpr (CAT && FC >= 0) {
    lean = cat_ok && !leader && ncat <= kWave;
    for (int e = 0; e < ne && lean; e++) lean = sh_pos[e].p.ss_alias != 0;  // simple (the host's mark)
  }
  if (lean) {
    // per class: a leaf's state is state0 under its category's pass bit (a
    // 0 / -1 mask); the leaf-pair store; the parent's state and positive-
    // children mask from the same masks (pA / pB: the lane's leaves that have
    // room, at their bits of the parent's mask); rows and parents by pointer
    const int lsz = rack_f > 0 ? s.level_size[s.L - 2] : 0;
    const int poff = rack_f > 0 ? s.level_off[s.L - 2] : 0;
    const bool has_par = rack_f > 0 && valid[0] && parent < lsz && b.rack_pos != nullptr;
    const uint64_t pA = (valid[0] && state0[0] > 0) ? 1ull << (kPairLP * gpos) : 0ull;
    const uint64_t pB = (valid[1] && state0[1] > 0) ? 2ull << (kPairLP * gpos) : 0ull;
    uint64_t* rpp = b.rack_pos ? b.rack_pos + int64_t(e0) * lsz + parent : nullptr;
    // fast-LFC chunk tables from the fill: the wave's (category, value) pairs
    bool lfc_any = false;
    if constexpr (LF) {
      if (b.lfc_fill)
        for (int e = 0; e < ne; e++) lfc_any = lfc_any || sh_pos[e].p.lfc_slot >= 0;
    }
    if (lfc_any) {
      const int wv = int(threadIdx.x >> 6);
      const bool a0 = valid[0] && state0[0] > 0, a1 = valid[1] && state0[1] > 0;
      const uint64_t k0 = (uint64_t(uint32_t(did[0])) << 32) | uint32_t(state0[0]);
      const uint64_t k1 = (uint64_t(uint32_t(did[1])) << 32) | uint32_t(state0[1]);
      uint64_t p0 = ballot(a0), p1 = ballot(a1);
      int nt = 0;
      while (p0 | p1) {
        const bool first = p0 != 0;
        const int src = __ffsll((unsigned long long)(first ? p0 : p1)) - 1;
        const uint64_t key = bcast64(first ? k0 : k1, src);
        const uint64_t m0 = ballot(a0 && k0 == key), m1 = ballot(a1 && k1 == key);
        if (lane == 0) {
          sh_tv[wv * kTri + nt] = int32_t(uint32_t(key));
          sh_tc[wv * kTri + nt] = ((__popcll(m0) + __popcll(m1)) << 8) | int32_t(key >> 32);
        }
        nt++;
        p0 &= ~m0;
        p1 &= ~m1;
      }
      if (lane == 0) sh_tn[wv] = nt;
    }
    const int lfc_chunk = (tile * kPairTile) / kLfcChunk;  // the block's leaves lie in one LFC chunk
    for (int e = 0; e < ne; e++, rpp += lsz) {
      int32_t* const rowp = b.counters + int64_t(sh_pos[e].p.ctr_row) * b.ctr_sd;
      const uint64_t pm = sh_passd[2 * e];
      const int32_t m0 = int32_t(uint32_t(pm >> did[0]) << 31) >> 31;
      const int32_t m1 = int32_t(uint32_t(pm >> did[1]) << 31) >> 31;
      const int32_t st0 = state0[0] & m0, st1 = state0[1] & m1;
      if (lfc_any) {
        const int lslot = sh_pos[e].p.lfc_slot;  // block-uniform
        if (lslot >= 0) {  // the byte copy of the class's leaf values (lfc_emit_kernel)
          uint8_t* u8 = b.lfc_u8 + int64_t(lslot) * b.lfc_nchunks * kLfcChunk + leaf0;
          const uint32_t c0 = uint32_t(min(st0, 255)), c1 = uint32_t(min(st1, 255));
          if (full_tile) *reinterpret_cast<uint16_t*>(u8) = uint16_t(c0 | (c1 << 8));
          else {
            if (valid[0]) u8[0] = uint8_t(c0);
            if (valid[1]) u8[1] = uint8_t(c1);
          }
        }
      }
      // (the sliceState row is not stored: FillEvalParams::ss_alias)
      if (full_tile) {
        *reinterpret_cast<int2*>(rowp + gleaf0) = make_int2(st0, st1);
      } else {
        if (valid[0]) rowp[gleaf0] = st0;
        if (valid[1]) rowp[gleaf0 + 1] = st1;
      }
      if (rack_f > 0) {  // fused fillInCountsHelper (:1658-1719) of the leaves' parents
        const int32_t cap2 = group_reduce(w_add(st0, st1), half, OpWAdd());
        const uint64_t bits = (uint64_t(int64_t(m0)) & pA) | (uint64_t(int64_t(m1)) & pB);
        uint64_t posm = uint32_t(group_reduce(int32_t(uint32_t(bits)), half, OpOr()));
        if (rack_f > 32) posm |= uint64_t(uint32_t(group_reduce(int32_t(uint32_t(bits >> 32)), half, OpOr()))) << 32;
        if (gpos == 0 && has_par) {
          *rpp = posm;
          rowp[poff + parent] = cap2;
        }
      }
    }
    if (lfc_any) {  // the slot classes' counts: wave w takes classes w, w + 4, ...
      __syncthreads();  // every wave's pairs
      const int wv = int(threadIdx.x >> 6);
      const int nvalid = min(kPairTile, N - tile * kPairTile);
      for (int e = wv; e < ne; e += kFillThreads / kWave) {
        const int lslot = sh_pos[e].p.lfc_slot;
        if (lslot < 0) continue;
        const uint64_t pm = sh_passd[2 * e];
        uint32_t* ch = b.lfc_ch + (int64_t(lslot) * b.lfc_nchunks + lfc_chunk) * kLfcBins;
        int pos_cnt = 0;
        unsigned long long osum = 0;
        for (int w2 = 0; w2 < kFillThreads / kWave; w2++) {
          const int nt = sh_tn[w2];
          for (int i = lane; i < nt; i += kWave) {
            const int32_t v = sh_tv[w2 * kTri + i];
            const int32_t tc = sh_tc[w2 * kTri + i];
            const int cnt = tc >> 8, d = tc & 0xff;
            if ((pm >> d) & 1ull) {  // the class takes this category: value v on cnt leaves
              atomicAdd(&ch[v >= kLfcBins - 1 ? kLfcBins - 1 : v], uint32_t(cnt));
              pos_cnt += cnt;
              if (v >= kLfcBins - 1) osum += (unsigned long long)int64_t(v) * (unsigned long long)cnt;
            }
          }
        }
        pos_cnt = int(wave_sum_i64(pos_cnt));
        osum = (unsigned long long)wave_sum_i64(int64_t(osum));
        if (lane == 0) {
          if (nvalid - pos_cnt > 0) atomicAdd(&ch[0], uint32_t(nvalid - pos_cnt));  // value 0: every other leaf
          if (osum)
            atomicAdd(reinterpret_cast<unsigned long long*>(&b.lfc_ovs[int64_t(lslot) * b.lfc_nchunks + lfc_chunk]), osum);
        }
      }
    }
  }
  KTAS_FILL_STAMP(5);
  for (int e = 0; e < ne && !lean; e++) {
    const int4* pq = reinterpret_cast<const int4*>(&sh_pos[e].p);
    const int4 q0 = pq[0], q1 = pq[1], q2 = pq[2];
    if constexpr (MR) {
      if (uni(q2.w)) count_run(e);  // sig_new
    }
    const int eid = uni(q0.x);
    const int nsel = uni(q0.y);
    const int32_t slice_size = uni(q0.z), slice_level = uni(q0.w);
    const int32_t p_inner = uni(q1.x), sel_far = uni(q1.y), aff_begin = uni(q1.z), aff_end = uni(q1.w);
    const int32_t dom_begin = uni(q2.x), dom_end = uni(q2.y);
    // per-leaf classification as selects (fillInCounts :1578-1643, first
    // exclusion wins: taint, nodeSelector, affinity, required domain, then
    // a resource giving state 0): every condition below is either
    // wave-uniform (a scalar branch) or a v_cndmask, no divergent branch
    int32_t state[kPairLP], swl[kPairLP], ls[kPairLP], ss[kPairLP], sswl[kPairLP];
    bool okm[kPairLP];
    int kind[kPairLP], id[kPairLP];
    const bool hn = s.lowest_is_hostname != 0;
    int4 c0 = make_int4(0, 0, 0, 0), c1 = c0, v0 = c0, v1 = c0;
    if (hn && nsel > 0) {
      c0 = pq[4];
      c1 = pq[5];
      v0 = pq[6];
      v1 = pq[7];
    }
    const int32_t sc[KUEUE_TAS_MAX_SELECTORS] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const int32_t sv[KUEUE_TAS_MAX_SELECTORS] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    bool sel_fast = false;
    uint32_t sel_mlo = 0u, sel_mhi = 0u, sel_wlo = 0u, sel_whi = 0u;
    if (hn && nsel > 0) {
      const int4 m = pq[9];
      sel_fast = uni(pq[10].x) != 0;
      sel_mlo = uint32_t(uni(m.x));
      sel_mhi = uint32_t(uni(m.y));
      sel_wlo = uint32_t(uni(m.z));
      sel_whi = uint32_t(uni(m.w));
    }
    // CAT: the class's pass mask over the block's categories (the verdicts
    // and the ExclusionStats were settled before the loop)
    const bool cat_cls = CAT && cat_ok;  // block-uniform
    if (cat_cls) {
      const uint64_t p0 = sh_passd[2 * e], p1 = sh_passd[2 * e + 1];
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        const uint64_t w = did[j] >= kWave ? p1 : p0;
        okm[j] = cslot[j] >= 0 && ((w >> (did[j] & 63)) & 1ull);
        state[j] = okm[j] ? state0[j] : 0;
      }
    }
    if (!cat_cls) {
#pragma unroll
    for (int j = 0; j < kPairLP; j++) {
      const int leaf = leaf0 + j;
      bool ok = live[j];
      int k = (valid[j] && !live[j]) ? EX_DEAD : EX_NONE;
      int idv = -1;
      if (hn && s.taint_profile) {
        int t;
        if constexpr (TS) t = sh_pos[e].taint[prof[j]];
        else t = b.taint_table[uni(q2.z) + prof[j]];
        const bool x = ok & (t >= 0);
        k = x ? EX_TAINT : k;
        idv = x ? t : idv;
        ok = ok & !x;
      }
      if (hn && nsel > 0) {
        const int32_t l0 = lab[j][0], l1 = lab[j][1], l2 = lab[j][2], l3 = lab[j][3];
        bool mis = false;
        if (sel_fast) {  // wave-uniform: one masked compare of the packed key
          mis = ((pk_lo[j] & sel_mlo) != sel_wlo) | ((pk_hi[j] & sel_mhi) != sel_whi);
        } else if (!GL || !sel_far) {
#pragma unroll
          for (int q = 0; q < KUEUE_TAS_MAX_SELECTORS; q++) {
            if (q < nsel) {  // wave-uniform
              const int col = uni(sc[q]);
              int32_t v = l0;
              v = col == 1 ? l1 : v;
              v = col == 2 ? l2 : v;
              v = col == 3 ? l3 : v;
              mis = mis | (v != uni(sv[q]));
            }
          }
        } else if (ok) {
          auto label_at = [s, leaf, l0, l1, l2, l3](int col) { return staged_label(s, leaf, col, l0, l1, l2, l3); };
#pragma unroll
          for (int q = 0; q < KUEUE_TAS_MAX_SELECTORS; q++)
            if (q < nsel && !mis && label_at(uni(sc[q])) != uni(sv[q])) mis = true;
          if constexpr (GL) {
            const int32_t sxb = uni(pq[3].w);
            if (!mis && sxb >= 0 && !selector_ext_match(b, sxb, uni(pq[8].x), leaf, label_at)) mis = true;
          }
        }
        const bool x = ok & mis;
        k = x ? EX_SELECTOR : k;
        ok = ok & !mis;
      }
      if constexpr (GL) {
        if (hn && aff_begin >= 0 && ok) {
          const int32_t l0 = lab[j][0], l1 = lab[j][1], l2 = lab[j][2], l3 = lab[j][3];
          auto label_at = [s, leaf, l0, l1, l2, l3](int col) { return staged_label(s, leaf, col, l0, l1, l2, l3); };
          if (!affinity_match(b, aff_begin, aff_end, leaf, label_at)) {
            k = EX_AFFINITY;
            ok = false;
          }
        }
      }
      if (dom_begin >= 0) {
        const bool x = ok & outside_domain(dom_begin, dom_end, leaf);
        k = x ? EX_TOPOLOGY : k;
        ok = ok & !x;
      }
      state[j] = ok ? state0[j] : 0;
      okm[j] = ok;
      const bool rx = ok & (state0[j] == 0) & (lim0[j] >= 0);
      kind[j] = rx ? EX_RESOURCE : k;
      id[j] = rx ? lim0[j] : idv;
    }
    }  // !cat_cls
    // a simple class (no leader, one-pod slices at the leaf level, no inner
    // slice rounding — every class of C3): sliceState is state and no
    // leader field exists, one wave-uniform branch instead of one per field
    const bool simple = !leader && s.L - 1 == slice_level && slice_size == 1 && (p_inner == 0 || p_inner == 1);
    if (simple) {
#pragma unroll
      for (int j = 0; j < kPairLP; j++) ss[j] = state[j];
    } else {
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        swl[j] = okm[j] ? swl0[j] : 0;
        ls[j] = okm[j] ? ls0[j] : 0;
        ss[j] = sswl[j] = 0;
        if (s.L - 1 == slice_level) {
          if (slice_size == 1) {
            ss[j] = state[j];
            sswl[j] = swl[j];
          } else {
            ss[j] = go_div32(state[j], slice_size);
            sswl[j] = leader ? go_div32(swl[j], slice_size) : ss[j];
          }
        }
      }
    }
    int32_t* base = ctr_base(b, e0 + e);  // the class's row: its fill position
    auto storev = [&](int64_t off, const int32_t (&v)[kPairLP]) {  // counter words of leaves leaf0 .. leaf0 + kPairLP - 1
      if (full_tile) {
        if constexpr (kPairLP == 4) *reinterpret_cast<int4*>(base + off + gleaf0) = make_int4(v[0], v[1], v[2], v[3]);
        else *reinterpret_cast<int2*>(base + off + gleaf0) = make_int2(v[0], v[1]);
      } else {
#pragma unroll
        for (int j = 0; j < kPairLP; j++)
          if (valid[j]) base[off + gleaf0 + j] = v[j];
      }
    };
    // a simple class's sliceState is its state: the host marks it (ss_alias)
    // and every reader takes the state row
    const bool alias = uni(sh_pos[e].p.ss_alias) != 0;
    storev(0, state);
    if (!alias) storev(SD, ss);
    if (b.lfc_fill) {  // a fast-LFC slot class (always simple: its values are state)
      const int lslot = uni(sh_pos[e].p.lfc_slot);
      if (lslot >= 0) {
        const int lv[kPairLP] = {leaf0, leaf0 + 1};
        lfc_fill_accum(b, lslot, state, lv, valid, kPairLP);
      }
    }
    if (leader) {
      storev(2 * SD, swl);
      storev(3 * SD, sswl);
      storev(4 * SD, ls);
    }
    // positive children of the lane's parent group: bits kPairLP*gpos ..
    // kPairLP*gpos + kPairLP - 1 of the parent's mask
    auto pos_mask = [&]() -> uint64_t {
      uint32_t pb = 0;
#pragma unroll
      for (int j = 0; j < kPairLP; j++) pb |= uint32_t(valid[j] && ss[j] > 0) << j;
      if (rack_f <= 32) return uint32_t(group_reduce(int32_t(pb << (kPairLP * gpos)), half, OpOr()));
      const int lo_groups = 32 / kPairLP;
      const uint32_t lo = uint32_t(group_reduce(int32_t(gpos < lo_groups ? pb << (kPairLP * gpos) : 0u), half, OpOr()));
      const uint32_t hi = uint32_t(group_reduce(int32_t(gpos >= lo_groups ? pb << (kPairLP * gpos - 32) : 0u), half, OpOr()));
      return (uint64_t(hi) << 32) | lo;
    };
    // fused fillInCountsHelper (:1658-1719) of the leaves' parents
    if (rack_f > 0 && simple) {  // sliceState == state at the parent too
      int32_t cap2 = 0;
#pragma unroll
      for (int j = 0; j < kPairLP; j++) cap2 = w_add(cap2, state[j]);
      cap2 = group_reduce(cap2, half, OpWAdd());
      const uint64_t posm = pos_mask();
      if (gpos == 0 && valid[0] && parent < s.level_size[s.L - 2]) {
        b.rack_pos[int64_t(e0 + e) * s.level_size[s.L - 2] + parent] = posm;
        const int g = s.level_off[s.L - 2] + parent;
        base[g] = cap2;
        if (!alias) base[SD + g] = cap2;
      }
    } else if (rack_f > 0) {
      const int32_t inner = p_inner;
      int32_t cap2 = 0, slc = 0, lead = 0, minD = 0x7fffffff, minSD = 0x7fffffff, has = 0;
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        int32_t cs = state[j], csw = swl[j];
        if (inner != 0 && inner != 1) {
          cs = w_mul(go_div32(cs, inner), inner);
          csw = w_mul(go_div32(csw, inner), inner);
        }
        cap2 = w_add(cap2, cs);
        slc = w_add(slc, ss[j]);
        lead = max(lead, ls[j]);
        if (!leader || ls[j] > 0) {
          has = 1;
          minD = min(minD, w_sub(cs, csw));
          minSD = min(minSD, w_sub(ss[j], sswl[j]));
        }
      }
      const bool same = s.L - 1 == slice_level && inner == 1 && slice_size == 1;  // wave-uniform: slc == cap2
      cap2 = group_reduce(cap2, half, OpWAdd());
      if (s.L - 1 != slice_level) slc = 0;
      else if (same) slc = cap2;
      else slc = group_reduce(slc, half, OpWAdd());
      if (leader) {
        minD = group_reduce(minD, half, OpMin());
        minSD = group_reduce(minSD, half, OpMin());
        lead = group_reduce(lead, half, OpMax());
        has = group_reduce(has, half, OpMax());
      }
      const uint64_t posm = pos_mask();
      if (gpos == 0 && valid[0] && parent < s.level_size[s.L - 2]) {
        b.rack_pos[int64_t(e0 + e) * s.level_size[s.L - 2] + parent] = posm;
        const int32_t pswl = has ? w_sub(cap2, minD) : 0;
        int32_t psswl = has ? w_sub(slc, minSD) : 0;
        if (s.L - 2 == slice_level) {
          slc = go_div32(cap2, slice_size);
          psswl = go_div32(pswl, slice_size);
        }
        const int g = s.level_off[s.L - 2] + parent;
        base[g] = cap2;
        if (!alias) base[SD + g] = slc;
        if (leader) {
          base[2 * SD + g] = pswl;
          base[3 * SD + g] = psswl;
          base[4 * SD + g] = lead;
        }
      }
    }
    // the same over ragged parents (no leader classes here): per lane the
    // summary of its second leaf's parent segment (just that leaf when it
    // starts a parent, else both leaves), segmented inclusive scans bounded
    // by the segment's first lane; a parent ending at the lane's first leaf
    // takes the previous lane's scan plus that leaf
    if constexpr (FC < 0) {
      const int32_t inner = p_inner;
      int32_t v[kPairLP];
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        v[j] = state[j];
        if (inner != 0 && inner != 1) v[j] = w_mul(go_div32(v[j], inner), inner);
      }
      auto seg_sum = [&](int32_t a0, int32_t a1, int32_t* t0, int32_t* t1) {
        const int32_t S = seg_incl_scan(head1 ? a1 : w_add(a0, a1), lane, seg0, OpWAdd());
        const int32_t Sp = __shfl(S, lane > 0 ? lane - 1 : 0);
        *t1 = S;
        *t0 = w_add(head0 ? 0 : Sp, a0);
      };
      int32_t cap0, cap1, slc0 = 0, slc1 = 0;
      seg_sum(v[0], v[1], &cap0, &cap1);
      if (s.L - 1 != slice_level) {  // wave-uniform: the leaves' sliceState is 0
      } else if (inner == 1 && slice_size == 1) {  // wave-uniform: sliceState == state
        slc0 = cap0;
        slc1 = cap1;
      } else {
        seg_sum(ss[0], ss[1], &slc0, &slc1);
      }
      const bool masks = b.rack_pos != nullptr;  // every parent <= 64 leaves
      uint64_t pm0 = 0, pm1 = 0;
      if (masks) {  // positive children: disjoint bits per parent, so the segment sums are its ORs
        const uint64_t m0 = (valid[0] && ss[0] > 0) ? 1ull << ((kPairLP * lane - st0) & 63) : 0ull;
        const uint64_t m1 = (valid[1] && ss[1] > 0) ? 1ull << ((kPairLP * lane + 1 - st1) & 63) : 0ull;
        int32_t lo0, lo1, hi0, hi1;
        seg_sum(int32_t(uint32_t(m0)), int32_t(uint32_t(m1)), &lo0, &lo1);
        seg_sum(int32_t(uint32_t(m0 >> 32)), int32_t(uint32_t(m1 >> 32)), &hi0, &hi1);
        pm0 = (uint64_t(uint32_t(hi0)) << 32) | uint32_t(lo0);
        pm1 = (uint64_t(uint32_t(hi1)) << 32) | uint32_t(lo1);
      }
      auto put_parent = [&](int par, int32_t cp, int32_t sl, uint64_t pm) {
        const int g = s.level_off[s.L - 2] + par;
        if (wide_slot) {  // (wave-uniform) one piece of a wider parent: the pieces' sums add up
          // (int32 wrap: in any order) into the zeroed parent; a sliceState at
          // the slice level is the whole sum's quotient (wide_parents_finish_kernel)
          atomicAdd(&base[g], cp);
          if (!alias && s.L - 2 != slice_level) atomicAdd(&base[SD + g], sl);
          return;
        }
        if (masks) b.rack_pos[int64_t(e0 + e) * s.level_size[s.L - 2] + par] = pm;
        if (s.L - 2 == slice_level) sl = go_div32(cp, slice_size);
        base[g] = cp;
        if (!alias) base[SD + g] = sl;
      };
      if (tail0) put_parent(rp[0], cap0, slc0, pm0);
      if (tail1) put_parent(rp[1], cap1, slc1, pm1);
    }
    // ExclusionStats (:1579-1634): every excluded leaf maps to its stats slot
    // (nodeSelector, affinity, topologyDomain, taint id, resource id); one
    // loop over the distinct slots present in the wave's 128 leaves, each a
    // ballot per leaf of the lane, the counts gathered in the lane that owns
    // the slot (kMaxFillStats == 64 slots, one per lane) and added to LDS
    // with one conflict-free ds_add per lane: no per-kind sections, no
    // single-lane atomics (exec-mask bookkeeping on the scalar unit)
    if (cat_cls) continue;  // counted per category above
    if (lds_stats) {
      static_assert(kMaxFillStats == kWave, "one stats slot per lane");
      int sl[kPairLP];
      uint64_t m[kPairLP];
      uint64_t any = 0;
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        int x = -1;
        x = kind[j] == EX_SELECTOR ? 0 : x;
        x = kind[j] == EX_AFFINITY ? 1 : x;
        x = kind[j] == EX_TOPOLOGY ? 2 : x;
        x = kind[j] == EX_TAINT ? kStatFixed + id[j] : x;
        x = kind[j] == EX_RESOURCE ? kStatFixed + b.num_taints + id[j] : x;
        sl[j] = valid[j] ? x : -1;
        m[j] = ballot(sl[j] >= 0);
        any |= m[j];
      }
      if (any == 0) continue;
      int32_t acc = 0;
      while (any) {  // wave-uniform: one trip per distinct slot
        int x = 0;
#pragma unroll
        for (int j = kPairLP - 1; j >= 0; j--)
          if (m[j]) x = bcast(sl[j], __ffsll((unsigned long long)m[j]) - 1);
        int c = 0;
        any = 0;
#pragma unroll
        for (int j = 0; j < kPairLP; j++) {
          const uint64_t h = ballot(sl[j] == x);
          c += __popcll(h);
          m[j] &= ~h;
          any |= m[j];
        }
        acc += lane == x ? c : 0;
      }
      atomicAdd(&sh_stats[e][lane], acc);
      continue;
    }
    uint64_t anyx = 0;
#pragma unroll
    for (int j = 0; j < kPairLP; j++) anyx |= ballot(valid[j] && kind[j] != EX_NONE && kind[j] != EX_DEAD);
    if (anyx == 0) continue;
    auto count_kind = [&](int k, int slot, int32_t* gl) {
      int c = 0;
#pragma unroll
      for (int j = 0; j < kPairLP; j++) c += __popcll(ballot(kind[j] == k));
      if (lane == 0 && c) {
        if (lds_stats) atomicAdd(&sh_stats[e][slot], c);
        else atomicAdd(gl, c);
      }
    };
    if (nsel > 0) count_kind(EX_SELECTOR, 0, &b.sel_counts[eid]);
    if (aff_begin >= 0) count_kind(EX_AFFINITY, 1, &b.aff_counts[eid]);
    if (dom_begin >= 0) count_kind(EX_TOPOLOGY, 2, &b.dom_counts[eid]);
    // per taint / resource id: the first remaining lane's id, both halves counted together
    auto count_ids = [&](int k, int slot0, int32_t* gl) {
      uint64_t m[kPairLP];
      uint64_t any = 0;
#pragma unroll
      for (int j = 0; j < kPairLP; j++) {
        m[j] = ballot(kind[j] == k);
        any |= m[j];
      }
      while (any) {
        int x = 0;  // the id of the first lane / leaf still to count
#pragma unroll
        for (int j = kPairLP - 1; j >= 0; j--)
          if (m[j]) x = bcast(id[j], __ffsll((unsigned long long)m[j]) - 1);
        int c = 0;
        any = 0;
#pragma unroll
        for (int j = 0; j < kPairLP; j++) {
          const uint64_t h = ballot(kind[j] == k && id[j] == x);
          c += __popcll(h);
          m[j] &= ~h;
          any |= m[j];
        }
        if (lane == 0) {
          if (lds_stats) atomicAdd(&sh_stats[e][slot0 + x], c);
          else atomicAdd(gl + x, c);
        }
      }
    };
    count_ids(EX_TAINT, kStatFixed, b.taint_counts + int64_t(eid) * b.num_taints);
    count_ids(EX_RESOURCE, kStatFixed + b.num_taints, b.res_counts + int64_t(eid) * s.R);
  }
  if (lds_stats) {  // per-block partials [fill position][tile][stat]; slots past this grid's tiles zeroed
    __syncthreads();
    const int nb = b.nstat_blocks;
    for (int i = threadIdx.x; i < ne * b.nstat; i += kFillThreads) {
      const int e = i / b.nstat, k = i % b.nstat;
      b.fill_stats[(int64_t(e0 + e) * nb + tile) * b.nstat + k] = sh_stats[e][k];
      for (int t = tile + int(gridDim.x); t < nb; t += int(gridDim.x))
        b.fill_stats[(int64_t(e0 + e) * nb + t) * b.nstat + k] = 0;
    }
  }
}

// Leaf parents wider than a fill slot (DevSnap::wide_parents): zeroed in every
// class row before fill_pair_kernel's ragged mode adds its pieces' sums, and
// afterwards, for classes whose slice level is the parents' level, their
// sliceState = state / sliceSize (fillInCountsHelper :1712-1716).
__global__ __launch_bounds__(256) void wide_parents_zero_kernel(DevSnap s, DevBatch b) {
  const int row = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= b.nfill || i >= s.n_wide) return;
  int32_t* base = ctr_base(b, row);
  const int g = s.level_off[s.L - 2] + s.wide_parents[i];
  base[g] = 0;
  if (!b.fill_pos[row].p.ss_alias) base[s.SD + g] = 0;
}
__global__ __launch_bounds__(256) void wide_parents_finish_kernel(DevSnap s, DevBatch b) {
  const int row = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= b.nfill || i >= s.n_wide) return;
  const FillEvalParams& P = b.fill_pos[row].p;
  if (P.slice_level != s.L - 2 || P.ss_alias) return;
  int32_t* base = ctr_base(b, row);
  const int g = s.level_off[s.L - 2] + s.wide_parents[i];
  base[s.SD + g] = go_div32(base[g], P.slice_size);
}

// ExclusionStats of the staged fill's classes (fillInCounts :1578-1634:
// first untolerated taint, then nodeSelector, then a resource giving state 0)
// in a kernel of their own, off the fill's critical path: it runs on a
// third stream beside the roll-up and select.  Same grid and masks as the
// fill; the resource case reads the limiting resource the fill recorded per
// (chunk, leaf) where the chunk's signature gives state 0.
template <bool TS>  // as fill_leaves_staged_kernel
__global__ __launch_bounds__(kFillThreads) void fill_exclusion_kernel(DevSnap s, DevBatch b) {
  __shared__ int32_t sh_toff[kEvalsPerBlock];
  __shared__ int32_t sh_nsel[kEvalsPerBlock];
  __shared__ int32_t sh_run[kEvalsPerBlock];
  __shared__ int32_t sh_aff[kEvalsPerBlock][4];  // affinity range, required-domain leaf range
  __shared__ int32_t sh_sel[kEvalsPerBlock][2 * KUEUE_TAS_MAX_SELECTORS];
  __shared__ int32_t sh_sx[kEvalsPerBlock][2];  // nodeSelector requirements beyond the inline pairs
  __shared__ int32_t sh_taint[kEvalsPerBlock][kStagedProfiles];
  __shared__ int32_t sh_stats[kEvalsPerBlock][kMaxFillStats];
  for (int i = threadIdx.x; i < kEvalsPerBlock * kMaxFillStats; i += kFillThreads) (&sh_stats[0][0])[i] = 0;
  const int e0 = b.fill_chunks[2 * blockIdx.y];
  const int ne = b.fill_chunks[2 * blockIdx.y + 1];
  constexpr bool stage_taints = TS;
  if (int(threadIdx.x) < ne) {
    const DevEval& ev = b.evals[b.fill_ids[e0 + threadIdx.x]];
    sh_toff[threadIdx.x] = ev.taint_table;
    sh_nsel[threadIdx.x] = ev.nsel;
    sh_run[threadIdx.x] = b.fill_run[e0 + threadIdx.x];
    const bool aff = (ev.flags & KUEUE_TAS_F_AFFINITY) != 0;
    sh_aff[threadIdx.x][0] = aff ? ev.aff_begin : -1;
    sh_aff[threadIdx.x][1] = aff ? ev.aff_end : -1;
    sh_aff[threadIdx.x][2] = ev.dom_begin;
    sh_aff[threadIdx.x][3] = ev.dom_end;
    for (int k = 0; k < KUEUE_TAS_MAX_SELECTORS; k++) {
      sh_sel[threadIdx.x][2 * k] = ev.sel_col[k];
      sh_sel[threadIdx.x][2 * k + 1] = ev.sel_val[k];
    }
    sh_sx[threadIdx.x][0] = ev.sx_begin;
    sh_sx[threadIdx.x][1] = ev.sx_end;
  }
  __syncthreads();
  if (s.taint_profile && stage_taints) {
    for (int i = threadIdx.x; i < ne * kStagedProfiles; i += kFillThreads) {
      const int e = i / kStagedProfiles, p = i % kStagedProfiles;
      sh_taint[e][p] = p < b.num_profiles ? b.taint_table[sh_toff[e] + p] : -1;
    }
  }
  __syncthreads();
  const int leaf = blockIdx.x * kFillThreads + threadIdx.x;
  const bool valid = leaf < s.N;
  const int N = s.N;
  const int lane = lane_id();
  const int prof = (valid && s.taint_profile) ? s.taint_profile[leaf] : 0;
  int lim = -1;  // limiting resource of the position's signature run (the fill recorded it)
  int32_t lab[kStagedLabels];
#pragma unroll
  for (int k = 0; k < kStagedLabels; k++) lab[k] = (valid && s.label_values && k < s.K) ? s.label_values[int64_t(k) * N + leaf] : 0;
  static_assert(kStagedLabels == 4, "staged_label takes four staged columns");
  const int32_t lab0 = lab[0], lab1 = lab[1], lab2 = lab[2], lab3 = lab[3];
  auto label_at = [s, leaf, lab0, lab1, lab2, lab3](int col) {  // by value: nothing escapes to scratch
    return staged_label(s, leaf, col, lab0, lab1, lab2, lab3);
  };
  const bool dead = valid && leaf_out(s, leaf);
  for (int e = 0; e < ne; e++) {
    const int run = uni(sh_run[e]);
    if (e == 0 || run != uni(sh_run[e - 1])) lim = valid ? int(b.fill_lim[int64_t(run) * N + leaf]) : -1;
    int kind = EX_NONE, id = -1;
    if (valid && !dead) {
      if (s.lowest_is_hostname) {
        if (s.taint_profile) {
          int t;
          if constexpr (TS) t = sh_taint[e][prof];
          else t = b.taint_table[uni(sh_toff[e]) + prof];
          if (t >= 0) {
            kind = EX_TAINT;
            id = t;
          }
        }
        if (kind == EX_NONE) {
          const int nsel = uni(sh_nsel[e]);
          for (int k = 0; k < nsel; k++) {
            const int col = uni(sh_sel[e][2 * k]);
            int32_t v;
            if (col < kStagedLabels) {
              v = lab[0];
#pragma unroll
              for (int q = 1; q < kStagedLabels; q++) v = col == q ? lab[q] : v;
            } else {
              v = s.label_values[int64_t(col) * N + leaf];
            }
            if (v != uni(sh_sel[e][2 * k + 1])) {
              kind = EX_SELECTOR;
              break;
            }
          }
          const int sxb = uni(sh_sx[e][0]);
          if (kind == EX_NONE && sxb >= 0 && !selector_ext_match(b, sxb, uni(sh_sx[e][1]), leaf, label_at))
            kind = EX_SELECTOR;
        }
        const int ab = uni(sh_aff[e][0]);
        if (kind == EX_NONE && ab >= 0 && !affinity_match(b, ab, uni(sh_aff[e][1]), leaf, label_at)) kind = EX_AFFINITY;
      }
      if (kind == EX_NONE && outside_domain(uni(sh_aff[e][2]), uni(sh_aff[e][3]), leaf)) kind = EX_TOPOLOGY;
      if (kind == EX_NONE && lim >= 0) {
        kind = EX_RESOURCE;
        id = lim;
      }
    }
    const uint64_t selm = ballot(kind == EX_SELECTOR);
    if (lane == 0 && selm) atomicAdd(&sh_stats[e][0], __popcll(selm));
    const uint64_t affm = ballot(kind == EX_AFFINITY);
    if (lane == 0 && affm) atomicAdd(&sh_stats[e][1], __popcll(affm));
    const uint64_t domm = ballot(kind == EX_TOPOLOGY);
    if (lane == 0 && domm) atomicAdd(&sh_stats[e][2], __popcll(domm));
    uint64_t tm = ballot(kind == EX_TAINT);
    while (tm) {
      const int tid = bcast(id, __ffsll((unsigned long long)tm) - 1);
      const uint64_t mm = ballot(kind == EX_TAINT && id == tid);
      if (lane == 0) atomicAdd(&sh_stats[e][kStatFixed + tid], __popcll(mm));
      tm &= ~mm;
    }
    uint64_t rm = ballot(kind == EX_RESOURCE);
    while (rm) {
      const int rid = bcast(id, __ffsll((unsigned long long)rm) - 1);
      const uint64_t mm = ballot(kind == EX_RESOURCE && id == rid);
      if (lane == 0) atomicAdd(&sh_stats[e][kStatFixed + b.num_taints + rid], __popcll(mm));
      rm &= ~mm;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ne * b.nstat; i += kFillThreads) {
    const int e = i / b.nstat, k = i % b.nstat;
    b.fill_stats[(int64_t(e0 + e) * b.nstat_blocks + blockIdx.x) * b.nstat + k] = sh_stats[e][k];
  }
}

// Sum the per-block ExclusionStats partials of every phase-1 class; with
// class member lists, also store them for every other member of the class.
__global__ __launch_bounds__(256) void fill_stats_reduce_kernel(DevBatch b, int nblk) {

  const int f = blockIdx.x;
  const int eid = b.fill_ids[f];
  const int wv = threadIdx.x >> 6, lane = lane_id();
  for (int k = wv; k < b.nstat; k += 4) {  // one wave per statistic, lanes over the fill blocks
    const int32_t* p = b.fill_stats + int64_t(f) * nblk * b.nstat + k;
    int32_t acc = 0;
#pragma unroll 8
    for (int j = lane; j < nblk; j += kWave) acc += p[int64_t(j) * b.nstat];
    acc = wave_sum_wrap32(acc);
    const int m0 = b.cls_member_off ? b.cls_member_off[f] : 0;
    const int m1 = b.cls_member_off ? b.cls_member_off[f + 1] : 0;
    for (int m = m0 - 1 + lane; m < m1; m += kWave) {  // m0 - 1: the rep itself
      const int d = m < m0 ? eid : b.cls_members[m];
      if (k == 0) b.sel_counts[d] = acc;
      else if (k == 1) b.aff_counts[d] = acc;
      else if (k == 2) b.dom_counts[d] = acc;
      else if (k < kStatFixed + b.num_taints) b.taint_counts[int64_t(d) * b.num_taints + (k - kStatFixed)] = acc;
      else b.res_counts[int64_t(d) * b.nstat_R + (k - kStatFixed - b.num_taints)] = acc;
    }
  }
}

// ----------------------------------------------------------------------------
// K2: fillInCountsHelper, one level (parents at `level`)
// ----------------------------------------------------------------------------
// fillInCountsHelper (:1658-1719) of one parent domain p of `level` for
// class eid, one thread over the CSR children (wrapping int32 sums, min/max:
// the order of the children does not matter).
__device__ __forceinline__ void rollup_parent(const DevSnap& s, const DevBatch& b, int row, const DevEval& ev, int level,
                                              int p) {
  const bool leaderReq = (ev.flags & KUEUE_TAS_F_LEADER) != 0;
  const int cl = level + 1;
  const int32_t inner = ev.ssal[cl];
  const bool hasInner = inner != 0;
  const int cb = s.child_off[s.child_base[level] + p];
  const int ce = s.child_off[s.child_base[level] + p + 1];
  int32_t* base = ctr_base(b, row);
  const int64_t SD = s.SD;
  const int64_t SSO = ss_off(b, row, SD);
  const int coff = s.level_off[cl];
  int32_t cap = 0, slc = 0, minD = 0x7fffffff, minSD = 0x7fffffff, lead = 0;
  bool has = false;
  // children in batches of kRU: the batch's loads are issued together (one
  // memory latency per batch, not per child)
  constexpr int kRU = 8;
  for (int c0 = cb; c0 < ce; c0 += kRU) {
    int32_t vs[kRU], vss[kRU], vsw[kRU], vsswl[kRU], vls[kRU];
#pragma unroll
    for (int u = 0; u < kRU; u++) {
      const int g = coff + min(c0 + u, ce - 1);
      vs[u] = base[g];
      vss[u] = base[SSO + g];
      vsw[u] = vs[u];
      vsswl[u] = vss[u];
      vls[u] = 0;
      if (leaderReq) {
        vsw[u] = base[2 * SD + g];
        vsswl[u] = base[3 * SD + g];
        vls[u] = base[4 * SD + g];
      }
    }
#pragma unroll
    for (int u = 0; u < kRU; u++) {
    if (c0 + u >= ce) break;
    int32_t cs = vs[u];
    const int32_t css = vss[u];
    int32_t csw = vsw[u];
    const int32_t csswl = vsswl[u], cls = vls[u];
    if (hasInner) {
      cs = w_mul(go_div32(cs, inner), inner);
      csw = w_mul(go_div32(csw, inner), inner);
    }
    cap = w_add(cap, cs);
    slc = w_add(slc, css);
    if (!leaderReq || cls > 0) {
      has = true;
      minD = min(w_sub(cs, csw), minD);
      minSD = min(w_sub(css, csswl), minSD);
    }
    lead = max(cls, lead);
    }
  }
  int32_t state = cap;
  int32_t swl = has ? w_sub(cap, minD) : 0;
  int32_t sswl = has ? w_sub(slc, minSD) : 0;
  if (level == ev.slice_level) {
    slc = go_div32(state, ev.slice_size);
    sswl = go_div32(swl, ev.slice_size);
  }
  const int g = s.level_off[level] + p;
  base[g] = state;
  if (SSO) base[SD + g] = slc;
  if (leaderReq) {
    base[2 * SD + g] = swl;
    base[3 * SD + g] = sswl;
    base[4 * SD + g] = lead;
  }
}

__global__ __launch_bounds__(256) void rollup_level_kernel(DevSnap s, DevBatch b, int level) {
  if (int(blockIdx.y) >= b.nfill) return;
  const int eid = b.fill_ids[blockIdx.y];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= s.level_size[level]) return;
  rollup_parent(s, b, int(blockIdx.y), b.evals[eid], level, p);
}

// Same reduction with one wave per parent: lanes stride over the CSR children
// (coalesced reads), then a wave reduction.  Used when the mean fan-out is
// large (e.g. leaves -> racks).  kParentsPerWave parents per wave.
constexpr int kParentsPerWave = 4;
__global__ __launch_bounds__(256) void rollup_level_wave_kernel(DevSnap s, DevBatch b, int level) {
  if (int(blockIdx.y) >= b.nfill) return;
  const int eid = b.fill_ids[blockIdx.y];
  const DevEval& ev = b.evals[eid];
  const bool leaderReq = (ev.flags & KUEUE_TAS_F_LEADER) != 0;
  const int cl = level + 1;
  const int32_t inner = ev.ssal[cl];
  const bool hasInner = inner != 0;
  int32_t* base = ctr_base(b, int(blockIdx.y));  // the class's row: its fill position
  const int64_t SD = s.SD;
  const int64_t SSO = ss_off(b, int(blockIdx.y), SD);
  const int coff = s.level_off[cl];
  const int lane = lane_id();
  const int p0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kParentsPerWave;
  for (int j = 0; j < kParentsPerWave; j++) {
    const int p = p0 + j;
    if (p >= s.level_size[level]) return;
    const int cb = s.child_off[s.child_base[level] + p];
    const int ce = s.child_off[s.child_base[level] + p + 1];
    int32_t cap = 0, slc = 0, minD = 0x7fffffff, minSD = 0x7fffffff, lead = 0;
    int has = 0;
    for (int c = cb + lane; c < ce; c += kWave) {
      const int g = coff + c;
      int32_t cs = base[g];
      int32_t css = base[SSO + g];
      int32_t csw = cs, csswl = css, cls = 0;
      if (leaderReq) {
        csw = base[2 * SD + g];
        csswl = base[3 * SD + g];
        cls = base[4 * SD + g];
      }
      if (hasInner) {
        cs = w_mul(go_div32(cs, inner), inner);
        csw = w_mul(go_div32(csw, inner), inner);
      }
      cap = w_add(cap, cs);
      slc = w_add(slc, css);
      if (!leaderReq || cls > 0) {
        has = 1;
        minD = min(w_sub(cs, csw), minD);
        minSD = min(w_sub(css, csswl), minSD);
      }
      lead = max(cls, lead);
    }
#pragma unroll
    for (int m = 1; m <= 32; m <<= 1) {
      cap = w_add(cap, xor_lane(cap, m));
      slc = w_add(slc, xor_lane(slc, m));
      minD = min(minD, xor_lane(minD, m));
      minSD = min(minSD, xor_lane(minSD, m));
      lead = max(lead, xor_lane(lead, m));
      has |= xor_lane(has, m);
    }
    if (lane == 0) {
      int32_t state = cap;
      int32_t swl = has ? w_sub(cap, minD) : 0;
      int32_t sswl = has ? w_sub(slc, minSD) : 0;
      if (level == ev.slice_level) {
        slc = go_div32(state, ev.slice_size);
        sswl = go_div32(swl, ev.slice_size);
      }
      const int g = s.level_off[level] + p;
      base[g] = state;
      if (SSO) base[SD + g] = slc;
      if (leaderReq) {
        base[2 * SD + g] = swl;
        base[3 * SD + g] = sswl;
        base[4 * SD + g] = lead;
      }
    }
  }
}

// Per phase-1 class and level above the leaves: the maximum sliceState, the
// sliceState of the first domain of sortedDomainsWithLeader (:1511-1535) for
// a leaderless eval.  find_level skips a level whose maximum cannot hold
// the eval's slices without scanning it (required: notFitMessage's count,
// :1271-1274; preferred: the recursion to the level above, :1275-1277).
// One block per (class, level): the level's sliceState read as int4 (levels
// start 16-byte aligned), every load of a thread issued before the reduction.
__global__ __launch_bounds__(256) void level_max_kernel(DevSnap s, DevBatch b) {
  __shared__ int32_t red[4];
  const int row = blockIdx.x;  // the class's fill position
  const int l = blockIdx.y;
  const int D = s.level_size[l];
  const int4* ss4 = reinterpret_cast<const int4*>(ctr_base(b, row) + ss_off(b, row, s.SD) + s.level_off[l]);
  const int nq = (D + 3) / 4;
  int32_t m = INT32_MIN;
  constexpr int U = 8;
  for (int q0 = 0; q0 < nq; q0 += U * 256) {
    int4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ss4[min(q0 + u * 256 + int(threadIdx.x), nq - 1)];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int q = q0 + u * 256 + int(threadIdx.x);
      if (q < nq) {
        const int32_t e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (4 * q + k < D) m = max(m, e[k]);
      }
    }
  }
  m = group_reduce(m, 64, OpMax());
  if (lane_id() == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) b.level_max[int64_t(row) * kMaxLevels + l] = max(max(red[0], red[1]), max(red[2], red[3]));
}

// The top of the tree in one launch (fillInCountsHelper :1658-1719 for
// levels `level` .. 0, plus the level maxima findLevelWithFitDomains' skip
// reads): the grid rolls level `level` up, one wave per parent as
// rollup_level_wave_kernel, and records the maximum sliceState of the
// children it reads (level + 1, when that is not the leaf level) with one
// atomicMax per block; the last block of each class to finish (a release
// fence and a per-class arrival counter) then rolls up levels level-1 .. 0
// itself — a few hundred parents — reading its siblings' parents through
// L2, and writes those levels' maxima.  One launch instead of one per level
// plus level_max_kernel.  b.level_max rows start at INT32_MIN and the
// counters at 0 (host staging upload).
__device__ __forceinline__ int32_t load_l2_i32(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool L2>
__device__ __forceinline__ void rollup_parent_wave(const DevSnap& s, int32_t* base, int64_t SSO, const DevEval& ev,
                                                   bool leaderReq, int level, int p, int32_t* cmax) {
  const int cl = level + 1;
  const int32_t inner = ev.ssal[cl];
  const bool hasInner = inner != 0;
  const int64_t SD = s.SD;
  const int coff = s.level_off[cl];
  const int lane = lane_id();
  const int cb = s.child_off[s.child_base[level] + p];
  const int ce = s.child_off[s.child_base[level] + p + 1];
  auto ld = [&](int64_t o) { return L2 ? load_l2_i32(base + o) : base[o]; };
  int32_t cap = 0, slc = 0, minD = 0x7fffffff, minSD = 0x7fffffff, lead = 0, mx = INT32_MIN;
  int has = 0;
  for (int c = cb + lane; c < ce; c += kWave) {
    const int g = coff + c;
    int32_t cs = ld(g);
    const int32_t css = ld(SSO + g);
    int32_t csw = cs, csswl = css, cls = 0;
    if (leaderReq) {
      csw = ld(2 * SD + g);
      csswl = ld(3 * SD + g);
      cls = ld(4 * SD + g);
    }
    mx = max(mx, css);
    if (hasInner) {
      cs = w_mul(go_div32(cs, inner), inner);
      csw = w_mul(go_div32(csw, inner), inner);
    }
    cap = w_add(cap, cs);
    slc = w_add(slc, css);
    if (!leaderReq || cls > 0) {
      has = 1;
      minD = min(w_sub(cs, csw), minD);
      minSD = min(w_sub(css, csswl), minSD);
    }
    lead = max(cls, lead);
  }
#pragma unroll
  for (int m = 1; m <= 32; m <<= 1) {
    cap = w_add(cap, xor_lane(cap, m));
    slc = w_add(slc, xor_lane(slc, m));
    minD = min(minD, xor_lane(minD, m));
    minSD = min(minSD, xor_lane(minSD, m));
    lead = max(lead, xor_lane(lead, m));
    has |= xor_lane(has, m);
    mx = max(mx, xor_lane(mx, m));
  }
  *cmax = max(*cmax, mx);
  if (lane == 0) {
    const int32_t state = cap;
    const int32_t swl = has ? w_sub(cap, minD) : 0;
    int32_t sswl = has ? w_sub(slc, minSD) : 0;
    if (level == ev.slice_level) {
      slc = go_div32(state, ev.slice_size);
      sswl = go_div32(swl, ev.slice_size);
    }
    const int g = s.level_off[level] + p;
    base[g] = state;
    if (SSO) base[SD + g] = slc;
    if (leaderReq) {
      base[2 * SD + g] = swl;
      base[3 * SD + g] = sswl;
      base[4 * SD + g] = lead;
    }
  }
}

__global__ __launch_bounds__(256) void rollup_top_kernel(DevSnap s, DevBatch b, int level, int32_t* arrivals) {
  __shared__ int32_t red[4];
  __shared__ int32_t last;
  const int row = blockIdx.y;  // the class's fill position
  const int eid = b.fill_ids[row];
  const DevEval& ev = b.evals[eid];
  const bool leaderReq = (ev.flags & KUEUE_TAS_F_LEADER) != 0;
  int32_t* base = ctr_base(b, row);
  const int64_t SSO = ss_off(b, row, s.SD);
  const int wv = threadIdx.x >> 6;
  int32_t cmax = INT32_MIN;
  const int p0 = (blockIdx.x * 4 + wv) * kParentsPerWave;
  for (int j = 0; j < kParentsPerWave; j++) {
    const int p = p0 + j;
    if (p < s.level_size[level]) rollup_parent_wave<false>(s, base, SSO, ev, leaderReq, level, p, &cmax);
  }
  if (lane_id() == 0) red[wv] = cmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int32_t m = max(max(red[0], red[1]), max(red[2], red[3]));
    if (level + 1 < s.L - 1 && b.level_max) atomicMax(&b.level_max[int64_t(row) * kMaxLevels + level + 1], m);
    __threadfence();  // this block's parents reach L2 before its arrival counts
    last = atomicAdd(&arrivals[row], 1) == int(gridDim.x) - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (int l = level - 1; l >= -1; l--) {
    // l >= 0: roll level l up from level l + 1; the maximum of level l + 1 comes with the reads
    int32_t lm = INT32_MIN;
    if (l >= 0) {
      for (int p = wv; p < s.level_size[l]; p += 4) rollup_parent_wave<true>(s, base, SSO, ev, leaderReq, l, p, &lm);
    } else {  // level 0's own maximum
      const int32_t* ss = base + SSO + s.level_off[0];
      for (int i = threadIdx.x; i < s.level_size[0]; i += 256) lm = max(lm, load_l2_i32(ss + i));
      lm = group_reduce(lm, 64, OpMax());
    }
    if (lane_id() == 0) red[wv] = lm;
    __syncthreads();
    if (threadIdx.x == 0 && b.level_max && l + 1 < s.L - 1)
      b.level_max[int64_t(row) * kMaxLevels + l + 1] = max(max(red[0], red[1]), max(red[2], red[3]));
    __threadfence_block();
    __syncthreads();
  }
}

// The roll-up's small top levels and every level's maximum sliceState in one
// launch: one block per class rolls up levels top .. 0 (a few parents each,
// one wave per parent, levels in order with a block barrier between), then
// streams each level l < L-1's sliceState row for its maximum (findLevel's
// level scans: b.level_max).  Replaces the per-level launches of those
// levels and level_max_kernel.
constexpr int kTailParents = 16;  // levels of at most this many domains go to rollup_tail_kernel
__global__ __launch_bounds__(256) void rollup_tail_kernel(DevSnap s, DevBatch b, int top) {
  __shared__ int32_t red[4];
  const int row = blockIdx.x;  // the class's fill position
  const DevEval& ev = b.evals[b.fill_ids[row]];
  const bool leaderReq = (ev.flags & KUEUE_TAS_F_LEADER) != 0;
  int32_t* base = ctr_base(b, row);
  const int64_t SSO = ss_off(b, row, s.SD);
  const int wv = threadIdx.x >> 6;
  for (int l = top; l >= 0; l--) {
    int32_t unused = INT32_MIN;
    for (int p = wv; p < s.level_size[l]; p += 4) rollup_parent_wave<true>(s, base, SSO, ev, leaderReq, l, p, &unused);
    __threadfence_block();
    __syncthreads();
  }
  if (!b.level_max) return;
  for (int l = 0; l + 1 < s.L; l++) {
    const int32_t* ss = base + SSO + s.level_off[l];
    int32_t m = INT32_MIN;
    if (l <= top) {  // this block's own parents: through L2
      for (int i = threadIdx.x; i < s.level_size[l]; i += 256) m = max(m, load_l2_i32(ss + i));
    } else {  // written by earlier launches: int4 loads (levels start 16-byte aligned), all issued first
      const int D = s.level_size[l];
      const int nq = (D + 3) / 4;
      const int4* ss4 = reinterpret_cast<const int4*>(ss);
      constexpr int U = 4;
      for (int q0 = 0; q0 < nq; q0 += U * 256) {
        int4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ss4[min(q0 + u * 256 + int(threadIdx.x), nq - 1)];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int q = q0 + u * 256 + int(threadIdx.x);
          const int32_t e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (q < nq && 4 * q + k < D) m = max(m, e[k]);
        }
      }
    }
    m = group_reduce(m, 64, OpMax());
    if (lane_id() == 0) red[wv] = m;
    __syncthreads();
    if (threadIdx.x == 0) b.level_max[int64_t(row) * kMaxLevels + l] = max(max(red[0], red[1]), max(red[2], red[3]));
    __syncthreads();
  }
}

// Leaf-level selection partials for evals whose requested level is the leaf
// level: per 64-leaf wave, the reductions findLevelWithFitDomains needs
// (:1244-1270): first/last sortedDomainsWithLeader key, LFC first fit,
// BestFit best fit and the minimum sliceState.  Reads the leaf counters.
__global__ __launch_bounds__(kFillThreads) void leaf_partials_kernel(DevSnap s, DevBatch b, const int32_t* ids,
                                                                    int nids) {
  const int e0 = blockIdx.y * kEvalsPerBlock;
  const int ne = min(kEvalsPerBlock, nids - e0);
  const int leaf = blockIdx.x * kFillThreads + threadIdx.x;
  const bool valid = leaf < s.N;
  const int gleaf = s.level_off[s.L - 1] + leaf;
  const int lane = lane_id();
  const int64_t SD = s.SD;
  for (int e = 0; e < ne; e++) {
    const int eid = uni(ids[e0 + e]);
    const DevEval& ev = b.evals[eid];
    const uint32_t flags = uint32_t(uni(int32_t(ev.flags)));
    const bool leader = (flags & KUEUE_TAS_F_LEADER) != 0;
    const bool lfc = (flags & KUEUE_TAS_F_LFC) != 0;
    const int32_t sliceCount = go_div32(uni(ev.count), uni(ev.slice_size));
    const int32_t* base = ctr_base(b, b.rep_of[eid]);
    const int64_t SSO = ss_off(b, b.rep_of[eid], SD);
    int32_t state = 0, ss = 0, swl = 0, sswl = 0, ls = 0;
    if (valid) {
      state = base[gleaf];
      ss = base[SSO + gleaf];
      swl = state;
      sswl = ss;
      if (leader) {
        swl = base[2 * SD + gleaf];
        sswl = base[3 * SD + gleaf];
        ls = base[4 * SD + gleaf];
      }
    }
    Key k = key_wl(lfc, ls, sswl, swl, leaf);
    Key top = valid ? k : key_max();
    Key inv = valid ? Key{~k.hi, ~k.lo} : key_max();
    Key lf = (valid && ss >= sliceCount) ? k : key_max();
    const int32_t st = leader ? sswl : ss;
    uint32_t bst = (valid && st >= sliceCount) ? s_asc(st) : ~0u;
    uint32_t mss = valid ? s_asc(ss) : ~0u;
    top = wave_min_key(top);
    inv = wave_min_key(inv);
    lf = wave_min_key(lf);
    bst = uint32_t(wave_min_u64(bst));
    mss = uint32_t(wave_min_u64(mss));
    Key bk = (valid && st >= sliceCount && s_asc(st) == bst) ? k : key_max();
    bk = wave_min_key(bk);
    if (lane == 0) {
      LeafPartial pt;
      pt.top = top;
      pt.last = Key{~inv.hi, ~inv.lo};
      pt.lfcfit = lf;
      pt.bfkey = bk;
      pt.bfst = bst;
      pt.minss = int32_t(mss ^ 0x80000000u);
      pt.pad[0] = pt.pad[1] = 0;
      b.partials[int64_t(e0 + e) * b.nblk + blockIdx.x * (kFillThreads / kWave) + (threadIdx.x >> 6)] = pt;
    }
  }
}

// Replicate the exclusion stats of a class representative to another member
// of its class (global-atomic stats path; the counters are shared: every
// member reads its class's row, DevBatch::rep_of).  pairs: (rep, ~member).
__global__ __launch_bounds__(256) void replicate_kernel(DevSnap s, DevBatch b, const int32_t* pairs, int npairs) {
  const int pi = blockIdx.y;
  if (pi >= npairs) return;
  const int src = pairs[2 * pi], dst = ~pairs[2 * pi + 1];
  if (blockIdx.x == 0) {
    for (int i = threadIdx.x; i < b.num_taints; i += blockDim.x)
      b.taint_counts[int64_t(dst) * b.num_taints + i] = b.taint_counts[int64_t(src) * b.num_taints + i];
    for (int i = threadIdx.x; i < s.R; i += blockDim.x)
      b.res_counts[int64_t(dst) * s.R + i] = b.res_counts[int64_t(src) * s.R + i];
    if (threadIdx.x == 0) {
      b.sel_counts[dst] = b.sel_counts[src];
      b.aff_counts[dst] = b.aff_counts[src];
      b.dom_counts[dst] = b.dom_counts[src];
    }
  }
}


// ----------------------------------------------------------------------------
// LeastFreeCapacity leaf tables (see LfcJob in tas_internal.h)
// ----------------------------------------------------------------------------
// Per (class slot, chunk of kLfcChunk leaves): counts of each leaf value
// (sliceState == state for fast-LFC classes) and the sum of the values that
// land in the overflow bin.
__global__ __launch_bounds__(256) void lfc_hist_kernel(DevSnap s, DevBatch b) {
  __shared__ uint32_t h[kLfcBins];
  __shared__ unsigned long long ovs;
  const int slot = blockIdx.y, chunk = blockIdx.x;
  for (int i = threadIdx.x; i < kLfcBins; i += blockDim.x) h[i] = 0;
  if (threadIdx.x == 0) ovs = 0;
  __syncthreads();
  const int32_t* v = ctr_base(b, b.lfc_rep[slot]) + ss_off(b, b.lfc_rep[slot], s.SD) +
                     s.level_off[s.L - 1];
  const int lo = chunk * kLfcChunk, hi = min(s.N, lo + kLfcChunk);
  uint64_t mysum = 0;
  const int lane = lane_id();
  // every load of the chunk issued before the first bin loop (the loop's LDS
  // atomics would otherwise order each load after the previous group's work)
  constexpr int kPer = kLfcChunk / 256;  // launched with 256 threads
  int32_t xs[kPer];
#pragma unroll
  for (int u = 0; u < kPer; u++) {
    const int i = lo + u * 256 + int(threadIdx.x);
    xs[u] = i < hi ? v[i] : 0;
  }
#pragma unroll
  for (int u = 0; u < kPer; u++) {  // wave-uniform trip count
    const int i = lo + u * 256 + int(threadIdx.x);
    const bool act = i < hi;
    const int32_t x = xs[u];
    const bool over = x >= kLfcBins - 1 || x < 0;  // x < 0 cannot occur at a leaf (CountIn clamps at 0)
    if (act && over) mysum += uint64_t(int64_t(x));
    const int bin = over ? kLfcBins - 1 : x;
    // one LDS atomic per distinct bin of the wave (leaf values are few and repetitive)
    uint64_t pending = ballot(act);
    while (pending) {
      const int src = __ffsll((unsigned long long)pending) - 1;
      const int b0 = bcast(bin, src);
      const uint64_t m = ballot(act && bin == b0);
      if (lane == src) atomicAdd(&h[b0], uint32_t(__popcll(m)));
      pending &= ~m;
    }
  }
  // the chunk's values as bytes, min(v, 255), for lfc_emit_kernel: a greedy
  // threshold below 255 needs no wider value (a quarter of the emit's reads)
  {
    uint8_t* u8 = b.lfc_u8 + int64_t(slot) * b.lfc_nchunks * kLfcChunk + int64_t(lo);
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int32_t x = xs[u];
      u8[u * 256 + int(threadIdx.x)] = uint8_t(x < 0 ? 0 : x > 255 ? 255 : x);
    }
  }
  mysum = uint64_t(wave_sum_i64(int64_t(mysum)));
  if (lane == 0 && mysum) atomicAdd(&ovs, (unsigned long long)mysum);
  __syncthreads();
  uint32_t* out = b.lfc_ch + (int64_t(slot) * b.lfc_nchunks + chunk) * kLfcBins;
  for (int i = threadIdx.x; i < kLfcBins; i += blockDim.x) out[i] = h[i];
  if (threadIdx.x == 0) b.lfc_ovs[int64_t(slot) * b.lfc_nchunks + chunk] = ovs;
}

// Per slot: exclusive prefix of every bin over the chunks, totals, overflow sum.
__global__ __launch_bounds__(kLfcBins) void lfc_total_kernel(DevBatch b) {
  const int slot = blockIdx.x, bin = threadIdx.x;
  if (slot == 0 && bin == 0) *b.lfc_nitems = 0;  // select appends the emit work items after this kernel
  const int64_t base = int64_t(slot) * b.lfc_nchunks;
  constexpr int U = 16;  // chunk counts loaded ahead of the running prefix
  uint32_t acc = 0;
  for (int c0 = 0; c0 < b.lfc_nchunks; c0 += U) {
    uint32_t v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = c0 + u < b.lfc_nchunks ? b.lfc_ch[(base + c0 + u) * kLfcBins + bin] : 0u;
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (c0 + u < b.lfc_nchunks) b.lfc_cp[(base + c0 + u) * kLfcBins + bin] = acc;
      acc += v[u];
    }
  }
  b.lfc_tot[int64_t(slot) * kLfcBins + bin] = acc;
  if (bin < kWave) {
    uint64_t o = 0;
    for (int c = bin; c < b.lfc_nchunks; c += kWave) o += b.lfc_ovs[base + c];
    o = uint64_t(wave_sum_i64(int64_t(o)));
    if (bin == 0) b.lfc_ovtot[slot] = o;
  }
}

// ----------------------------------------------------------------------------
// K3: phase 2, one wave per eval
// ----------------------------------------------------------------------------
enum Field : int { F_STATE = 0, F_SLICE = 1, F_SWL = 2, F_SSWL = 3, F_LS = 4 };

// Profiling build (-DKTAS_PROFILE=1, libkueue_tas_prof.so): per-eval ticks
// of the select kernel's phases into DevBatch::prof (diagnostics only).
#ifndef KTAS_PROFILE
#define KTAS_PROFILE 0
#endif
enum ProfCat : int {
  P_LDS_SORT = 0, P_THRESHOLD, P_GATHER, P_EMIT, P_WALK, P_GLOBAL_SORT, P_UPDATE, P_FIND,
  P_TW_KEYS, P_TW_SELECT, P_TW_EMIT, P_SETUP, P_FINAL,
  P_FW_PARENTS, P_FW_CHILDREN, P_FW_LOADS, P_FW_SELECT, P_FW_EMIT, P_WS_FILTER, P_SEL_EMIT, P_NCAT
};

// The select path's snapshot descriptor, in the constant address space: the
// walk's helpers (not inlined) read its fields with scalar loads from a known
// address.  A pointer to the by-value kernel argument instead made the
// compiler copy the argument into scratch and chase two dependent scratch
// loads (Wave -> descriptor -> field) per access.  Written by the host on the
// batch's stream before the select launches (kueue_tas_eval_batch holds a
// process-wide lock, so contexts do not interleave their descriptors).
__constant__ DevSnap g_select_snap;

// One (leaf, count) entry of an assignment (buildAssignment :1490-1501) as
// one 8-byte store into the eval's region of pinned host memory, plus the
// leaf's tag (kueue_tas_snapshot_set_leaf_tags: the host's Values address)
// at the same pair index of the tag region when tags are on.
__device__ __forceinline__ void put_entry(int32_t* ent, int pos, int32_t leaf, int32_t count) {
  *reinterpret_cast<int2*>(ent + 2 * pos) = make_int2(leaf, count);
  const uint64_t* lt = g_select_snap.leaf_tag;
  if (lt) g_select_snap.tag_out[((ent - g_select_snap.ent_base) >> 1) + pos] = lt[leaf];
}

struct Wave {
  const DevEval* ev;
  int eid;
  bool leader, lfc, bf, unconstrained;
  const int32_t* ctr;  // phase-1 counters of this eval's class (shared, read-only here)
  const uint64_t* rack_pos;  // the class's positive-child masks of level L-2 (or null)
  int32_t* ov;         // private overlay [5][SD]
  int32_t* tag;        // [SD] overlay ownership tags
  int32_t my_tag;
  bool dirty;
  int64_t SD;
  int64_t ssoff;  // the sliceState field's offset in ctr: SD, or 0 for a simple class (ss_off)
  Key* lds;        // per-wave LDS buffer (list_cap keys; lds_bytes in all)
  int cap;
  int lds_bytes;
  int32_t* listA;  // global scratch lists (lcap entries each)
  int32_t* listB;
  int32_t* listC;
  int32_t* listD;
  Key* gkeys;      // global scratch keys (lcap entries)
  Key* gkeys2;
  int lcap;
  bool overflow;
  const LeafPartial* partials;  // leaf-level partial reductions of this eval (or null)
  int nblk;
  const int32_t* level_max;     // level_max_kernel row of this eval's class (or null)
#if KTAS_PROFILE
  uint64_t prof[P_NCAT];
#endif

  // Phase-2 mutations go to a private copy-on-write overlay (ov, tag ==
  // my_tag marks the domains it holds) so evals of one phase-1 class share
  // the class counters `ctr` read-only: no per-eval replication.  Until the
  // first mutation (`dirty`, wave-uniform: findLevelWithFitDomains never
  // mutates) reads go straight to ctr.
  __device__ int32_t get(Field f, int g) const {
    if (!leader) {
      if (f == F_LS) return 0;
      if (f == F_SWL) f = F_STATE;
      if (f == F_SSWL) f = F_SLICE;
    }
    const int64_t o = int64_t(f) * SD + g;
    const int64_t co = (f == F_SLICE ? ssoff : int64_t(f) * SD) + g;
    if (!dirty) return ctr[co];
    const int32_t shared = ctr[co], own = ov[o];
    return tag[g] == my_tag ? own : shared;
  }
  // first write of a domain: copy its counters into the overlay
  __device__ void own(int g) {
    if (tag[g] != my_tag) {
      const int nf = leader ? 5 : 2;
      for (int f = 0; f < nf; f++) ov[int64_t(f) * SD + g] = ctr[(f == F_SLICE ? ssoff : int64_t(f) * SD) + g];
      tag[g] = my_tag;
    }
  }
  // Stored by every lane (see file header).
  __device__ void set(Field f, int g, int32_t v) {
    if (!leader) {
      if (f == F_LS || f == F_SWL || f == F_SSWL) return;
    }
    dirty = true;
    own(g);
    ov[int64_t(f) * SD + g] = v;
  }
  // Lane-private first write of a domain a leaderless walk has just read clean
  // (non-leader evals hold two fields): stores only, no ownership check.
  __device__ void set_walked(int g, int32_t state, int32_t slice) {
    ov[int64_t(F_STATE) * SD + g] = state;
    ov[int64_t(F_SLICE) * SD + g] = slice;
    tag[g] = my_tag;
  }
  // Stored by one lane for a domain only it handles in a lane-parallel pass;
  // readers on other lanes come after a fence (callers have set dirty).
  __device__ void set_lane(Field f, int g, int32_t v) {
    if (!leader && (f == F_LS || f == F_SWL || f == F_SSWL)) return;
    this->own(g);
    ov[g + int64_t(f) * SD] = v;  // lane-private
  }
  // Reads of domains this eval has not mutated (the children a walk is
  // about to sort: every domain has one parent and is walked once).
  __device__ int32_t get_clean(Field f, int g) const {
    if (!leader) {
      if (f == F_LS) return 0;
      if (f == F_SWL) f = F_STATE;
      if (f == F_SSWL) f = F_SLICE;
    }
    return ctr[(f == F_SLICE ? ssoff : int64_t(f) * SD) + g];
  }
  __device__ Key kplain_clean(int g) const {
    int idx = g - g_select_snap.level_off[level_of(g)];
    return key_plain(lfc, get_clean(F_SLICE, g), get_clean(F_STATE, g), idx);
  }
  __device__ Key kplain(int g) const {
    int idx = g - g_select_snap.level_off[level_of(g)];
    return key_plain(lfc, get(F_SLICE, g), get(F_STATE, g), idx);
  }
  __device__ int level_of(int g) const {
    int l = 0;
    while (l + 1 < g_select_snap.L && g >= g_select_snap.level_off[l + 1]) l++;
    return l;
  }
};

struct ProfScope {
#if KTAS_PROFILE
  uint64_t* slot;
  uint64_t t0;
  __device__ ProfScope(Wave& w, int cat) : slot(&w.prof[cat]), t0(wall_clock64()) {}
  __device__ ~ProfScope() { *slot += wall_clock64() - t0; }
#else
  __device__ ProfScope(Wave&, int) {}
#endif
};

// ---- LDS bitonic sort of m keys (one wave) ----
// Each stage visits the m/2 compare-exchange pairs (lane p handles pair p:
// i = p with a zero bit inserted at `stride`, j = i | stride), kSortU pairs
// per lane in flight, so the LDS round trips of one stage overlap.
constexpr int kSortU = 4;
__device__ void lds_sort(Key* k, int n, int lane) {
  int m = 1;
  while (m < n) m <<= 1;
  for (int i = n + lane; i < m; i += kWave) k[i] = key_max();
  wave_sync();
  const int half = m >> 1;
  for (int size = 2; size <= m; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p0 = 0; p0 < half; p0 += kSortU * kWave) {
        Key a[kSortU], c[kSortU];
        int ii[kSortU];
#pragma unroll
        for (int u = 0; u < kSortU; u++) {
          const int p = min(p0 + u * kWave + lane, half - 1);
          const int i = ((p & ~(stride - 1)) << 1) | (p & (stride - 1));
          ii[u] = i;
          a[u] = k[i];
          c[u] = k[i | stride];
        }
#pragma unroll
        for (int u = 0; u < kSortU; u++) {
          const int p = p0 + u * kWave + lane;
          const int i = ii[u];
          const bool asc = (i & size) == 0;
          if (p < half && key_lt(c[u], a[u]) == asc) {
            k[i] = c[u];
            k[i | stride] = a[u];
          }
        }
      }
      wave_sync();
    }
  }
}

// ---- global merge sort of n keys in `a` (tmp same size); result in a ----
__device__ void global_sort(Wave& w, Key* a, Key* tmp, int n) {
  ProfScope prof_scope_(w, P_GLOBAL_SORT);
  const int lane = lane_id();
  const int run = w.cap;
  // sort runs of `run` in LDS
  for (int r0 = 0; r0 < n; r0 += run) {
    int m = min(run, n - r0);
    for (int i = lane; i < m; i += kWave) w.lds[i] = a[r0 + i];
    wave_sync();
    {
      ProfScope ps_(w, P_LDS_SORT);
      lds_sort(w.lds, m, lane);
    }
    for (int i = lane; i < m; i += kWave) a[r0 + i] = w.lds[i];
    wave_sync();
  }
  Key* src = a;
  Key* dst = tmp;
  for (int width = run; width < n; width <<= 1) {
    for (int r0 = 0; r0 < n; r0 += 2 * width) {
      int aN = min(width, n - r0);
      int bN = min(width, max(0, n - r0 - width));
      const Key* A = src + r0;
      const Key* B = src + r0 + aN;
      for (int i = lane; i < aN; i += kWave) {  // rank in B: lower_bound
        int lo = 0, hi = bN;
        while (lo < hi) {
          int mid = (lo + hi) >> 1;
          if (key_lt(B[mid], A[i])) lo = mid + 1;
          else hi = mid;
        }
        dst[r0 + i + lo] = A[i];
      }
      for (int j = lane; j < bN; j += kWave) {  // rank in A: upper_bound
        int lo = 0, hi = aN;
        while (lo < hi) {
          int mid = (lo + hi) >> 1;
          if (key_le(A[mid], B[j])) lo = mid + 1;
          else hi = mid;
        }
        dst[r0 + j + lo] = B[j];
      }
    }
    wave_fence();
    Key* t = src;
    src = dst;
    dst = t;
  }
  if (src != a) {
    for (int i = lane; i < n; i += kWave) a[i] = src[i];
    wave_fence();
  }
}

// ---- sequences walked by updateCountsToMinimumGeneric ----
// Explicit order: domain gids at positions [0, n) (LDS keys or a global list).
struct SeqLds {
  Wave* w;
  int n, level_off, pos;
  __device__ int size() const { return n; }
  __device__ bool done() const { return pos >= n; }
  __device__ int cur() const { return level_off + int(uint32_t(w->lds[pos].lo)); }
  __device__ void next() { pos++; }
  __device__ int at(int p) const { return level_off + int(uint32_t(w->lds[p].lo)); }
  // findBestFitDomainBy over domains[pos:] (:1216-1231)
  __device__ int bestfit(int32_t needed, Field f) const {
    int g0 = cur();
    if (w->get(f, g0) < needed) return g0;
    uint64_t best = ~0ull;
    for (int p = pos + lane_id(); p < n; p += kWave) {
      int32_t st = w->get(f, at(p));
      if (st >= needed) {
        uint64_t k = (uint64_t(s_asc(st)) << 32) | uint32_t(p);
        best = k < best ? k : best;
      }
    }
    best = wave_min_u64(best);
    return at(int(uint32_t(best)));
  }
};

struct SeqList {
  Wave* w;
  const int32_t* g;
  int n, pos;
  __device__ int size() const { return n; }
  __device__ bool done() const { return pos >= n; }
  __device__ int cur() const { return g[pos]; }
  __device__ void next() { pos++; }
  __device__ int bestfit(int32_t needed, Field f) const {
    int g0 = cur();
    if (w->get(f, g0) < needed) return g0;
    uint64_t best = ~0ull;
    for (int p = pos + lane_id(); p < n; p += kWave) {
      int32_t st = w->get(f, g[p]);
      if (st >= needed) {
        uint64_t k = (uint64_t(s_asc(st)) << 32) | uint32_t(p);
        best = k < best ? k : best;
      }
    }
    best = wave_min_u64(best);
    return g[int(uint32_t(best))];
  }
};

// Explicit order from keys sorted in global memory (lists longer than the LDS).
struct SeqKeys {
  Wave* w;
  const Key* k;
  int n, level_off, pos;
  __device__ bool done() const { return pos >= n; }
  __device__ int at(int p) const { return level_off + int(uint32_t(k[p].lo)); }
  __device__ int cur() const { return at(pos); }
  __device__ void next() { pos++; }
  __device__ int bestfit(int32_t needed, Field f) const {
    int g0 = cur();
    if (w->get(f, g0) < needed) return g0;
    uint64_t best = ~0ull;
    for (int p = pos + lane_id(); p < n; p += kWave) {
      int32_t st = w->get(f, at(p));
      if (st >= needed) {
        uint64_t kk = (uint64_t(s_asc(st)) << 32) | uint32_t(p);
        best = kk < best ? kk : best;
      }
    }
    best = wave_min_u64(best);
    return at(int(uint32_t(best)));
  }
};

// Lazy sorted iteration over n materialized (unsorted) keys of one level.
struct SeqLazy {
  Wave* w;
  const Key* k;
  int n, level_off;
  Key curk;
  bool valid;
  __device__ void find_next(bool first) {
    Key best = key_max();
    for (int i = lane_id(); i < n; i += kWave) {
      Key x = k[i];
      if ((first || key_lt(curk, x)) && key_lt(x, best)) best = x;
    }
    best = wave_min_key(best);
    valid = !(best.hi == ~0ull && best.lo == ~0ull);
    curk = best;
  }
  __device__ void start() { find_next(true); }
  __device__ bool done() const { return !valid; }
  __device__ int cur() const { return level_off + int(uint32_t(curk.lo)); }
  __device__ void next() { find_next(false); }
  __device__ int bestfit(int32_t needed, Field f) const {
    int g0 = cur();
    if (w->get(f, g0) < needed) return g0;
    uint32_t bst = ~0u;
    for (int i = lane_id(); i < n; i += kWave) {
      Key x = k[i];
      if (key_le(curk, x)) {
        int32_t st = w->get(f, level_off + int(uint32_t(x.lo)));
        if (st >= needed && s_asc(st) < bst) bst = s_asc(st);
      }
    }
    bst = uint32_t(wave_min_u64(uint64_t(bst)));
    Key best = key_max();
    for (int i = lane_id(); i < n; i += kWave) {
      Key x = k[i];
      if (key_le(curk, x) && key_lt(x, best)) {
        int32_t st = w->get(f, level_off + int(uint32_t(x.lo)));
        if (st >= needed && s_asc(st) == bst) best = x;
      }
    }
    best = wave_min_key(best);
    return level_off + int(uint32_t(best.lo));
  }
};

// consumeWithLeadersGeneric (:1348-1403)
template <class Seq>
__device__ int consume_with_leaders(Wave& w, Seq& seq, int domain, int32_t* remP, int32_t* remL, Field wl, Field pr,
                                    int32_t sliceSize, bool slices, bool* completed) {
  if (w.bf && w.get(wl, domain) >= *remP && w.get(F_LS, domain) >= *remL) {
    if (slices) {
      domain = seq.bestfit(*remP, *remL > 0 ? F_SSWL : F_SLICE);
      wl = F_SSWL;
      pr = F_SLICE;
    } else {
      domain = seq.bestfit(*remP, *remL > 0 ? F_SWL : F_STATE);
      wl = F_SWL;
      pr = F_STATE;
    }
  }
  if (w.get(wl, domain) >= *remP && w.get(F_LS, domain) >= *remL) {
    w.set(pr, domain, *remP);
    w.set(F_LS, domain, *remL);
    w.set(F_STATE, domain, w_mul(*remP, sliceSize));
    *completed = true;
    return domain;
  }
  if (slices) {
    if (w.get(wl, domain) > *remP) w.set(wl, domain, *remP);
    if (w.get(F_LS, domain) > *remL) w.set(F_LS, domain, *remL);
    w.set(F_STATE, domain, w_mul(w.get(wl, domain), sliceSize));
    *remL = w_sub(*remL, w.get(F_LS, domain));
    *remP = w_sub(*remP, w.get(wl, domain));
    *completed = false;
    return domain;
  }
  *remP = w_sub(*remP, w.get(wl, domain));
  *remL = w_sub(*remL, w.get(F_LS, domain));
  if (w.get(wl, domain) > *remP) w.set(wl, domain, *remP);
  if (w.get(F_LS, domain) > *remL) w.set(F_LS, domain, *remL);
  *completed = false;
  return domain;
}

// updateCountsToMinimumGeneric (:1405-1469).  Appends to out[*np..].  Returns
// false on the "code assumptions violated" path (Go returns nil): the appended
// entries are then dropped.
template <class Seq>
__device__ bool update_counts(Wave& w, Seq& seq, int32_t count, int32_t leaderCount, int32_t sliceSize, bool slices,
                              int32_t* out, int* np) {
  ProfScope prof_scope_(w, P_UPDATE);
  const int start = *np;
  int32_t remP = slices ? go_div32(count, sliceSize) : count;
  int32_t remL = leaderCount;
  auto push = [&](int g) {
    if (*np < w.lcap) out[*np] = g;
    else w.overflow = true;
    (*np)++;
  };
  for (; !seq.done(); seq.next()) {
    int dom = seq.cur();
    if (remL > 0) {
      bool completed = false;
      int d = slices ? consume_with_leaders(w, seq, dom, &remP, &remL, F_SSWL, F_SLICE, sliceSize, true, &completed)
                     : consume_with_leaders(w, seq, dom, &remP, &remL, F_SWL, F_STATE, 1, false, &completed);
      push(d);
      if (completed) return true;
      continue;
    }
    if (slices) {
      if (w.bf && w.get(F_SLICE, dom) >= remP) dom = seq.bestfit(remP, F_SLICE);
      w.set(F_LS, dom, 0);
      int32_t sl = w.get(F_SLICE, dom);
      if (sl >= remP) {
        w.set(F_STATE, dom, w_mul(remP, sliceSize));
        w.set(F_SLICE, dom, remP);
        push(dom);
        return true;
      }
      w.set(F_STATE, dom, w_mul(sl, sliceSize));
      remP = w_sub(remP, sl);
      push(dom);
      continue;
    }
    if (w.bf && w.get(F_STATE, dom) >= remP) dom = seq.bestfit(remP, F_STATE);
    w.set(F_LS, dom, 0);
    int32_t st = w.get(F_STATE, dom);
    if (st >= remP) {
      w.set(F_STATE, dom, remP);
      push(dom);
      return true;
    }
    remP = w_sub(remP, st);
    push(dom);
  }
  *np = start;
  return false;
}

// ---- threshold walk: updateCountsToMinimumGeneric without leaders, no sort ----
// Without leaders the walk (:1434-1468) takes the sorted list's elements in
// order until the running sum of their weight w (sliceState with slices,
// state without) reaches rem; the element at that crossing is replaced by
// BestFit's best fit over the rest of the list (:1435, :1453), everything
// before it is taken whole.  Every descent consumer of the result is
// order-independent (lowerLevelDomains is re-sorted, per-parent walks are
// independent, buildAssignment sorts), so only WHICH elements are taken and
// their final counters matter.  With w >= 0 the crossing is found with
// weighted histograms over the sort key's components (sliceState, then state,
// then the domain index within one (sliceState, state) class) in a few
// coalesced passes instead of an O(n log n) sort plus an O(k) dependent walk.

// Decode the components of a key_plain key.
__device__ __forceinline__ int32_t kp_ss(bool lfc, const Key& k) {
  uint32_t k0 = uint32_t(k.hi >> 32);
  return int32_t((lfc ? k0 : ~k0) ^ 0x80000000u);
}
__device__ __forceinline__ int32_t kp_st(const Key& k) { return int32_t(uint32_t(k.hi) ^ 0x80000000u); }

// Strided wave loops with kU independent loads in flight per lane: the loads
// of kU strided indices are issued first (clamped index, so unconditional),
// then the body runs for them in index order.  wave_for: body(i, v) only for
// i < n; wave_for_all: every lane runs body(i, v, valid) (bodies with wave
// collectives).  Single-wave passes over long lists are latency bound; this
// keeps kU requests per lane outstanding instead of one.
constexpr int kU = 8;
template <class T, class Load, class Body>
__device__ __forceinline__ void wave_for(int n, Load load, Body body) {
  const int lane = lane_id();
  for (int base = 0; base < n; base += kU * kWave) {
    T v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) v[u] = load(min(base + u * kWave + lane, n - 1));
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = base + u * kWave + lane;
      if (i < n) body(i, v[u]);
    }
  }
}
template <class T, class Load, class Body>
__device__ __forceinline__ void wave_for_all(int n, Load load, Body body) {
  const int lane = lane_id();
  for (int base = 0; base < n; base += kU * kWave) {
    T v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) v[u] = load(min(base + u * kWave + lane, n - 1));
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = base + u * kWave + lane;
      body(i, v[u], i < n);
    }
  }
}


// m-th smallest (1-based) of cnt uint32 values < 2^bits in LDS (one wave):
// MSB-first radix select with 9-bit digits (hist: 512 LDS words), no sort.
__device__ uint32_t lds_select_kth(const uint32_t* v, int cnt, int m, uint32_t* hist, int lane, int bits,
                                   int digit_bits) {
  if (m == cnt || m == 1) {  // the maximum / minimum: one reduction
    uint32_t r = m == 1 ? ~0u : 0u;
    for (int i = lane; i < cnt; i += kWave) r = m == 1 ? min(r, v[i]) : max(r, v[i]);
#pragma unroll
    for (int d = 1; d <= 32; d <<= 1) {
      const uint32_t o = xor_lane(r, d);
      r = m == 1 ? min(r, o) : max(r, o);
    }
    return r;
  }
  const int NB = 1 << digit_bits;  // 256 or 512
  uint32_t prefix = 0, pmask = 0;
  const int rounds = (bits + digit_bits - 1) / digit_bits;
  for (int rd = rounds - 1; rd >= 0; rd--) {
    const int shift = rd * digit_bits;
    for (int i = lane; i < NB; i += kWave) hist[i] = 0;
    wave_sync();
    for (int i = lane; i < cnt; i += kWave) {
      const uint32_t x = v[i];
      if ((x & pmask) == prefix) atomicAdd(&hist[(x >> shift) & uint32_t(NB - 1)], 1u);
    }
    wave_sync();
    const int PER = NB / kWave;  // bins per lane (4 or 8)
    uint32_t c[8];
    uint32_t lsum = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      c[k] = k < PER ? hist[PER * lane + k] : 0u;
      lsum += c[k];
    }
    const uint32_t x = uint32_t(wave_incl_scan(int(lsum)));
    const uint64_t hit = ballot(x >= uint32_t(m));
    const int src = __ffsll((unsigned long long)hit) - 1;  // exists: m <= matching count
    int digit = 0;
    uint32_t before = x - lsum;
    if (lane == src) {
      int k = 0;
      while (k < PER - 1 && before + c[k] < uint32_t(m)) before += c[k++];
      digit = PER * lane + k;
    }
    digit = bcast(digit, src);
    before = bcast(before, src);
    m -= int(before);
    prefix |= uint32_t(digit) << shift;
    pmask |= uint32_t(NB - 1) << shift;
    wave_sync();
  }
  return prefix;
}


// First position p (in scan order: bin i = p, or kBins-1-p when desc) whose
// inclusive weighted sum reaches need.  Returns the bin (or -1: total < need,
// *before = total) and the sum before it.
constexpr int kThrBins = 256;
__device__ int bins_threshold(const uint64_t* hist, bool desc, int64_t need, int64_t* before) {
  const int lane = lane_id();
  int64_t local[4];
  int64_t lsum = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int p = 4 * lane + k;
    local[k] = int64_t(hist[desc ? kThrBins - 1 - p : p]);
    lsum += local[k];
  }
  int64_t x = lsum;
  for (int d = 1; d < 64; d <<= 1) {
    int64_t y = int64_t(shfl_u64(uint64_t(x), max(lane - d, 0)));
    if (lane >= d) x += y;
  }
  const int64_t excl = x - lsum;
  const uint64_t m = ballot(x >= need);
  if (!m) {
    *before = int64_t(bcast64(uint64_t(x), 63));
    return -1;
  }
  const int src = __ffsll((unsigned long long)m) - 1;
  int pp = -1;
  int64_t bb = excl;
  if (lane == src) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (pp < 0) {
        if (bb + local[k] >= need) pp = 4 * lane + k;
        else bb += local[k];
      }
    }
  }
  pp = bcast(pp, src);
  *before = int64_t(bcast64(uint64_t(bb), src));
  return desc ? kThrBins - 1 - pp : pp;
}

// Returns 1 (taken elements appended to out), 0 (Go returns nil: the list
// cannot hold rem; mutations of a discarded list are unobservable) or -1
// (preconditions unmet: caller sorts).  Keys are materialized in w.gkeys.
__device__ int threshold_walk(Wave& w, const int32_t* gids, int n, int level, int32_t count, int32_t sliceSize,
                              bool slices, int32_t* out, int* np) {
  ProfScope prof_scope_(w, P_THRESHOLD);
  if (w.cap * int(sizeof(Key)) < kThrBins * int(sizeof(uint64_t))) return -1;
  const int loff = g_select_snap.level_off[level];
  const bool lfc = w.lfc;
  const int32_t rem = slices ? go_div32(count, sliceSize) : count;
  Key* keys = w.gkeys;
  uint64_t* hist = reinterpret_cast<uint64_t*>(w.lds);
  for (int i = lane_id(); i < kThrBins; i += kWave) hist[i] = 0;
  wave_sync();
  // pass A: keys, range of the primary component, minimum weight, and the
  // weight per sliceState value for values in [0, kThrBins) (pass B when the
  // values fall outside); all_eq: sliceState == state everywhere
  int32_t vmin = 0x7fffffff, vmax = int32_t(0x80000000u), wmin = 0x7fffffff;
  int64_t wsum = 0;
  bool neq = false;
  {
  ProfScope ps_keys(w, P_TW_KEYS);
  for (int base = 0; base < n; base += kU * kWave) {
    int g[kU];
    int32_t ss[kU], st[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) g[u] = gids[min(base + u * kWave + lane_id(), n - 1)];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      ss[u] = w.get_clean(F_SLICE, g[u]);
      st[u] = w.get_clean(F_STATE, g[u]);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int i = base + u * kWave + lane_id();
      if (i < n) {
        keys[i] = key_plain(lfc, ss[u], st[u], g[u] - loff);
        vmin = min(vmin, ss[u]);
        vmax = max(vmax, ss[u]);
        const int32_t wt = slices ? ss[u] : st[u];
        wmin = min(wmin, wt);
        wsum += wt;
        neq |= ss[u] != st[u];
        if (wt > 0 && ss[u] >= 0 && ss[u] < kThrBins)
          atomicAdd((unsigned long long*)&hist[ss[u]], (unsigned long long)wt);
      }
    }
  }
  }
  wsum = wave_sum_i64(wsum);
#pragma unroll
  for (int m = 1; m <= 32; m <<= 1) {
    vmin = min(vmin, xor_lane(vmin, m));
    vmax = max(vmax, xor_lane(vmax, m));
    wmin = min(wmin, xor_lane(wmin, m));
  }
  const bool all_eq = ballot(neq) == 0;
  wave_fence();
  wave_sync();
  if (wmin < 0 || wsum >= (int64_t(1) << 31)) return -1;  // int32 rem arithmetic never wraps
  Key ck;          // key of the crossing element
  int32_t remc;    // rem left when the walk reaches it
  if (rem <= 0) {  // the first element already satisfies rem
    Key k = key_max();
    wave_for<Key>(n, [&](int i) { return keys[i]; }, [&](int, const Key& x) { k = key_min2(k, x); });
    ck = wave_min_key(k);
    remc = rem;
  } else {
    if (int64_t(vmax) - int64_t(vmin) >= kThrBins) return -1;
    int32_t hbase = 0;  // value of bin 0
    if (vmin < 0 || vmax >= kThrBins) {
      // pass B: weight per sliceState value, bins from vmin
      hbase = vmin;
      for (int i = lane_id(); i < kThrBins; i += kWave) hist[i] = 0;
      wave_sync();
      wave_for<Key>(n, [&](int i) { return keys[i]; }, [&](int, const Key& k) {
        const int32_t ss = kp_ss(lfc, k);
        const int32_t wt = slices ? ss : kp_st(k);
        if (wt > 0) atomicAdd((unsigned long long*)&hist[ss - vmin], (unsigned long long)wt);
      });
      wave_sync();
    }
    int64_t before1;
    const int b1 = bins_threshold(hist, !lfc, rem, &before1);
    if (b1 < 0) return 0;  // the list cannot hold rem (:1469)
    const int32_t t = hbase + b1;
    const int64_t rem1 = rem - before1;
    int32_t u;
    int64_t rem2;
    if (all_eq) {  // class t holds state t only
      u = t;
      rem2 = rem1;
    } else {
    // pass C: state range inside class t
    int32_t umin = 0x7fffffff, umax = int32_t(0x80000000u);
    wave_for<Key>(n, [&](int i) { return keys[i]; }, [&](int, const Key& k) {
      if (kp_ss(lfc, k) == t) {
        umin = min(umin, kp_st(k));
        umax = max(umax, kp_st(k));
      }
    });
#pragma unroll
    for (int m = 1; m <= 32; m <<= 1) {
      umin = min(umin, xor_lane(umin, m));
      umax = max(umax, xor_lane(umax, m));
    }
    if (int64_t(umax) - int64_t(umin) >= kThrBins) return -1;
    // pass D: weight per state value inside class t
    wave_sync();
    for (int i = lane_id(); i < kThrBins; i += kWave) hist[i] = 0;
    wave_sync();
    wave_for<Key>(n, [&](int i) { return keys[i]; }, [&](int, const Key& k) {
      if (kp_ss(lfc, k) == t) {
        const int32_t wt = slices ? t : kp_st(k);
        if (wt > 0) atomicAdd((unsigned long long*)&hist[kp_st(k) - umin], (unsigned long long)wt);
      }
    });
    wave_sync();
    int64_t before2;
    const int b2 = bins_threshold(hist, false, rem1, &before2);
    if (b2 < 0) return -1;  // unreachable: class t holds rem1
    u = umin + b2;
    rem2 = rem1 - before2;
    }
    const int64_t wt = slices ? t : u;  // > 0: the class added weight
    const int64_t m = (rem2 + wt - 1) / wt;
    remc = int32_t(rem2 - (m - 1) * wt);
    // pass E: the m-th smallest index of class (t, u) (radix select in LDS)
    wave_sync();
    uint32_t* cand = reinterpret_cast<uint32_t*>(w.lds);
    const int dbits = w.cap >= 512 ? 9 : 8;         // radix-select digit width (histogram 2^dbits words)
    const int ccap = w.cap * 4 - (1 << dbits);      // uint32 candidate slots before the histogram
    int cnt = 0;
    wave_for_all<Key>(n, [&](int i) { return keys[i]; }, [&](int, const Key& k, bool valid) {
      const bool in = valid && kp_ss(lfc, k) == t && kp_st(k) == u;
      const uint64_t bm = ballot(in);
      const int pos = cnt + __popcll(bm & ((1ull << lane_id()) - 1ull));
      if (in && pos < ccap) cand[pos] = uint32_t(k.lo);
      cnt += __popcll(bm);
    });
    if (cnt > ccap) return -1;
    wave_sync();
    uint32_t kth;
    {
      ProfScope ps_sel(w, P_TW_SELECT);
      const int nbits = 32 - __builtin_clz(uint32_t(max(g_select_snap.level_size[level] - 1, 1)));  // indices < level size
      kth = lds_select_kth(cand, cnt, int(m), cand + ccap, lane_id(), nbits, dbits);
    }
    ck = key_plain(lfc, t, u, int32_t(kth));
    wave_sync();
  }
  // one pass: emit the whole elements before the crossing (lane-private
  // stores) and, BestFit, find the best fit over the crossing and everything
  // after it (findBestFitDomainBy :1216-1231: per lane (weight, key), then a
  // wave arg-min)
  uint32_t bst = ~0u;
  Key best = key_max();
  int cnt = *np;
  ProfScope ps_emit(w, P_TW_EMIT);
  wave_for_all<Key>(n, [&](int i) { return keys[i]; }, [&](int, const Key& k, bool valid) {
    const bool take = valid && key_lt(k, ck);
    const uint64_t bm = ballot(take);
    const int pos = cnt + __popcll(bm & ((1ull << lane_id()) - 1ull));
    if (take) {
      const int g = loff + int(uint32_t(k.lo));
      // !leader: no F_LS; the value only changes if sliceSize * sliceState != state
      if (slices && w_mul(kp_ss(lfc, k), sliceSize) != kp_st(k))
        w.set_walked(g, w_mul(kp_ss(lfc, k), sliceSize), kp_ss(lfc, k));
      if (pos < w.lcap) out[pos] = g;
    } else if (valid && w.bf) {
      const int32_t wt = slices ? kp_ss(lfc, k) : kp_st(k);
      if (wt >= remc) {
        const uint32_t sw = s_asc(wt);
        if (sw < bst || (sw == bst && key_lt(k, best))) {
          bst = sw;
          best = k;
        }
      }
    }
    cnt += __popcll(bm);
  });
  int chosen = loff + int(uint32_t(ck.lo));
  if (w.bf) {
    const uint32_t wbst = uint32_t(wave_min_u64(bst));
    best = wave_min_key(bst == wbst ? best : key_max());
    chosen = loff + int(uint32_t(best.lo));
  }
  wave_fence();
  // the crossing element (or its best fit) takes the remainder
  w.set(F_LS, chosen, 0);
  if (slices) {
    w.set(F_STATE, chosen, w_mul(remc, sliceSize));
    w.set(F_SLICE, chosen, remc);
  } else {
    w.set(F_STATE, chosen, remc);
  }
  if (cnt < w.lcap) out[cnt] = chosen;
  cnt++;
  if (cnt > w.lcap) w.overflow = true;
  *np = cnt;
  wave_fence();
  return 1;
}

// The same leaderless walk over a list already sorted in LDS: the crossing
// is the first position whose inclusive weight sum reaches rem (the
// walk's `w_i >= rem_i` test, :1444/:1459, is exactly S_i >= rem while no int32
// arithmetic wraps), found with a wave scan; elements before it are emitted in
// parallel.  Returns 1 / 0 (nil) / -1 (would wrap: caller walks).
__device__ int lds_prefix_walk(Wave& w, int n, int loff, int32_t count, int32_t sliceSize, bool slices, int32_t* out,
                               int* np) {
  const bool lfc = w.lfc;
  const int32_t rem = slices ? go_div32(count, sliceSize) : count;
  int64_t absum = 0;
  for (int i = lane_id(); i < n; i += kWave) {
    const Key k = w.lds[i];
    const int64_t wt = slices ? kp_ss(lfc, k) : kp_st(k);
    absum += wt < 0 ? -wt : wt;
  }
  absum = wave_sum_i64(absum);
  if (absum + (rem < 0 ? -int64_t(rem) : int64_t(rem)) >= (int64_t(1) << 31)) return -1;
  int64_t run = 0;
  int cross = -1;
  int64_t before = 0;
  for (int i0 = 0; i0 < n; i0 += kWave) {
    const int i = i0 + lane_id();
    int64_t wt = 0;
    if (i < n) {
      const Key k = w.lds[i];
      wt = slices ? kp_ss(lfc, k) : kp_st(k);
    }
    int64_t x = wt;
    for (int d = 1; d < 64; d <<= 1) {
      int64_t y = int64_t(shfl_u64(uint64_t(x), max(lane_id() - d, 0)));
      if (lane_id() >= d) x += y;
    }
    const uint64_t m = ballot(i < n && run + x >= rem);
    if (m) {
      const int src = __ffsll((unsigned long long)m) - 1;
      cross = i0 + src;
      before = run + int64_t(bcast64(uint64_t(x - wt), src));
      break;
    }
    run += int64_t(bcast64(uint64_t(x), 63));
  }
  if (cross < 0) return 0;
  const int32_t remc = int32_t(rem - before);
  int pick = cross;
  if (w.bf) {  // findBestFitDomainBy over [cross, n) (:1216-1231)
    uint64_t best = ~0ull;
    for (int i = cross + lane_id(); i < n; i += kWave) {
      const Key k = w.lds[i];
      const int32_t wt = slices ? kp_ss(lfc, k) : kp_st(k);
      if (wt >= remc) best = min(best, (uint64_t(s_asc(wt)) << 32) | uint32_t(i));
    }
    pick = int(uint32_t(wave_min_u64(best)));
  }
  int cnt = *np;
  for (int i = lane_id(); i < cross; i += kWave) {
    const Key k = w.lds[i];
    const int g = loff + int(uint32_t(k.lo));
    if (slices && w_mul(kp_ss(lfc, k), sliceSize) != kp_st(k))  // !leader: no F_LS; only real changes
      w.set_walked(g, w_mul(kp_ss(lfc, k), sliceSize), kp_ss(lfc, k));
    if (cnt + i < w.lcap) out[cnt + i] = g;
  }
  cnt += cross;
  wave_fence();
  const int chosen = loff + int(uint32_t(w.lds[pick].lo));
  w.set(F_LS, chosen, 0);
  if (slices) {
    w.set(F_STATE, chosen, w_mul(remc, sliceSize));
    w.set(F_SLICE, chosen, remc);
  } else {
    w.set(F_STATE, chosen, remc);
  }
  if (cnt < w.lcap) out[cnt] = chosen;
  cnt++;
  if (cnt > w.lcap) w.overflow = true;
  *np = cnt;
  wave_fence();
  return 1;
}

// Walk an explicit list of gids of one level in the order given by `plain`
// sortedDomains: LDS sort when it fits, lazy iteration otherwise.
__device__ bool walk_sorted(Wave& w, const int32_t* gids, int n, int level, int32_t count, int32_t leaderCount,
                            int32_t sliceSize, bool slices, int32_t sliceRecompute, int32_t* out, int* np) {
  ProfScope prof_scope_(w, P_WALK);
  const int loff = g_select_snap.level_off[level];
  // leaderless walks need no sequential pass (see threshold_walk)
  const bool leaderless = !w.leader && leaderCount <= 0 && sliceRecompute <= 1;
  constexpr int kSmallWalk = 64;  // shorter lists: sort + prefix walk
  if (leaderless && w.bf && slices && n > kSmallWalk && gids != w.listD && go_div32(count, sliceSize) > 0) {
    ProfScope ps_filter(w, P_WS_FILTER);
    // BestFit slice walk with rem > 0: elements with sliceState <= 0 sort after
    // every positive one (sliceState desc), cannot move the running sum up to
    // rem, and cannot be the best fit (weight >= remc > 0), so they are never
    // taken (:1452-1467): walk the positive ones only.
    int m = 0;
    for (int base = 0; base < n; base += kU * kWave) {
      int g[kU];
      int32_t v[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) g[u] = gids[min(base + u * kWave + lane_id(), n - 1)];
#pragma unroll
      for (int u = 0; u < kU; u++) v[u] = w.get_clean(F_SLICE, g[u]);
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const bool keep = base + u * kWave + lane_id() < n && v[u] > 0;
        const uint64_t bm = ballot(keep);
        if (keep) w.listD[m + __popcll(bm & ((1ull << lane_id()) - 1ull))] = g[u];
        m += __popcll(bm);
      }
    }
    wave_fence();
    gids = w.listD;
    n = m;
  }
  if (leaderless && n > kSmallWalk && n <= w.lcap) {  // sort-free histogram walk
    const int r = threshold_walk(w, gids, n, level, count, sliceSize, slices, out, np);
    if (r >= 0) return r == 1;
  }
  if (n <= w.cap) {
    for (int i = lane_id(); i < n; i += kWave) w.lds[i] = w.kplain_clean(gids[i]);
    wave_sync();
    {
      ProfScope ps_(w, P_LDS_SORT);
      lds_sort(w.lds, n, lane_id());
    }
    if (leaderless) {
      const int r = lds_prefix_walk(w, n, loff, count, sliceSize, slices, out, np);
      if (r >= 0) {
        wave_sync();
        return r == 1;
      }
    }
    if (sliceRecompute > 1) {  // multi-layer: recompute sliceState after sorting (:956-965)
      for (int i = 0; i < n; i++) {
        int g = loff + int(uint32_t(w.lds[i].lo));
        w.set(F_SLICE, g, go_div32(w.get(F_STATE, g), sliceRecompute));
        w.set(F_SSWL, g, go_div32(w.get(F_SWL, g), sliceRecompute));
      }
    }
    SeqLds seq{&w, n, loff, 0};
    bool ok = update_counts(w, seq, count, leaderCount, sliceSize, slices, out, np);
    wave_sync();
    return ok;
  }
  if (n > w.lcap) {
    w.overflow = true;
    return false;
  }
  if (leaderless) {
    const int r = threshold_walk(w, gids, n, level, count, sliceSize, slices, out, np);
    if (r >= 0) return r == 1;
  }
  // longer than the LDS: merge-sort the keys in global memory once (O(n log n)),
  // then walk them in order
  for (int i = lane_id(); i < n; i += kWave) w.gkeys[i] = w.kplain_clean(gids[i]);
  wave_fence();
  global_sort(w, w.gkeys, w.gkeys2, n);
  if (sliceRecompute > 1) {
    for (int i = 0; i < n; i++) {
      int g = loff + int(uint32_t(w.gkeys[i].lo));
      w.set(F_SLICE, g, go_div32(w.get(F_STATE, g), sliceRecompute));
      w.set(F_SSWL, g, go_div32(w.get(F_SWL, g), sliceRecompute));
    }
  }
  SeqKeys seq{&w, w.gkeys, n, loff, 0};
  return update_counts(w, seq, count, leaderCount, sliceSize, slices, out, np);
}

// Children (CSR) of `n` domains at `level` appended to out (lowerLevelDomains :1503-1509).
__device__ int gather_children(Wave& w, const int32_t* parents, int n, int level, int32_t* out) {
  ProfScope prof_scope_(w, P_GATHER);
  const DevSnap& s = g_select_snap;
  const int poff = s.level_off[level];
  const int coff = s.level_off[level + 1];
  const int32_t* co = s.child_off + s.child_base[level];
  int np = 0;
  for (int i0 = 0; i0 < n; i0 += kWave) {  // 64 parents per step: ranges, then a scan for the offsets
    const int i = i0 + lane_id();
    int cb = 0, cnt = 0;
    if (i < n) {
      const int p = parents[i] - poff;
      cb = co[p];
      cnt = co[p + 1] - cb;
    }
    int tot;
    const int ex = wave_excl_scan(cnt, &tot);
    if (np + tot > w.lcap) {
      w.overflow = true;
      return np;
    }
    for (int j = 0; j < cnt; j++) out[np + ex + j] = coff + cb + j;
    np += tot;
  }
  wave_fence();
  return np;
}

// gather_children restricted to children with sliceState > 0 (clean reads):
// the BestFit slice walk only ever takes those (see walk_sorted), so the
// filtered list is walked directly.  64 parents per step; their children are
// visited as one flattened range, kU loads in flight per lane.
__device__ int gather_children_positive(Wave& w, const int32_t* parents, int n, int level, int32_t* out) {
  ProfScope prof_scope_(w, P_GATHER);
  const DevSnap& s = g_select_snap;
  const int poff = s.level_off[level];
  const int coff = s.level_off[level + 1];
  const int32_t* co = s.child_off + s.child_base[level];
  int32_t* sh_ex = reinterpret_cast<int32_t*>(w.lds);  // [64] exclusive child offsets of the step's parents
  int32_t* sh_cb = sh_ex + kWave;                        // [64] first child of each
  int np = 0;
  if (w.rack_pos && level == s.L - 2) {
    // children are leaves: the fill's per-parent positive masks give them without loads
    for (int i0 = 0; i0 < n; i0 += kWave) {
      const int i = i0 + lane_id();
      uint64_t m = 0;
      int cb = 0;
      if (i < n) {
        const int p = parents[i] - poff;
        m = w.rack_pos[p];
        cb = co[p];
      }
      int tot;
      int pos = np + wave_excl_scan(__popcll(m), &tot);
      for (; m; m &= m - 1)
        if (pos < w.lcap) out[pos++] = coff + cb + __builtin_ctzll(m);
        else pos++;
      np += tot;
    }
    if (np > w.lcap) w.overflow = true;
    wave_fence();
    return np;
  }
  for (int i0 = 0; i0 < n; i0 += kWave) {
    const int i = i0 + lane_id();
    int cb = 0, cnt = 0;
    if (i < n) {
      const int p = parents[i] - poff;
      cb = co[p];
      cnt = co[p + 1] - cb;
    }
    int tot;
    const int ex = wave_excl_scan(cnt, &tot);
    wave_sync();
    sh_ex[lane_id()] = ex;
    sh_cb[lane_id()] = cb;
    wave_sync();
    const int nparents = min(kWave, n - i0);
    // uniform power-of-two fan-out in this step: element e belongs to parent e >> sh
    const int f0 = bcast(cnt, 0);
    const bool uniform = f0 > 0 && (f0 & (f0 - 1)) == 0 && ballot(i < n && cnt != f0) == 0;
    const int sh = uniform ? __builtin_ctz(f0) : 0;
    for (int b0 = 0; b0 < tot; b0 += kU * kWave) {
      int g[kU];
      int32_t v[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const int e = min(b0 + u * kWave + lane_id(), tot - 1);
        if (uniform) {
          g[u] = coff + __shfl(cb, e >> sh, 64) + (e & (f0 - 1));
        } else {
          int lo = 0, hi = nparents - 1;  // last parent with ex <= e
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (sh_ex[mid] <= e) lo = mid;
            else hi = mid - 1;
          }
          g[u] = coff + sh_cb[lo] + (e - sh_ex[lo]);
        }
      }
#pragma unroll
      for (int u = 0; u < kU; u++) v[u] = w.get_clean(F_SLICE, g[u]);
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const bool keep = b0 + u * kWave + lane_id() < tot && v[u] > 0;
        const uint64_t km = ballot(keep);
        if (keep) {
          const int pos = np + __popcll(km & ((1ull << lane_id()) - 1ull));
          if (pos < w.lcap) out[pos] = g[u];
        }
        np += __popcll(km);
      }
    }
    if (np > w.lcap) {
      w.overflow = true;
      return np;
    }
  }
  wave_fence();
  wave_sync();
  return np;
}

// ---- one descent step in LDS: the children of the chosen parents ----
// The leaderless BestFit descent above the slice level when the slice level
// is the leaf level (:930-935): every level's step is
// updateCountsToMinimumGeneric over sortedDomains(lowerLevelDomains(chosen))
// with the full count.  Walk the positive children of the chosen parents
// (the threshold walk above: take whole elements in sortedDomains order
// until their sliceState reaches sliceCount, the crossing replaced by
// findBestFitDomainBy's best fit).  The parents are sorted first, so their
// children arrive in index order; the candidates' (index, sliceState,
// state) live in LDS (SoA), so every pass is an LDS sweep.  At the last step
// (level = L-2, `ent` set) the (leaf, count) entries of buildAssignment
// (:1472-1501) are written directly; at a step above it (`out` set) the
// chosen children, in index order, become the next step's parents.  Nothing
// is mutated: a level's counters are read by nobody after its walk (the
// next step reads the children's, and a taken leaf ends with sliceState *
// sliceSize, the best fit with the remainder * sliceSize, exactly what the
// generic walk's updates + emit produce).  Returns 1 (written, *nout), 0
// (Go's nil: the children cannot hold sliceCount) or -1 (too many parents /
// candidates or a threshold precondition unmet: nothing written, the caller
// runs the generic path for this level).
// Parents and the chosen children of a step above the last one stay in LDS
// between steps (lds_walk_chosen: the parent-bitmap region), so a step
// issues no global store that a later load's vmcnt wait would drain.
constexpr int kWalkHist = kThrBins;  // lds_level_walk's LDS layout: hist | SP | BM | CI | CS | CT
constexpr int kWalkMaxPar = 1024;
__device__ __forceinline__ int32_t* lds_walk_chosen(const Wave& w) {
  return reinterpret_cast<int32_t*>(w.lds) + kWalkHist + kWalkMaxPar;
}
__device__ int lds_level_walk(Wave& w, int level, const int32_t* parents, int np, bool parents_lds, int32_t count,
                              int32_t sliceSize, int32_t* ent, int ecap, int32_t* out, int* nout, bool* out_lds) {
  ProfScope prof_scope_(w, P_FINAL);
  const DevSnap& s = g_select_snap;
  const int lane = lane_id();
  const int32_t rem = go_div32(count, sliceSize);
  const uint64_t* rack_pos = level == s.L - 2 ? w.rack_pos : nullptr;  // the fill's positive-leaf masks
  constexpr int kHist = kWalkHist;    // weight per sliceState value (u32: the weight sum stays < 2^31)
  constexpr int kMaxPar = kWalkMaxPar;  // parents (sorted list) and parent-bitmap words
  if (np > kMaxPar || np <= 0 || rem <= 0) return -1;
  const int cmax = (w.lds_bytes - (kHist + 2 * kMaxPar) * 4) / 12;
  uint32_t* hist = reinterpret_cast<uint32_t*>(w.lds);
  int32_t* SP = reinterpret_cast<int32_t*>(hist + kHist);  // parents in index order
  uint32_t* BM = reinterpret_cast<uint32_t*>(SP + kMaxPar); // parent bitmap over [pmin, pmax]
  int32_t* CI = reinterpret_cast<int32_t*>(BM + kMaxPar);   // candidates: leaf index, sliceState, state
  int32_t* CS = CI + max(cmax, 0);
  int32_t* CT = CS + max(cmax, 0);
  const int poff = s.level_off[level], coff = s.level_off[level + 1];
  const int32_t* co = s.child_off + s.child_base[level];
  // weight per sliceState value, by absolute value (the candidates are
  // positive); cleared while the parents' loads are in flight
  for (int i = lane; i < kHist; i += kWave) hist[i] = 0;
  // parents in index order through an LDS bitmap (the walk above listed
  // them in its sort order); up to 64 of them stay in a register
  [[maybe_unused]] uint64_t t_prof = KTAS_PROFILE ? wall_clock64() : 0;
  auto lap_prof = [&](int cat) {
#if KTAS_PROFILE
    const uint64_t t = wall_clock64();
    w.prof[cat] += t - t_prof;
    t_prof = t;
#else
    (void)cat;
#endif
  };
  if (cmax <= 0) return -1;
  int nsp = 0;
  if (parents_lds) {  // the previous step's chosen children: in LDS, in index order
    const int32_t* P = lds_walk_chosen(w);
    for (int i = lane; i < np; i += kWave) SP[i] = P[i] - poff;
    nsp = np;
  } else {
    const int32_t p_reg = lane < np ? parents[lane] : INT32_MAX;
    int32_t pmin = p_reg, pmax = lane < np ? p_reg : INT32_MIN;
    for (int i = kWave + lane; i < np; i += kWave) {
      pmin = min(pmin, parents[i]);
      pmax = max(pmax, parents[i]);
    }
    pmin = group_reduce(pmin, 64, OpMin());
    pmax = group_reduce(pmax, 64, OpMax());
    const int words = (pmax - pmin) / 32 + 1;
    if (words > kMaxPar) return -1;
    for (int i = lane; i < words; i += kWave) BM[i] = 0;
    wave_sync();
    if (lane < np) atomicOr(&BM[(p_reg - pmin) >> 5], 1u << ((p_reg - pmin) & 31));
    for (int i = kWave + lane; i < np; i += kWave) atomicOr(&BM[(parents[i] - pmin) >> 5], 1u << ((parents[i] - pmin) & 31));
    wave_sync();
    for (int j0 = 0; j0 < words; j0 += kWave) {
      const int j = j0 + lane;
      const uint32_t word = j < words ? BM[j] : 0u;
      int tot;
      int pos = nsp + wave_excl_scan(__popc(word), &tot);
      for (uint32_t x = word; x; x &= x - 1) SP[pos++] = pmin + 32 * j + __builtin_ctz(x) - poff;
      nsp += tot;
    }
  }
  wave_sync();
  lap_prof(P_FW_PARENTS);
  // their children (leaf indices), in leaf order: 64 parents per step
  int total = 0;
  for (int p0 = 0; p0 < nsp; p0 += kWave) {
    const bool act = p0 + lane < nsp;
    const int p = act ? SP[p0 + lane] : 0;
    const int cb = act ? co[p] : 0;
    uint64_t mask = 0;  // positive children of this lane's parent (bit j: child cb + j)
    int nc = 0;
    if (rack_pos) {  // the fill's per-parent masks: no counter loads
      mask = act ? rack_pos[p] : 0ull;
      nc = __popcll(mask);
    } else {
      nc = act ? co[p + 1] - cb : 0;
    }
    int tot;
    int off = total + wave_excl_scan(nc, &tot);
    if (total + tot > cmax) return -1;
    if (rack_pos) {
      for (uint64_t m = mask; m; m &= m - 1) CI[off++] = cb + __builtin_ctzll(m);
    } else {
      for (int j = 0; j < nc; j++) CI[off + j] = cb + j;
    }
    total += tot;
  }
  wave_sync();
  lap_prof(P_FW_CHILDREN);
  // the candidates' counters (clean reads: nothing of this level was walked
  // before), kU loads in flight; the non-positive ones drop.  Pass A rides
  // along: range, weight sum, sliceState == state everywhere, and the weight
  // per value for values below kHist
  int n = 0;
  int32_t vmin = INT32_MAX, vmax = INT32_MIN;
  int64_t wsum = 0;
  bool neq = false;
  for (int base = 0; base < total; base += kU * kWave) {
    int32_t ix[kU], ss[kU], st[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) ix[u] = CI[min(base + u * kWave + lane, total - 1)];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      ss[u] = w.get_clean(F_SLICE, coff + ix[u]);
      st[u] = w.get_clean(F_STATE, coff + ix[u]);
    }
    wave_sync();
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const bool keep = base + u * kWave + lane < total && ss[u] > 0;
      const uint64_t km = ballot(keep);
      if (keep) {
        const int pos = n + __popcll(km & ((1ull << lane) - 1ull));
        CI[pos] = ix[u];
        CS[pos] = ss[u];
        CT[pos] = st[u];
        vmin = min(vmin, ss[u]);
        vmax = max(vmax, ss[u]);
        wsum += ss[u];
        neq |= ss[u] != st[u];
        if (ss[u] < kHist) atomicAdd(&hist[ss[u]], uint32_t(ss[u]));
      }
      n += __popcll(km);
    }
    wave_sync();
  }
  vmin = group_reduce(vmin, 64, OpMin());
  vmax = group_reduce(vmax, 64, OpMax());
  wsum = wave_sum_i64(wsum);
  const bool all_eq = ballot(neq) == 0;
  lap_prof(P_FW_LOADS);
  if (n == 0 || wsum >= (int64_t(1) << 31) || int64_t(vmax) - vmin >= kHist) return -1;
  if (wsum < rem) return 0;  // the list cannot hold rem (:1469)
  int32_t hbase = 0;  // value of bin 0
  if (vmax >= kHist) {  // values past the absolute bins: rebuild from vmin
    hbase = vmin;
    for (int i = lane; i < kHist; i += kWave) hist[i] = 0;
    wave_sync();
    for (int i = lane; i < n; i += kWave) atomicAdd(&hist[CS[i] - vmin], uint32_t(CS[i]));
  }
  wave_sync();
  // the crossing class t: first value (descending) whose inclusive weight reaches rem
  int32_t t;
  int64_t before1;
  {
    int64_t local[4], lsum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int b = kHist - 1 - (4 * lane + k);
      local[k] = hist[b];
      lsum += local[k];
    }
    int64_t x = lsum;
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t y = int64_t(shfl_u64(uint64_t(x), max(lane - d, 0)));
      if (lane >= d) x += y;
    }
    const uint64_t hit = ballot(x >= rem);  // exists: wsum >= rem
    const int src = __ffsll((unsigned long long)hit) - 1;
    int pp = -1;
    int64_t bb = x - lsum;
    if (lane == src) {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (pp < 0) {
          if (bb + local[k] >= rem) pp = 4 * lane + k;
          else bb += local[k];
        }
    }
    t = hbase + (kHist - 1 - bcast(pp, src));
    before1 = int64_t(bcast64(uint64_t(bb), src));
  }
  const int64_t rem1 = rem - before1;
  // inside class t the order is state ascending: the crossing state u
  int32_t u = t;
  int64_t rem2 = rem1;
  if (!all_eq) {
    int32_t umin = INT32_MAX, umax = INT32_MIN;
    for (int i = lane; i < n; i += kWave)
      if (CS[i] == t) {
        umin = min(umin, CT[i]);
        umax = max(umax, CT[i]);
      }
    umin = group_reduce(umin, 64, OpMin());
    umax = group_reduce(umax, 64, OpMax());
    if (int64_t(umax) - umin >= kHist) return -1;
    wave_sync();
    for (int i = lane; i < kHist; i += kWave) hist[i] = 0;
    wave_sync();
    for (int i = lane; i < n; i += kWave)
      if (CS[i] == t) atomicAdd(&hist[CT[i] - umin], uint32_t(t));
    wave_sync();
    int64_t acc = 0;
    int j = 0;
    for (; j < kHist; j++) {  // wave-uniform walk over the class's state values
      const uint32_t h = hist[j];
      if (acc + h >= rem1) break;
      acc += h;
    }
    u = umin + j;
    rem2 = rem1 - acc;
  }
  const int64_t m = (rem2 + t - 1) / t;  // elements of class (t, u) taken; the m-th is the crossing
  const int32_t remc = int32_t(rem2 - (m - 1) * t);
  // One pass: the crossing (the m-th element of class (t, u) in candidate =
  // index order) and findBestFitDomainBy over the crossing and everything
  // after it (:1216-1231: minimal sliceState >= remc, first in sorted order).
  // Elements of value v in [remc, t) all sort after the crossing (value
  // desc), so their minimum needs no crossing; when there is none, the best
  // fit has value t: the crossing itself (all_eq: state == t for the whole
  // class, so the crossing is its first element not taken), else the
  // generic pass below.
  int32_t kth = -1;
  uint64_t bv = ~0ull;  // (s_asc(weight), s_asc(state))
  int32_t bix = INT32_MAX;
  {
    int64_t seen = 0;
    for (int i0 = 0; i0 < n; i0 += kWave) {
      const int i = i0 + lane;
      int32_t v = 0, st = 0, ix = 0;
      if (i < n) {
        v = CS[i];
        st = CT[i];
        ix = CI[i];
      }
      const bool in = i < n && v == t && st == u;
      const uint64_t bm = ballot(in);
      const int c = __popcll(bm);
      if (kth < 0 && seen + c >= m) {
        const int r = int(m - seen);  // r-th set bit of bm (1-based)
        const bool mine = in && __popcll(bm & ((1ull << lane) - 1ull)) == r - 1;
        kth = bcast(ix, __ffsll((unsigned long long)ballot(mine)) - 1);
      }
      seen += c;
      if (i < n && v < t && v >= remc) {
        const uint64_t k = (uint64_t(s_asc(v)) << 32) | s_asc(st);
        if (k < bv || (k == bv && ix < bix)) {
          bv = k;
          bix = ix;
        }
      }
    }
  }
  // key order (sortedDomains, BestFit: sliceState desc, state asc, index asc)
  auto before_cross = [&](int32_t v, int32_t st, int32_t ix) {
    return v > t || (v == t && (st < u || (st == u && ix < kth)));
  };
  if (!all_eq) {  // value-t elements after the crossing compete with the lower values
    for (int i = lane; i < n; i += kWave) {
      const int32_t v = CS[i], st = CT[i], ix = CI[i];
      if (v == t && !before_cross(v, st, ix)) {
        const uint64_t k = (uint64_t(s_asc(v)) << 32) | s_asc(st);
        if (k < bv || (k == bv && ix < bix)) {
          bv = k;
          bix = ix;
        }
      }
    }
  }
  butterfly(64, [&](auto mm) {
    constexpr int M = decltype(mm)::value;
    const uint64_t ov = bfly64<M>(bv);
    const int32_t oi = bfly_i<M>(bix);
    if (ov < bv || (ov == bv && oi < bix)) {
      bv = ov;
      bix = oi;
    }
  });
  const int32_t chosen = bv == ~0ull ? kth : bix;  // all_eq without a lower value: the crossing
  lap_prof(P_FW_SELECT);
  // emission in index order: taken children with sliceState * sliceSize, the
  // best fit with the remainder; zero counts dropped (buildAssignment :1478);
  // above the last step the chosen children (taken and the best fit)
  int cnt = 0;
  const bool to_lds = !ent && n <= kMaxPar;  // the chosen children stay in LDS (the bitmap region)
  int32_t* chosen_lds = lds_walk_chosen(w);
  const int ocap = ent ? ecap : w.lcap;
  for (int i0 = 0; i0 < n; i0 += kWave) {
    const int i = i0 + lane;
    int32_t ix = 0, c = 0;
    if (i < n) {
      ix = CI[i];
      if (before_cross(CS[i], CT[i], ix)) c = ent ? w_mul(CS[i], sliceSize) : 1;
      else if (ix == chosen) c = ent ? w_mul(remc, sliceSize) : 1;
    }
    const bool keep = c != 0;
    const uint64_t km = ballot(keep);
    if (keep) {
      const int pos = cnt + __popcll(km & ((1ull << lane) - 1ull));
      if (ent) {
        if (pos < ocap) put_entry(ent, pos, ix, c);  // one 8-byte store
      } else if (to_lds) {
        chosen_lds[pos] = coff + ix;
      } else if (pos < ocap) {
        out[pos] = coff + ix;
      }
    }
    cnt += __popcll(km);
  }
  if (!ent && !to_lds && cnt > ocap) w.overflow = true;
  wave_sync();
  lap_prof(P_FW_EMIT);
  *nout = cnt;
  *out_lds = to_lds;
  return 1;
}

// multiLayerNotFitMessage numbers (:1754-1793)
__device__ void multilayer_message(Wave& w, int level, kueue_tas_eval_out& o) {
  const DevSnap& s = g_select_snap;
  const int D = s.level_size[level];
  const int loff = s.level_off[level];
  uint64_t best = ~0ull;
  for (int i = lane_id(); i < D; i += kWave) {
    int g = loff + i;
    uint32_t rank = s.id_rank ? uint32_t(s.id_rank[g]) : uint32_t(i);
    // highest sliceState, ties: smaller DomainID string
    uint64_t k = (uint64_t(s_desc(w.get(F_SLICE, g))) << 32) | rank;
    best = k < best ? k : best;
  }
  best = wave_min_u64(best);
  // recover the index of the domain with that rank
  int bidx = -1;
  uint32_t brank = uint32_t(best);
  for (int i = lane_id(); i < D; i += kWave) {
    uint32_t rank = s.id_rank ? uint32_t(s.id_rank[loff + i]) : uint32_t(i);
    if (rank == brank) bidx = i;
  }
  for (int m = 1; m <= 32; m <<= 1) bidx = max(bidx, xor_lane(bidx, m));
  for (int c = 0; c < w.ev->num_layers && c < KUEUE_TAS_MAX_LAYERS; c++) {
    int t = w.ev->layer_level[c];
    int32_t size = w.ev->layer_size[c];
    o.ml_need[c] = go_div32(w.ev->count, size);
    int32_t fit = 0;
    if (t == level) {
      fit = go_div32(w.get(F_STATE, loff + bidx), size);
    } else if (t > level) {
      int lo = bidx, hi = bidx + 1;
      for (int l = level; l < t; l++) {
        lo = s.child_off[s.child_base[l] + lo];
        hi = s.child_off[s.child_base[l] + hi];
      }
      int32_t acc = 0;
      for (int i = lo + lane_id(); i < hi; i += kWave) acc = w_add(acc, go_div32(w.get(F_STATE, s.level_off[t] + i), size));
      fit = wave_sum_wrap32(acc);
    }
    o.ml_fit[c] = fit;
  }
}

// notFitReason (:1253-1258)
__device__ void not_fit(Wave& w, int level, int32_t fit, int32_t total, kueue_tas_eval_out& o) {
  if (w.ev->flags & KUEUE_TAS_F_MULTILAYER) {
    o.status = KUEUE_TAS_ST_MULTILAYER;
    o.a = level;
    multilayer_message(w, level, o);
  } else {
    o.status = KUEUE_TAS_ST_NOT_FIT;
    o.a = fit;
    o.b = total;
  }
}

// Write (leaf, count) entries sorted by leaf index (buildAssignment :1490-1501).
__device__ int emit_sorted(Wave& w, const int32_t* gids, int n, bool use_ls, bool positive_only, int32_t* ent, int ent_cap,
                           int base) {
  ProfScope prof_scope_(w, P_EMIT);
  const int loff = g_select_snap.level_off[g_select_snap.L - 1];
  if (n > 0) {
    // Leaf-index range of the output: when its bitmap fits the wave's LDS,
    // mark the leaves and emit them in index order without sorting.
    int32_t mn = 0x7fffffff, mx = -1;
    wave_for<int32_t>(n, [&](int i) { return gids[i]; }, [&](int, int32_t g) {
      mn = min(mn, g - loff);
      mx = max(mx, g - loff);
    });
#pragma unroll
    for (int m = 1; m <= 32; m <<= 1) {
      mn = min(mn, xor_lane(mn, m));
      mx = max(mx, xor_lane(mx, m));
    }
    const int64_t words = (int64_t(mx) - mn + 32) / 32;
    if (words * 4 <= int64_t(w.cap) * int64_t(sizeof(Key))) {
      uint32_t* bm = reinterpret_cast<uint32_t*>(w.lds);
      wave_sync();
      for (int j = lane_id(); j < words; j += kWave) bm[j] = 0;
      wave_sync();
      wave_for<int32_t>(n, [&](int i) { return gids[i]; }, [&](int, int32_t g) {
        const int off = g - loff - mn;
        atomicOr(&bm[off >> 5], 1u << (off & 31));
      });
      wave_sync();
      // marked leaves in index order -> scratch list (stores only) ...
      int32_t* sorted = reinterpret_cast<int32_t*>(w.gkeys);
      int ns = 0;
      for (int64_t j0 = 0; j0 < words; j0 += kWave) {
        const int64_t j = j0 + lane_id();
        const uint32_t word = j < words ? bm[j] : 0u;
        int tot;
        int pos = ns + wave_excl_scan(__popc(word), &tot);
        for (uint32_t x = word; x; x &= x - 1) sorted[pos++] = mn + int32_t(j) * 32 + __builtin_ctz(x);
        ns += tot;
      }
      wave_fence();
      // ... then their counts with kU loads in flight, kept ones compacted in order
      int cnt = base;
      for (int b0 = 0; b0 < ns; b0 += kU * kWave) {
        int32_t lf[kU], v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) lf[u] = sorted[min(b0 + u * kWave + lane_id(), ns - 1)];
#pragma unroll
        for (int u = 0; u < kU; u++) v[u] = use_ls ? w.get(F_LS, loff + lf[u]) : w.get(F_STATE, loff + lf[u]);
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const bool keep = b0 + u * kWave + lane_id() < ns && (positive_only ? v[u] > 0 : v[u] != 0);
          const uint64_t km = ballot(keep);
          if (keep) {
            const int pos = cnt + __popcll(km & ((1ull << lane_id()) - 1ull));
            if (pos < ent_cap) {
              put_entry(ent, pos, lf[u], v[u]);
            }
          }
          cnt += __popcll(km);
        }
      }
      wave_sync();
      return cnt - base;
    }
  }
  Key* arr;
  if (n <= w.cap) {
    for (int i = lane_id(); i < n; i += kWave) w.lds[i] = Key{0, uint64_t(uint32_t(gids[i] - loff))};
    wave_sync();
    {
      ProfScope ps_(w, P_LDS_SORT);
      lds_sort(w.lds, n, lane_id());
    }
    arr = w.lds;
  } else {
    for (int i = lane_id(); i < n; i += kWave) w.gkeys[i] = Key{0, uint64_t(uint32_t(gids[i] - loff))};
    wave_fence();
    global_sort(w, w.gkeys, w.gkeys2, n);
    arr = w.gkeys;
  }
  int cnt = base;
  for (int i0 = 0; i0 < n; i0 += kWave) {
    int i = i0 + lane_id();
    int32_t leaf = 0, v = 0;
    bool keep = false;
    if (i < n) {
      leaf = int32_t(uint32_t(arr[i].lo));
      v = use_ls ? w.get(F_LS, loff + leaf) : w.get(F_STATE, loff + leaf);
      keep = positive_only ? v > 0 : v != 0;
    }
    uint64_t m = ballot(keep);
    int rank = __popcll(m & ((1ull << lane_id()) - 1ull));
    if (keep) {
      int pos = cnt + rank;
      if (pos < ent_cap) {
        put_entry(ent, pos, leaf, v);
      }
    }
    cnt += __popcll(m);
  }
  wave_sync();
  return cnt - base;
}

// Wave-wide exclusive prefix sum of per-lane counts.
// LeastFreeCapacity greedy over all leaves without leaders (the
// findLevelWithFitDomains greedy :1278-1318 followed by
// updateCountsToMinimumGeneric, LFC order) for n > LDS capacity: histogram
// threshold select on sliceState instead of a full sort.  Requires every
// leaf sliceState >= 0 (then zero-capacity leaves are output-invisible).
// Leaf counters are read 4 at a time (16-byte aligned level start).
// Returns 1 done, 0 needs the generic path.
__device__ int lfc_leaf_greedy(Wave& w, int32_t sliceCount, kueue_tas_eval_out& o, int32_t* ent, int ent_cap) {
  const DevSnap& s = g_select_snap;
  const int D = s.N;
  const int loff = s.level_off[s.L - 1];
  const int32_t ss = w.ev->slice_size;
  const int4* S4 = reinterpret_cast<const int4*>(w.ctr + loff);
  const int4* SS4 = reinterpret_cast<const int4*>(w.ctr + w.ssoff + loff);
  const int nq = (D + 3) / 4;
  constexpr int kBins = 256;
  uint32_t* hist = reinterpret_cast<uint32_t*>(w.lds);  // 1 KiB <= list_cap * 16 B (host: list_cap >= 64)
  for (int i = lane_id(); i < kBins; i += kWave) hist[i] = 0;
  wave_sync();
  int64_t over = 0;
  for (int q = lane_id(); q < nq; q += kWave) {
    int4 v4 = SS4[q];
    int vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int32_t v = vv[k];
      if (4 * q + k < D && v > 0) {
        if (v < kBins) atomicAdd(&hist[v], 1u);
        else over += v;
      }
    }
  }
  wave_sync();
  over = wave_sum_i64(over);
  // threshold value t (ascending): per-lane chunk sums of bins, then a scan
  int64_t need = sliceCount;
  int64_t before = 0;
  int t = -1;
  {
    // each lane owns 4 consecutive bins
    int64_t local[4];
    int64_t lsum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int v = 4 * lane_id() + k;
      local[k] = v >= 1 ? int64_t(hist[v]) * v : 0;
      lsum += local[k];
    }
    int64_t x = lsum;
    for (int d = 1; d < 64; d <<= 1) {
      int64_t y = int64_t(shfl_u64(uint64_t(x), max(lane_id() - d, 0)));
      if (lane_id() >= d) x += y;
    }
    int64_t excl = x - lsum;
    // first lane whose inclusive sum reaches need
    uint64_t m = ballot(x >= need);
    if (m) {
      int src = __ffsll((unsigned long long)m) - 1;
      int64_t e = int64_t(bcast64(uint64_t(excl), src));
      int tt = -1;
      int64_t bb = e;
      if (lane_id() == src) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (tt < 0) {
            if (bb + local[k] >= need) tt = 4 * lane_id() + k;
            else bb += local[k];
          }
        }
      }
      t = bcast(tt, src);
      before = int64_t(bcast64(uint64_t(bb), src));
    } else {
      before = int64_t(bcast64(uint64_t(x), 63));
    }
  }
  if (t < 0) {
    if (before + over >= need) return 0;  // threshold in the overflow range: generic path
    // not enough capacity: greedy fails with remaining = need - total (:1315-1316)
    int64_t total = before + over;
    not_fit(w, s.L - 1, int32_t(total), sliceCount, o);
    return 1;
  }
  int64_t m = (need - before + t - 1) / t;  // elements of value t taken (last one is the crossing)
  int32_t rem_last = int32_t(need - before - (m - 1) * t);
  // order inside value t: state asc, then index asc
  int32_t u = t * ss;  // state threshold
  int64_t mp = m;      // rank among (value t, state u) in index order
  if (ss > 1) {
    if (ss > kBins) return 0;
    wave_sync();
    for (int i = lane_id(); i < kBins; i += kWave) hist[i] = 0;
    wave_sync();
    for (int q = lane_id(); q < nq; q += kWave) {
      int4 v4 = SS4[q], s4 = S4[q];
      int vv[4] = {v4.x, v4.y, v4.z, v4.w}, st[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (4 * q + k < D && vv[k] == t) atomicAdd(&hist[st[k] - t * ss], 1u);
    }
    wave_sync();
    int64_t acc = 0;
    int j = 0;
    for (; j < ss; j++) {
      if (acc + hist[j] >= m) break;
      acc += hist[j];
    }
    u = t * ss + j;
    mp = m - acc;
  }
  // emit in index order: v < t (v > 0), or v == t && state < u, or (state == u && rank < mp)
  int64_t seen = 0;
  int cnt = 0;
  for (int q0 = 0; q0 < nq; q0 += kWave) {
    const int q = q0 + lane_id();
    int vv[4] = {0, 0, 0, 0}, st[4] = {0, 0, 0, 0};
    if (q < nq) {
      int4 v4 = SS4[q], s4 = S4[q];
      vv[0] = v4.x; vv[1] = v4.y; vv[2] = v4.z; vv[3] = v4.w;
      st[0] = s4.x; st[1] = s4.y; st[2] = s4.z; st[3] = s4.w;
    }
    int ntie = 0;
    bool tie[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      tie[k] = (4 * q + k < D) && vv[k] == t && st[k] == u;
      ntie += tie[k] ? 1 : 0;
    }
    int tie_total;
    int tie_excl = wave_excl_scan(ntie, &tie_total);
    int64_t r = seen + tie_excl;
    bool keep[4];
    int32_t val[4];
    int nkeep = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const bool in = 4 * q + k < D;
      keep[k] = in && ((vv[k] > 0 && vv[k] < t) || (vv[k] == t && st[k] < u) || (tie[k] && r < mp));
      const bool crossing = tie[k] && r == mp - 1;
      val[k] = crossing ? w_mul(rem_last, ss) : w_mul(vv[k], ss);
      if (tie[k]) r++;
      nkeep += keep[k] ? 1 : 0;
    }
    int keep_total;
    int pos = cnt + wave_excl_scan(nkeep, &keep_total);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (keep[k]) {
        if (pos < ent_cap) {
          put_entry(ent, pos, 4 * q + k, val[k]);
        }
        pos++;
      }
    }
    cnt += keep_total;
    seen += tie_total;
  }
  wave_sync();
  o.status = KUEUE_TAS_ST_OK;
  o.fit_level = s.L - 1;
  o.num_workers = cnt;
  if (cnt > ent_cap) o.status = KUEUE_TAS_ST_INTERNAL;
  return 1;
}

// ---- fast LeastFreeCapacity leaf path (LfcJob, tas_internal.h) ----
// For an unconstrained eval under TASProfileMixed without leader, with slice
// size 1 at the leaf level, findLevelWithFitDomains (:1236-1318) at the leaf
// level sorts leaves by (value asc, index asc) (sortedDomainsWithLeader /
// sortedDomains, LFC; value = sliceState = state).  Then:
//  * first fit (:1260-1265): the smallest value >= sliceCount, smallest index;
//    updateCountsToMinimumGeneric gives it state = count;
//  * otherwise the greedy (:1278-1318) takes leaves in that order until the
//    value mass reaches sliceCount: all leaves below a threshold value t and
//    the first m leaves of value t, the last one getting the remainder
//    (updateCountsToMinimumGeneric, slices, :1437-1450); zero-value leaves
//    end with state 0 and are dropped by buildAssignment (:1476-1480).
// Both only need the class's value histogram (lfc_total_kernel); the greedy
// output is expanded by lfc_emit_kernel.  Reads the class rep's counters in
// place and never writes counters, so evals of one class share them.

// Smallest leaf index whose value is v (tot[v] > 0): first chunk with a count, then a scan of it.
__device__ int lfc_first_leaf(const Wave& w, const DevBatch& b, int slot, const int32_t* V, int v) {
  const uint32_t* ch = b.lfc_ch + int64_t(slot) * b.lfc_nchunks * kLfcBins;
  int chunk = -1;
  for (int c0 = 0; c0 < b.lfc_nchunks && chunk < 0; c0 += kWave) {
    const int c = c0 + lane_id();
    const uint64_t m = ballot(c < b.lfc_nchunks && ch[int64_t(c) * kLfcBins + v] > 0);
    if (m) chunk = c0 + __ffsll((unsigned long long)m) - 1;
  }
  if (chunk < 0) return -1;
  // the chunk in rounds of 8 x 64 leaves, every load of a round issued
  // before its ballots (one memory round trip per 512 leaves, not per 64)
  const int lo = chunk * kLfcChunk, hi = min(g_select_snap.N, lo + kLfcChunk);
  constexpr int kU = 8;
  for (int i0 = lo; i0 < hi; i0 += kU * kWave) {
    int32_t x[kU];
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const int i = i0 + k * kWave + lane_id();
      x[k] = i < hi ? V[i] : -1;
    }
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const uint64_t m = ballot(x[k] == v);
      if (m) return i0 + k * kWave + __ffsll((unsigned long long)m) - 1;
    }
  }
  return -1;
}

// Greedy whose threshold lies among the overflow values (>= kLfcBins - 1):
// exact single-wave version (value windows over all leaves, then emission in
// index order).  Rare: leaf values that large need tiny requests.
__device__ void lfc_wide(Wave& w, int32_t need, const int32_t* V, int64_t before, int64_t below,
                         kueue_tas_eval_out& o, int32_t* ent, int ecap) {
  const DevSnap& s = g_select_snap;
  const int N = s.N;
  uint32_t* hist = reinterpret_cast<uint32_t*>(w.lds);  // 1 KiB <= list_cap * 16 B
  constexpr int kW = 256;
  int32_t lo = kLfcBins - 1;
  int32_t t = -1;
  for (;;) {
    // skip the gap to the next present value
    int32_t vmin = 0x7fffffff;
    for (int i = lane_id(); i < N; i += kWave) {
      const int32_t x = V[i];
      if (x >= lo && x < vmin) vmin = x;
    }
#pragma unroll
    for (int m = 1; m <= 32; m <<= 1) vmin = min(vmin, xor_lane(vmin, m));
    if (vmin == 0x7fffffff) break;
    lo = vmin;
    for (int i = lane_id(); i < kW; i += kWave) hist[i] = 0;
    wave_sync();
    for (int i = lane_id(); i < N; i += kWave) {
      const int32_t x = V[i];
      if (x >= lo && int64_t(x) < int64_t(lo) + kW) atomicAdd(&hist[x - lo], 1u);
    }
    wave_sync();
    int64_t acc = before, cnt = below;
    for (int k = 0; k < kW; k++) {  // wave-uniform walk over the window
      const uint32_t c = hist[k];
      if (!c) continue;
      const int64_t v = int64_t(lo) + k;
      if (acc + v * int64_t(c) >= need) {
        t = int32_t(v);
        break;
      }
      acc += v * int64_t(c);
      cnt += c;
    }
    before = acc;
    below = cnt;
    wave_sync();
    if (t >= 0 || int64_t(lo) + kW > 0x7fffffffLL) break;
    lo += kW;
  }
  if (t < 0) {  // cannot happen (the caller checked the total); keep the reference's failure shape
    not_fit(w, s.L - 1, int32_t(before), need, o);
    return;
  }
  const int64_t mt = (int64_t(need) - before + t - 1) / t;
  const int32_t rem_last = int32_t(int64_t(need) - before - (mt - 1) * t);
  int64_t seen = 0;
  int cnt = 0;
  for (int i0 = 0; i0 < N; i0 += kWave) {
    const int i = i0 + lane_id();
    const int32_t x = i < N ? V[i] : 0;
    const bool tie = i < N && x == t;
    const uint64_t tm = ballot(tie);
    const int64_t r = seen + __popcll(tm & ((1ull << lane_id()) - 1ull));
    const bool keep = (x > 0 && x < t) || (tie && r < mt);
    const uint64_t km = ballot(keep);
    if (keep) {
      const int pos = cnt + __popcll(km & ((1ull << lane_id()) - 1ull));
      if (pos < ecap) {
        put_entry(ent, pos, i, (tie && r == mt - 1) ? rem_last : x);
      }
    }
    cnt += __popcll(km);
    seen += __popcll(tm);
  }
  wave_sync();
  o.status = KUEUE_TAS_ST_OK;
  o.fit_level = s.L - 1;
  o.num_workers = cnt;
  if (cnt > ecap) o.status = KUEUE_TAS_ST_INTERNAL;
}

__device__ LfcJob lfc_fast(Wave& w, const DevBatch& b, int slot, kueue_tas_eval_out& o, int32_t* ent, int ecap) {
  const DevSnap& s = g_select_snap;
  const int L1 = s.L - 1;
  const int lane = lane_id();
  const int32_t* V = w.ctr + w.ssoff + s.level_off[L1];
  const int32_t need = w.ev->count;  // sliceCount = count / 1 (host: count >= 0)
  const uint32_t* tot = b.lfc_tot + int64_t(slot) * kLfcBins;
  LfcJob job{0, 0, 0, 0};
  static_assert(kLfcBins == 128, "two bins per lane");
  const uint32_t h0 = tot[lane], h1 = tot[lane + 64];
  const uint32_t nover = bcast(h1, 63);
  // LFC first fit (:1260-1265)
  int fit_leaf = -1;
  if (need <= kLfcBins - 2) {
    const uint64_t m0 = ballot(lane >= need && h0 > 0);
    const uint64_t m1 = ballot(lane + 64 >= need && lane + 64 < kLfcBins - 1 && h1 > 0);
    const int v = m0 ? __ffsll((unsigned long long)m0) - 1 : (m1 ? 64 + __ffsll((unsigned long long)m1) - 1 : -1);
    if (v >= 0) fit_leaf = lfc_first_leaf(w, b, slot, V, v);
  }
  if (fit_leaf < 0 && nover > 0) {  // the fit is among the overflow values: min (value, index) scan
    const int32_t lo = max(need, int32_t(kLfcBins - 1));
    uint64_t best = ~0ull;
    for (int i = lane; i < s.N; i += kWave) {
      const int32_t x = V[i];
      if (x >= lo) {
        const uint64_t k = (uint64_t(uint32_t(x)) << 32) | uint32_t(i);
        best = k < best ? k : best;
      }
    }
    best = wave_min_u64(best);
    if (best != ~0ull) fit_leaf = int(uint32_t(best));
  }
  if (fit_leaf >= 0) {
    o.status = KUEUE_TAS_ST_OK;
    o.fit_level = L1;
    if (need != 0) {
      if (lane == 0 && ecap > 0) {
        put_entry(ent, 0, fit_leaf, need);
      }
      o.num_workers = 1;
    }
    return job;
  }
  // greedy (:1278-1318): value mass over bins 1..126, lane owns bins 2*lane, 2*lane+1
  const int b0 = 2 * lane, b1 = 2 * lane + 1;
  const int64_t c0 = (b0 >= 1 && b0 <= kLfcBins - 2) ? int64_t(tot[b0]) : 0;
  const int64_t c1 = (b1 <= kLfcBins - 2) ? int64_t(tot[b1]) : 0;
  const int64_t l0 = c0 * b0, l1 = c1 * b1;
  int64_t x = l0 + l1, y = c0 + c1;
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t xs = int64_t(shfl_u64(uint64_t(x), max(lane - d, 0)));
    const int64_t ys = int64_t(shfl_u64(uint64_t(y), max(lane - d, 0)));
    if (lane >= d) {
      x += xs;
      y += ys;
    }
  }
  const uint64_t hit = ballot(x >= need);
  if (hit) {
    const int src = __ffsll((unsigned long long)hit) - 1;
    const int64_t ex = x - (l0 + l1), ey = y - (c0 + c1);
    int64_t before = ex, below = ey;
    int t = b0;
    if (ex + l0 < need) {
      t = b1;
      before = ex + l0;
      below = ey + c0;
    }
    t = bcast(t, src);
    before = int64_t(bcast64(uint64_t(before), src));
    below = int64_t(bcast64(uint64_t(below), src));
    const int64_t mt = (int64_t(need) - before + t - 1) / t;
    job.t = t;
    job.m = int32_t(mt);
    job.rem_last = int32_t(int64_t(need) - before - (mt - 1) * t);
    o.status = KUEUE_TAS_ST_OK;
    o.fit_level = L1;
    o.num_workers = int32_t(below + mt);
    if (o.num_workers > ecap) o.status = KUEUE_TAS_ST_INTERNAL;
    // work items for lfc_emit_kernel: the chunks holding output, with their
    // output offset (kept leaves in earlier chunks) and first tie rank
    for (int c0 = 0; c0 < b.lfc_nchunks; c0 += kWave) {
      const int ci = c0 + lane;
      int64_t base = 0, nkeep = 0, tb = 0;
      if (ci < b.lfc_nchunks) {
        const int64_t off = (int64_t(slot) * b.lfc_nchunks + ci) * kLfcBins;
        int64_t a = 0, cc = 0;
        for (int v0 = 1; v0 < t; v0 += 8) {  // 8 bins' loads in flight per round trip
          uint32_t pv[8], hv[8];
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const bool in = v0 + k < t;
            pv[k] = in ? b.lfc_cp[off + v0 + k] : 0u;
            hv[k] = in ? b.lfc_ch[off + v0 + k] : 0u;
          }
#pragma unroll
          for (int k = 0; k < 8; k++) {
            a += pv[k];
            cc += hv[k];
          }
        }
        tb = b.lfc_cp[off + t];
        const int64_t tin = b.lfc_ch[off + t];
        int64_t take = mt - tb;
        take = take < 0 ? 0 : (take > tin ? tin : take);
        base = a + (tb < mt ? tb : mt);
        nkeep = cc + take;
      }
      const uint64_t has = ballot(nkeep > 0);
      if (has) {
        int first = 0;
        if (lane == 0) first = atomicAdd(b.lfc_nitems, __popcll(has));
        first = bcast(first, 0);
        if (nkeep > 0) {
          LfcItem it;
          it.eid = w.eid;
          it.chunk = ci;
          it.base = int32_t(base);
          it.tie0 = int32_t(tb);
          b.lfc_items[first + __popcll(has & ((1ull << lane) - 1ull))] = it;
        }
      }
    }
    return job;
  }
  const int64_t bins_mass = int64_t(bcast64(uint64_t(x), 63));
  const int64_t bins_cnt = int64_t(bcast64(uint64_t(y), 63));
  const int64_t total = bins_mass + int64_t(b.lfc_ovtot[slot]);
  if (total < need) {  // not enough capacity: remaining = need - total (:1315-1316)
    not_fit(w, L1, int32_t(total), need, o);
    return job;
  }
  lfc_wide(w, need, V, bins_mass, bins_cnt, o, ent, ecap);
  return job;
}

// findLevelWithFitDomains (:1236-1321).  Returns: 0 ok (results in listA,
// *nres), 1 failure (o filled), 2 finished by the LFC fast path (o filled).
__device__ int find_level(Wave& w, int32_t* results, int* nres, int* fitLevel, kueue_tas_eval_out& o, int32_t* ent,
                          int ent_cap) {
  ProfScope prof_scope_(w, P_FIND);
  const DevSnap& s = g_select_snap;
  const DevEval& ev = *w.ev;
  const bool required = (ev.flags & KUEUE_TAS_F_REQUIRED) != 0;
  const int32_t leaderCount = w.leader ? 1 : 0;
  const int32_t sliceCount = go_div32(ev.count, ev.slice_size);
  int level = ev.requested_level;
  for (;;) {
    const int D = s.level_size[level];
    const int loff = s.level_off[level];
    if (D == 0) {
      o.status = KUEUE_TAS_ST_NO_DOMAINS;
      o.a = level;
      return 1;
    }
    // leaderless BestFit, no multi-layer message: when no domain of the level
    // holds sliceCount the top of the sorted level (max sliceState) does not
    // fit, so the level's outcome needs no scan
    if (w.level_max && !w.leader && w.bf && level < s.L - 1 && !(ev.flags & KUEUE_TAS_F_MULTILAYER)) {
      const int32_t mx = w.level_max[level];
      if (mx < sliceCount) {
        if (required) {
          not_fit(w, level, mx, sliceCount, o);  // notFitMessage(top.sliceState, sliceCount) (:1272-1274)
          return 1;
        }
        if (level > 0 && !w.unconstrained) {  // preferred: one level up (:1275-1277)
          level--;
          continue;
        }
      }
    }
    // sortedDomainsWithLeader: first (top), last, LFC first fit, BF best fit
    Key top = key_max(), lfcfit = key_max(), last = Key{0, 0};
    int32_t minss = 0x7fffffff;
    const bool use_partials = level == s.L - 1 && w.partials != nullptr;
    uint32_t pbst = ~0u;
    Key pbk = key_max();
    if (use_partials) {  // reductions precomputed per fill block
      Key inv = key_max();
      for (int i = lane_id(); i < w.nblk; i += kWave) {
        const LeafPartial& p = w.partials[i];
        top = key_min2(top, p.top);
        inv = key_min2(inv, Key{~p.last.hi, ~p.last.lo});
        lfcfit = key_min2(lfcfit, p.lfcfit);
        minss = min(minss, p.minss);
        pbst = min(pbst, p.bfst);
      }
      top = wave_min_key(top);
      lfcfit = wave_min_key(lfcfit);
      inv = wave_min_key(inv);
      last = Key{~inv.hi, ~inv.lo};
      pbst = uint32_t(wave_min_u64(pbst));
      for (int i = lane_id(); i < w.nblk; i += kWave)
        if (w.partials[i].bfst == pbst) pbk = key_min2(pbk, w.partials[i].bfkey);
      pbk = wave_min_key(pbk);
    } else if (!w.leader) {
      // no leader: the sortedDomainsWithLeader key is (k1(sliceState),
      // s_asc(state), index) under a constant leader part, so lanes compare
      // the packed 64-bit (k1 << 32 | s_asc(state)) and keep the first index
      // (each lane walks its indices in increasing order); the wave then
      // reduces (value, index) pairs.  The level's counters are read 4
      // domains per lane per load (levels start 16-byte aligned), 4 loads per
      // array in flight.  BestFit evals also track findBestFitDomainBy's
      // candidate (:1216-1231: min sliceState >= sliceCount, ties by key) in
      // the same pass; LFC evals the first fit, the last key and the minimum.
      const int4* S4 = reinterpret_cast<const int4*>(w.ctr + loff);
      const int4* SS4 = reinterpret_cast<const int4*>(w.ctr + w.ssoff + loff);
      const int nq = (D + 3) / 4;
      const bool lfc = w.lfc, bf = w.bf;
      uint64_t tv = ~0ull, fv = ~0ull, lv = 0, bv = ~0ull;
      int32_t ti = 0x7fffffff, fi = 0x7fffffff, li = -1, bi = 0x7fffffff;
      constexpr int QU = 4;
      for (int q0 = 0; q0 < nq; q0 += QU * kWave) {
        int4 sa[QU], ssa[QU];
#pragma unroll
        for (int u = 0; u < QU; u++) {
          const int q = min(q0 + u * kWave + lane_id(), nq - 1);
          sa[u] = S4[q];
          ssa[u] = SS4[q];
        }
#pragma unroll
        for (int u = 0; u < QU; u++) {
          const int q = q0 + u * kWave + lane_id();
          const int32_t st4[4] = {sa[u].x, sa[u].y, sa[u].z, sa[u].w};
          const int32_t ss4[4] = {ssa[u].x, ssa[u].y, ssa[u].z, ssa[u].w};
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const int i = 4 * q + k;
            if (q < nq && i < D) {
              const uint32_t lo = s_asc(st4[k]);
              const uint64_t v = (uint64_t(lfc ? s_asc(ss4[k]) : s_desc(ss4[k])) << 32) | lo;
              if (v < tv || (v == tv && i < ti)) {  // the index test only matters for the sentinel
                tv = v;
                ti = i;
              }
              const bool fits = ss4[k] >= sliceCount;
              if (lfc) {
                if (v >= lv) {
                  lv = v;
                  li = i;
                }
                if (fits && (v < fv || (v == fv && i < fi))) {
                  fv = v;
                  fi = i;
                }
                minss = min(minss, ss4[k]);
              }
              if (bf) {
                const uint64_t b = (uint64_t(s_asc(ss4[k])) << 32) | lo;
                if (fits && (b < bv || (b == bv && i < bi))) {
                  bv = b;
                  bi = i;
                }
              }
            }
          }
        }
      }
      wave_argmin(tv, ti);
      const uint64_t lead_hi = uint64_t(s_desc(0)) << 32;
      auto unpack = [&](uint64_t v, int32_t i) {
        return Key{lead_hi | (v >> 32), ((v & 0xffffffffull) << 32) | uint32_t(i)};
      };
      top = unpack(tv, ti);
      if (lfc) {
        wave_argmin(fv, fi);
        wave_argmax(lv, li);
        if (fi != 0x7fffffff) lfcfit = unpack(fv, fi);
        last = unpack(lv, li);
      }
      if (bf) {
        wave_argmin(bv, bi);
        if (bi != 0x7fffffff) pbk = Key{0, uint32_t(bi)};  // best-fit domain index (used below)
      }
    } else {
      bool has_last = false;
      for (int i = lane_id(); i < D; i += kWave) {
        int g = loff + i;
        int32_t ls = w.get(F_LS, g), sswl = w.get(F_SSWL, g), swl = w.get(F_SWL, g), ss = w.get(F_SLICE, g);
        Key k = key_wl(w.lfc, ls, sswl, swl, i);
        if (key_lt(k, top)) top = k;
        if (!has_last || key_lt(last, k)) {
          last = k;
          has_last = true;
        }
        if (ss >= sliceCount && key_lt(k, lfcfit)) lfcfit = k;
        minss = min(minss, ss);
      }
      top = wave_min_key(top);
      lfcfit = wave_min_key(lfcfit);
      Key inv{~last.hi, ~last.lo};
      if (!has_last) inv = key_max();
      inv = wave_min_key(inv);
      last = Key{~inv.hi, ~inv.lo};
    }
    for (int m = 1; m <= 32; m <<= 1) minss = min(minss, xor_lane(minss, m));
    int topg = loff + int(uint32_t(top.lo));
    if (w.bf && w.get(F_SSWL, topg) >= sliceCount && w.get(F_LS, topg) >= leaderCount) {
      // findBestFitDomainForSlices(sorted, sliceCount, leaderCount)
      Field f = leaderCount > 0 ? F_SSWL : F_SLICE;
      if (w.get(f, topg) >= sliceCount) {
        if (use_partials) {
          topg = loff + int(uint32_t(pbk.lo));
        } else if (!w.leader) {
          // found by the scan above (top fits, so a candidate exists)
          topg = loff + int(uint32_t(pbk.lo));
        } else {
          uint32_t bst = ~0u;
          for (int i = lane_id(); i < D; i += kWave) {
            int32_t st = w.get(f, loff + i);
            if (st >= sliceCount && s_asc(st) < bst) bst = s_asc(st);
          }
          bst = uint32_t(wave_min_u64(uint64_t(bst)));
          Key b = key_max();
          for (int i = lane_id(); i < D; i += kWave) {
            int g = loff + i;
            if (s_asc(w.get(f, g)) == bst) {
              Key k = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
              if (key_lt(k, b)) b = k;
            }
          }
          b = wave_min_key(b);
          topg = loff + int(uint32_t(b.lo));
        }
      }
    }
    if (w.lfc) {
      if (!(lfcfit.hi == ~0ull && lfcfit.lo == ~0ull)) {
        results[0] = loff + int(uint32_t(lfcfit.lo));
        *nres = 1;
        *fitLevel = level;
        return 0;
      }
      if (required) {
        not_fit(w, level, w.get(F_STATE, loff + int(uint32_t(last.lo))), sliceCount, o);
        return 1;
      }
    }
    if (w.get(F_SSWL, topg) < sliceCount || w.get(F_LS, topg) < leaderCount) {
      if (required) {
        not_fit(w, level, w.get(F_SLICE, topg), sliceCount, o);
        return 1;
      }
      if (level > 0 && !w.unconstrained) {
        level--;
        continue;
      }
      // ---- greedy over several domains (:1278-1318) ----
      int32_t remS = sliceCount, remL = leaderCount;
      int nr = 0;
      if (D <= w.cap) {
        for (int i = lane_id(); i < D; i += kWave) {
          int g = loff + i;
          w.lds[i] = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
        }
        wave_sync();
        {
          ProfScope ps_(w, P_LDS_SORT);
          lds_sort(w.lds, D, lane_id());
        }
        SeqLds seq{&w, D, loff, 0};
        int idx = 0;
        for (; remL > 0 && idx < D && w.get(F_LS, seq.at(idx)) > 0; idx++) {
          seq.pos = idx;
          int d = seq.at(idx);
          if (w.bf && w.get(F_SSWL, d) >= remS) d = seq.bestfit(remS, remL > 0 ? F_SSWL : F_SLICE);
          results[nr++] = d;
          remL = w_sub(remL, w.get(F_LS, d));
          remS = w_sub(remS, w.get(F_SSWL, d));
        }
        if (remL > 0) {
          not_fit(w, level, w_sub(leaderCount, remL), sliceCount, o);
          wave_sync();
          return 1;
        }
        // re-sort the remainder sortedDomainsWithLeader[idx:] with sortedDomains
        const int nrem = D - idx;
        for (int i = lane_id(); i < nrem; i += kWave) w.gkeys[i] = w.lds[idx + i];
        wave_fence();
        wave_sync();
        for (int i = lane_id(); i < nrem; i += kWave) w.lds[i] = w.kplain(loff + int(uint32_t(w.gkeys[i].lo)));
        wave_sync();
        {
          ProfScope ps_(w, P_LDS_SORT);
          lds_sort(w.lds, nrem, lane_id());
        }
        SeqLds seq2{&w, nrem, loff, 0};
        for (int i = 0; remS > 0 && i < nrem; i++) {
          seq2.pos = i;
          int d = seq2.at(i);
          if (w.bf && w.get(F_SLICE, d) >= remS) d = seq2.bestfit(remS, F_SLICE);
          results[nr++] = d;
          remS = w_sub(remS, w.get(F_SLICE, d));
        }
        wave_sync();
      } else {
        if (w.lfc && !w.leader && level == s.L - 1 && minss >= 0) {
          if (lfc_leaf_greedy(w, sliceCount, o, ent, ent_cap)) return 2;
        }
        // lazy iteration with live keys (no counter mutation inside findLevelWithFitDomains)
        Key lastwl{0, 0};
        bool consumed = false;
        Key cur = top;  // first in WL order
        bool valid = true;
        while (remL > 0 && valid && w.get(F_LS, loff + int(uint32_t(cur.lo))) > 0) {
          int d = loff + int(uint32_t(cur.lo));
          if (w.bf && w.get(F_SSWL, d) >= remS) {
            Field f = remL > 0 ? F_SSWL : F_SLICE;
            if (w.get(f, d) >= remS) {
              uint32_t bst = ~0u;
              for (int i = lane_id(); i < D; i += kWave) {
                int g = loff + i;
                Key k = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
                int32_t st = w.get(f, g);
                if (key_le(cur, k) && st >= remS && s_asc(st) < bst) bst = s_asc(st);
              }
              bst = uint32_t(wave_min_u64(uint64_t(bst)));
              Key b = key_max();
              for (int i = lane_id(); i < D; i += kWave) {
                int g = loff + i;
                Key k = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
                if (key_le(cur, k) && s_asc(w.get(f, g)) == bst && key_lt(k, b)) b = k;
              }
              b = wave_min_key(b);
              d = loff + int(uint32_t(b.lo));
            }
          }
          if (nr < w.lcap) results[nr] = d;
          else w.overflow = true;
          nr++;
          remL = w_sub(remL, w.get(F_LS, d));
          remS = w_sub(remS, w.get(F_SSWL, d));
          lastwl = cur;
          consumed = true;
          // next in WL order
          Key nb = key_max();
          for (int i = lane_id(); i < D; i += kWave) {
            int g = loff + i;
            Key k = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
            if (key_lt(cur, k) && key_lt(k, nb)) nb = k;
          }
          nb = wave_min_key(nb);
          valid = !(nb.hi == ~0ull && nb.lo == ~0ull);
          cur = nb;
        }
        if (remL > 0) {
          not_fit(w, level, w_sub(leaderCount, remL), sliceCount, o);
          return 1;
        }
        // remainder (WL key > lastwl) in sortedDomains order
        Key pc = key_max();
        bool first = true;
        for (;;) {
          if (remS <= 0) break;
          Key nb = key_max();
          for (int i = lane_id(); i < D; i += kWave) {
            int g = loff + i;
            if (consumed) {
              Key kw = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
              if (!key_lt(lastwl, kw)) continue;
            }
            Key kp = w.kplain(g);
            if ((first || key_lt(pc, kp)) && key_lt(kp, nb)) nb = kp;
          }
          nb = wave_min_key(nb);
          if (nb.hi == ~0ull && nb.lo == ~0ull) break;
          first = false;
          pc = nb;
          int d = loff + int(uint32_t(nb.lo));
          if (w.bf && w.get(F_SLICE, d) >= remS) {
            uint32_t bst = ~0u;
            for (int i = lane_id(); i < D; i += kWave) {
              int g = loff + i;
              if (consumed) {
                Key kw = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
                if (!key_lt(lastwl, kw)) continue;
              }
              Key kp = w.kplain(g);
              int32_t st = w.get(F_SLICE, g);
              if (key_le(pc, kp) && st >= remS && s_asc(st) < bst) bst = s_asc(st);
            }
            bst = uint32_t(wave_min_u64(uint64_t(bst)));
            Key b = key_max();
            for (int i = lane_id(); i < D; i += kWave) {
              int g = loff + i;
              if (consumed) {
                Key kw = key_wl(w.lfc, w.get(F_LS, g), w.get(F_SSWL, g), w.get(F_SWL, g), i);
                if (!key_lt(lastwl, kw)) continue;
              }
              Key kp = w.kplain(g);
              if (key_le(pc, kp) && s_asc(w.get(F_SLICE, g)) == bst && key_lt(kp, b)) b = kp;
            }
            b = wave_min_key(b);
            d = loff + int(uint32_t(b.lo));
          }
          if (nr < w.lcap) results[nr] = d;
          else w.overflow = true;
          nr++;
          remS = w_sub(remS, w.get(F_SLICE, d));
        }
      }
      if (remS > 0) {
        not_fit(w, level, w_sub(sliceCount, remS), sliceCount, o);
        return 1;
      }
      *nres = nr;
      *fitLevel = level;
      return 0;
    }
    results[0] = topg;
    *nres = 1;
    *fitLevel = level;
    return 0;
  }
}

// One wave per eval of `ids` (the BestFit-side and the fast-LFC evals are
// launched separately, on two streams).
constexpr int kSelectWaves = 1;  // select_kernel: one wave per block (a small LDS footprint lets blocks start beside other kernels)
constexpr int kFinalWalkLds = 32768;  // BestFit-side LDS bytes per wave (lds_level_walk: ~1,960 candidates)
__global__ __launch_bounds__(256) void select_kernel(DevSnap s, DevBatch b, const int32_t* ids, int nids) {
  extern __shared__ Key lds_all[];
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int slot = blockIdx.x * (blockDim.x >> 6) + wave;
  if (slot >= nids) return;
  const int eid = ids[slot];
  const uint64_t t_begin = wall_clock64();
  const DevEval& ev = b.evals[eid];
  // The wave's descriptor, result header and walk out-parameters live in LDS:
  // the walk's helpers are not inlined and take them by reference, which put
  // them in scratch (400 B/lane, a vector-memory round trip per field read).
  // Every field is wave-uniform (written alike by all lanes).
  __shared__ Wave sh_wave[kSelectWaves];
  __shared__ kueue_tas_eval_out sh_out[kSelectWaves];
  __shared__ int sh_ints[kSelectWaves][4];  // nres, fitLevel, nn
  Wave& w = sh_wave[wave];
  w.ev = &ev;
  w.eid = eid;
  w.leader = (ev.flags & KUEUE_TAS_F_LEADER) != 0;
  w.lfc = (ev.flags & KUEUE_TAS_F_LFC) != 0;
  w.bf = !w.lfc;
  w.unconstrained = (ev.flags & KUEUE_TAS_F_UNCONSTRAINED) != 0;
  w.ctr = ctr_base(b, b.rep_of[eid]);
  w.rack_pos = (b.rack_fanout && b.rack_pos) ? b.rack_pos + int64_t(b.rep_of[eid]) * s.level_size[s.L - 2] : nullptr;
  // per-launch-slot phase-2 buffers: the BestFit-side launch numbers its
  // evals 0..nbf-1; fast-LFC evals (the other launch) never touch them
  SelSlot q{0, 0, 0, 0};  // the fast-LFC launch: no lists, no overlay
  if (b.sel_slots) q = b.sel_slots[b.slot_base + slot];
  w.ov = b.overlay + q.ov_off;
  w.tag = b.tags + int64_t(q.tag_idx) * s.SD;
  w.my_tag = b.tag_epoch;
  w.dirty = false;
  w.SD = s.SD;
  w.ssoff = ss_off(b, b.rep_of[eid], s.SD);
  w.lds = lds_all + int64_t(wave) * (b.wave_lds / int(sizeof(Key)));
  w.cap = b.list_cap;
  w.lds_bytes = b.wave_lds;
  const int64_t lcap = q.lcap;  // 4 int32 lists (2 per u64) + 2 key arrays (2 u64 per key): 6 * lcap u64
  uint64_t* sc = b.scratch + q.scr_off;
  w.lcap = int(lcap);
  w.listA = reinterpret_cast<int32_t*>(sc);
  w.listB = w.listA + lcap;
  w.listC = w.listB + lcap;
  w.listD = w.listC + lcap;
  w.gkeys = reinterpret_cast<Key*>(sc + 2 * lcap);
  w.gkeys2 = w.gkeys + lcap;
  w.overflow = false;
#if KTAS_PROFILE
  for (auto& x : w.prof) x = 0;
#endif
  w.partials = (ev.requested_level == s.L - 1 && b.partial_idx[eid] >= 0)
                   ? b.partials + int64_t(b.partial_idx[eid]) * b.nblk : nullptr;
  w.nblk = b.nblk;
  w.level_max = b.level_max ? b.level_max + int64_t(b.rep_of[eid]) * kMaxLevels : nullptr;
  int32_t* ent = b.entries + int64_t(eid) * b.entry_cap * 2;
  const int ecap = b.entry_cap;

  kueue_tas_eval_out& o = sh_out[wave];
  o.status = KUEUE_TAS_ST_OK;
  o.a = o.b = 0;
  o.fit_level = 0;
  o.num_workers = o.num_leaders = 0;
  o.assignment_nil = 0;
  o.total_nodes = s.n_live;
  o.excl_selector = 0;  // set by the host from the stats region (counted concurrently, stream3)
  o.excl_affinity = 0;
  o.excl_topology = 0;
  for (int c = 0; c < KUEUE_TAS_MAX_LAYERS; c++) o.ml_fit[c] = o.ml_need[c] = 0;
  o.reserved[0] = o.reserved[1] = 0;

#if KTAS_PROFILE
  w.prof[P_SETUP] = wall_clock64() - t_begin;
#endif
  int& nres = sh_ints[wave][0];
  int& fitLevel = sh_ints[wave][1];
  nres = 0;
  fitLevel = 0;
  int r;
  const int lslot = b.lfc_slot[eid];
  if (lslot >= 0) {
    const LfcJob job = lfc_fast(w, b, lslot, o, ent, ecap);
    if (lane == 0) b.lfc_jobs[eid] = job;
    r = 2;
  } else {
    r = find_level(w, w.listA, &nres, &fitLevel, o, ent, ecap);
  }
  const uint64_t t_found = wall_clock64();
  w.dirty = true;  // the descent mutates (overlay)
  if (r == 0) {
    const int L = s.L;
    const int32_t leaderCount = w.leader ? 1 : 0;
    int32_t* cur = w.listB;
    int ncur = 0;
    // currFitDomain = updateCountsToMinimumGeneric(currFitDomain, ...) (:928)
    SeqList seq0{&w, w.listA, nres, 0};
    bool ok = update_counts(w, seq0, ev.count, leaderCount, ev.slice_size, true, cur, &ncur);
    if (!ok) o.assignment_nil = 1;
    int level = fitLevel;
    int32_t* spare = w.listA;
    bool emitted = false;  // the last step wrote the entries itself (lds_level_walk)
    bool cur_lds = false;  // cur's domains are in LDS (lds_walk_chosen), not in the global list
    for (; level < min(L - 1, ev.slice_level); level++) {  // above the slice level (:930-935)
      // leaderless BestFit slice walk with rem > 0: only positive children can be taken
      const bool positive = !w.leader && w.bf && go_div32(ev.count, ev.slice_size) > 0;
      const bool lds_step = positive && ev.slice_level == L - 1 && !w.overflow;
      if (lds_step) {  // the step in LDS
        int nw = 0;
        bool out_lds = false;
        const bool last = level == L - 2;
        const int r = lds_level_walk(w, level, cur, ncur, cur_lds, ev.count, ev.slice_size, last ? ent : nullptr, ecap,
                                     last ? nullptr : spare, &nw, &out_lds);
        if (r >= 0) {
          if (r == 0 || last) {  // entries written, or Go's nil (every later step is empty)
            if (r == 0) o.assignment_nil = 1;
            o.num_workers = r == 0 ? 0 : nw;
            emitted = true;
            level = L - 1;
            break;
          }
          if (!out_lds) {
            int32_t* t = cur;
            cur = spare;
            spare = t;
          }
          cur_lds = out_lds;
          ncur = nw;
          continue;
        }
      }
      if (cur_lds) {  // the generic step reads its parents from the global list
        const int32_t* P = lds_walk_chosen(w);
        for (int i = lane; i < ncur; i += kWave) cur[i] = P[i];
        wave_sync();
        cur_lds = false;
      }
      int32_t* kids = positive ? w.listD : w.listC;
      int nch = positive ? gather_children_positive(w, cur, ncur, level, kids) : gather_children(w, cur, ncur, level, kids);
      int& nn = sh_ints[wave][2];
      nn = 0;
      bool ok2 = walk_sorted(w, kids, nch, level + 1, ev.count, leaderCount, ev.slice_size, true, 0, spare, &nn);
      if (!ok2) o.assignment_nil = 1;
      int32_t* t = cur;
      cur = spare;
      spare = t;
      ncur = nn;
    }
    for (; level < L - 1; level++) {  // at/below the slice level (:937-971)
      int32_t sol = ev.slice_size;
      if (level >= ev.slice_level) {
        sol = 1;
        if (ev.ssal[level + 1] != 0) sol = ev.ssal[level + 1];
      }
      int& nn = sh_ints[wave][2];
      nn = 0;
      const int poff = s.level_off[level];
      for (int i = 0; i < ncur; i++) {
        int d = cur[i];
        int p = d - poff;
        int cb = s.child_off[s.child_base[level] + p];
        int ce = s.child_off[s.child_base[level] + p + 1];
        int nch = ce - cb;
        if (nch > w.lcap) {
          w.overflow = true;
          break;
        }
        for (int j = lane; j < nch; j += kWave) w.listC[j] = s.level_off[level + 1] + cb + j;
        wave_fence();
        bool ok3 = walk_sorted(w, w.listC, nch, level + 1, w.get(F_STATE, d), w.get(F_LS, d), sol, sol > 1, sol, spare,
                               &nn);
        if (!ok3) o.assignment_nil = 1;
      }
      int32_t* t = cur;
      cur = spare;
      spare = t;
      ncur = nn;
    }
    o.fit_level = fitLevel;
    if (emitted) {
    } else if (w.leader) {
      // leaders: copies with state = leaderState (:975-994)
      int nl = 0, nw = 0;
      for (int i = 0; i < ncur; i++) {
        if (w.get(F_LS, cur[i]) > 0) spare[nl++] = cur[i];
        if (w.get(F_STATE, cur[i]) > 0) w.listD[nw++] = cur[i];
      }
      o.num_workers = emit_sorted(w, w.listD, nw, false, false, ent, ecap, 0);
      o.num_leaders = emit_sorted(w, spare, nl, true, true, ent, ecap, o.num_workers);
    } else {
      o.num_workers = emit_sorted(w, cur, ncur, false, false, ent, ecap, 0);
    }
    if (o.num_workers + o.num_leaders > ecap) o.status = KUEUE_TAS_ST_INTERNAL;
  }
  if (w.overflow) o.status = KUEUE_TAS_ST_INTERNAL;
  o.reserved[0] = int32_t(wall_clock64() - t_begin);  // diagnostics: 100 MHz ticks in select,
  o.reserved[1] = int32_t(t_found - t_begin);         // of which findLevelWithFitDomains
  if (lane == 0) b.out[eid] = o;
#if KTAS_PROFILE
  if (lane == 0 && b.prof)
    for (int k = 0; k < P_NCAT; k++) b.prof[int64_t(eid) * P_NCAT + k] = int32_t(w.prof[k]);
#endif
}

// Expand fast-LFC greedy results (LfcJob) into (leaf, count) entries in leaf
// index order.  Persistent grid over the (eval, chunk) items select appended:
// one kLfcChunk-leaf chunk per item; its output offset and first tie rank
// come with the item, in-chunk positions from block scans.
__global__ __launch_bounds__(256) void lfc_emit_kernel(DevSnap s, DevBatch b) {
  __shared__ int32_t sh_wt[4], sh_wk[4];
  const int nitems = *b.lfc_nitems;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  for (int itx = blockIdx.x; itx < nitems; itx += gridDim.x) {
    const LfcItem item = b.lfc_items[itx];
    const int eid = item.eid;
    const LfcJob job = b.lfc_jobs[eid];
    const int slot = b.lfc_slot[eid];
    const int t = job.t;
    const int64_t mt = job.m;
    const int32_t* V = ctr_base(b, b.lfc_rep[slot]) + ss_off(b, b.lfc_rep[slot], s.SD) +
                       s.level_off[s.L - 1];
    const int lo = item.chunk * kLfcChunk + int(threadIdx.x) * 8;
    int32_t x[8];
    if (t < 255) {  // the byte copy decides every leaf: >= 255 is above the threshold
      // (the copy holds 0 past the last leaf: a full chunk of bytes per slot)
      const uint64_t w = *reinterpret_cast<const uint64_t*>(b.lfc_u8 + int64_t(slot) * b.lfc_nchunks * kLfcChunk + lo);
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = (lo + k < s.N) ? int32_t((w >> (8 * k)) & 0xffu) : 0;
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = (lo + k < s.N) ? V[lo + k] : 0;
    }
    int nt = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) nt += x[k] == t ? 1 : 0;
    int wt_total;
    const int tex = wave_excl_scan(nt, &wt_total);
    if (lane == 0) sh_wt[wv] = wt_total;
    __syncthreads();
    int64_t r = int64_t(item.tie0) + tex;
    for (int k = 0; k < wv; k++) r += sh_wt[k];
    bool keep[8];
    int nk = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const bool tie = x[k] == t;
      keep[k] = (x[k] > 0 && x[k] < t) || (tie && r < mt);
      if (tie) {
        if (r == mt - 1) x[k] = job.rem_last;
        r++;
      }
      nk += keep[k] ? 1 : 0;
    }
    int wk_total;
    const int kex = wave_excl_scan(nk, &wk_total);
    if (lane == 0) sh_wk[wv] = wk_total;
    __syncthreads();
    int64_t pos = int64_t(item.base) + kex;
    for (int k = 0; k < wv; k++) pos += sh_wk[k];
    int32_t* ent = b.entries + int64_t(eid) * b.entry_cap * 2;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (keep[k]) {
        if (pos < b.entry_cap && !(b.exp_flags & 1)) {
          put_entry(ent, pos, lo + k, x[k]);
        }
        pos++;
      }
    }
    __syncthreads();  // sh_wt / sh_wk reused by the next item
  }
}

// Snapshot delta: tas_usage[col][leaf] += delta (updateTASUsage :257-293)
// With `shadow` set the host mirror already holds these deltas (a host-layer
// AddUsage / RemoveUsage): the mirror's shadow takes them too, so the next
// diff (usage_diff_kernel) reports only what the device applied on its own.
__global__ void apply_deltas_kernel(int64_t* tas_usage, uint32_t* usage_present, int N, const kueue_tas_delta* d,
                                    int n, int64_t* shadow, uint32_t* pshadow) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  kueue_tas_delta x = d[i];
  const int64_t at = int64_t(x.col) * N + x.leaf;
  atomicAdd(reinterpret_cast<unsigned long long*>(&tas_usage[at]), (unsigned long long)(uint64_t(x.delta)));
  atomicOr(&usage_present[x.leaf], 1u << x.col);
  if (shadow) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&shadow[at]), (unsigned long long)(uint64_t(x.delta)));
    atomicOr(&pshadow[x.leaf], 1u << x.col);
  }
}

// Leaf free-capacity rows replaced after non-TAS pod events
// (nonTasUsageCache.update/delete, tas_non_tas_pod_cache.go:46-87, folded in by
// TASFlavorCache.snapshot, tas_flavor.go:133-137): one thread per (leaf, column),
// column-major stores so a wave writes one column of 64 leaves.
// Host-mirror diff (kueue_tas_snapshot_usage_changes): every (column, leaf)
// whose usage or presence bit differs from the shadow, with its value.
__global__ void usage_diff_kernel(const int64_t* usage, const uint32_t* present, const int64_t* shadow,
                                  const uint32_t* pshadow, int N, int R, kueue_tas_delta* out, int32_t* count) {
  const int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= int64_t(N) * R) return;
  const int col = int(idx / N), leaf = int(idx % N);
  const int64_t v = usage[idx];
  const bool p = (present[leaf] >> col) & 1u, ps = (pshadow[leaf] >> col) & 1u;
  if (v != shadow[idx] || p != ps) {
    const int k = atomicAdd(count, 1);
    out[k] = kueue_tas_delta{leaf, col, v};
  }
}

__global__ void set_free_kernel(int64_t* free_cap, uint32_t* free_present, int N, int R, const int32_t* leaves,
                                const int64_t* rows, const uint32_t* present, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int leaf = leaves[i];
  for (int col = 0; col < R; col++) free_cap[int64_t(col) * N + leaf] = rows[int64_t(i) * R + col];
  free_present[leaf] = present[i];
}

// Leaf taint profile and selector label columns replaced after in-place node
// updates (nodesCache.sync, tas_nodes_cache.go:38-50).
__global__ void set_leaf_attrs_kernel(int32_t* taint_profile, int32_t* label_values, int N, int K,
                                      const int32_t* leaves, const int32_t* profiles, const int32_t* labels, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int leaf = leaves[i];
  if (taint_profile) taint_profile[leaf] = profiles[i];
  if (label_values)
    for (int k = 0; k < K; k++) label_values[int64_t(k) * N + leaf] = labels[int64_t(i) * K + k];
}

// kueue_tas_snapshot_splice: every leaf of the new numbering takes its
// columns from its old index (src >= 0) or from joined row -src-1.
__global__ void splice_leaves_kernel(const int32_t* gsrc, int n_new, int n_old, int R, int K, int num_new,
                                     const int64_t* of, const int64_t* ou, const uint32_t* ofp, const uint32_t* oup,
                                     const int32_t* oprof, const int32_t* olab, const int64_t* nf, const int64_t* nu,
                                     const uint32_t* nfp, const uint32_t* nup, const int32_t* nprof, const int32_t* nlab,
                                     int64_t* f, int64_t* u, uint32_t* fp, uint32_t* up, int32_t* prof, int32_t* lab,
                                     const uint64_t* otag, const uint64_t* ntag, uint64_t* tag) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_new) return;
  const int src = gsrc[j];
  if (tag) tag[j] = src >= 0 ? otag[src] : ntag[-src - 1];
  if (src >= 0) {
    for (int c = 0; c < R; c++) {
      f[int64_t(c) * n_new + j] = of[int64_t(c) * n_old + src];
      u[int64_t(c) * n_new + j] = ou[int64_t(c) * n_old + src];
    }
    fp[j] = ofp[src];
    up[j] = oup[src];
    if (prof) prof[j] = oprof ? oprof[src] : 0;
    for (int k = 0; k < K; k++) lab[int64_t(k) * n_new + j] = olab[int64_t(k) * n_old + src];
  } else {
    const int k0 = -src - 1;
    for (int c = 0; c < R; c++) {
      f[int64_t(c) * n_new + j] = nf[int64_t(c) * num_new + k0];
      u[int64_t(c) * n_new + j] = nu[int64_t(c) * num_new + k0];
    }
    fp[j] = nfp[k0];
    up[j] = nup[k0];
    if (prof) prof[j] = nprof ? nprof[k0] : 0;
    for (int k = 0; k < K; k++) lab[int64_t(k) * n_new + j] = nlab[int64_t(k) * num_new + k0];
  }
}

// A load's parent tables from the CSR child offsets (one thread per padded
// domain slot, a binary search in its parent level's offsets): the global
// parent id of every domain (-1 for roots and padding; the v1beta2 leaf-mode
// encoder) and, when asked, each leaf's parent index within its level (the
// ragged fills' segmented scans).
__global__ void domain_parents_kernel(DevSnap s, int32_t* parent, int32_t* leaf_parent) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= s.SD) return;
  int l = 0;
  while (l + 1 < s.L && g >= s.level_off[l + 1]) l++;
  const int i = g - s.level_off[l];
  int p = -1;
  if (l > 0 && i < s.level_size[l]) {
    const int32_t* co = s.child_off + s.child_base[l - 1];
    int lo = 0, hi = s.level_size[l - 1];  // the last parent q with co[q] <= i
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (co[mid] <= i) lo = mid;
      else hi = mid;
    }
    p = lo;
    if (leaf_parent && l == s.L - 1) leaf_parent[i] = p;
  }
  parent[g] = p < 0 ? -1 : s.level_off[l - 1] + p;
}

__global__ void set_leaf_dead_kernel(uint8_t* dead, const int32_t* leaves_live, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dead[leaves_live[2 * i]] = leaves_live[2 * i + 1] ? 0 : 1;
}

// ---- v1beta2 compact encoding (pkg/util/tas/tas_assignment.go:135-259) ----
// fillSingleCompactSliceValues walks the values keeping a running prefix and
// suffix of value 0; by induction the prefix after value i is value0's prefix
// of length min_{j<=i} lcp(value0, value_j) (each step cuts it to the first
// mismatch or to len(value_i) <= which lcp is bounded), and likewise for the
// suffix.  So the walk is a min-reduction of per-value lcp / lcs lengths,
// done by one block per (assignment, level) over its domains.
struct EncodeArgs {
  const char* bytes;
  const int64_t* str_off;
  const int32_t* ids;     // explicit mode: [domain][num_levels] string ids (null: leaf mode)
  const int32_t* counts;  // explicit mode counts
  const int32_t* pairs;   // leaf mode: (leaf, count)
  const int32_t* parent;  // leaf mode: parent global domain id, [SD]
  const int64_t* off;     // [n_assign + 1]
  int32_t n_assign;
  int32_t num_levels;
  int32_t first_level;
  int32_t L;
  int32_t level_off[kMaxLevels];
  int64_t name_base[kMaxLevels];  // string id of level l's domain 0
  kueue_tas_level_enc* out;
  int32_t* same;
};

__device__ __forceinline__ int64_t enc_string_id(const EncodeArgs& a, int64_t j, int k) {
  if (a.ids) return a.ids[j * a.num_levels + k];
  const int lvl = a.first_level + k;
  int32_t g = a.level_off[a.L - 1] + a.pairs[2 * j];
  for (int l = a.L - 1; l > lvl; l--) g = a.parent[g];
  return a.name_base[lvl] + (g - a.level_off[lvl]);
}

__global__ __launch_bounds__(256) void encode_v1beta2_kernel(EncodeArgs a) {
  __shared__ int32_t red[4][4];
  __shared__ int32_t same_red[4];
  const int asg = blockIdx.x, k = blockIdx.y;
  const int64_t j0 = a.off[asg], j1 = a.off[asg + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (j1 <= j0) {
    if (threadIdx.x == 0) {
      a.out[int64_t(asg) * a.num_levels + k] = kueue_tas_level_enc{0, 0, 0, -1};
      if (k == 0) a.same[asg] = 0;
    }
    return;
  }
  const int64_t id0 = enc_string_id(a, j0, k);
  const char* s0 = a.bytes + a.str_off[id0];
  const int32_t len0 = int32_t(a.str_off[id0 + 1] - a.str_off[id0]);
  const int32_t c0 = a.ids ? a.counts[j0] : a.pairs[2 * j0 + 1];
  int32_t P = len0, S = len0, mn = len0, mx = len0, same = 1;
  for (int64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
    const int64_t id = enc_string_id(a, j, k);
    const char* sj = a.bytes + a.str_off[id];
    const int32_t lj = int32_t(a.str_off[id + 1] - a.str_off[id]);
    mn = min(mn, lj);
    mx = max(mx, lj);
    const int32_t m = min(min(len0, lj), P);  // lcp beyond the running minimum cannot lower it
    int32_t p = 0;
    while (p < m && sj[p] == s0[p]) p++;
    P = min(P, p);
    const int32_t ms = min(min(len0, lj), S);
    int32_t q = 0;
    while (q < ms && sj[lj - 1 - q] == s0[len0 - 1 - q]) q++;
    S = min(S, q);
    if (k == 0) same &= (a.ids ? a.counts[j] : a.pairs[2 * j + 1]) == c0;
  }
  for (int d = 1; d <= 32; d <<= 1) {
    P = min(P, xor_lane(P, d));
    S = min(S, xor_lane(S, d));
    mn = min(mn, xor_lane(mn, d));
    mx = max(mx, xor_lane(mx, d));
    same &= xor_lane(same, d);
  }
  if (lane == 0) {
    red[wave][0] = P;
    red[wave][1] = S;
    red[wave][2] = mn;
    red[wave][3] = mx;
    same_red[wave] = same;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int w = 1; w < nw; w++) {
      P = min(P, red[w][0]);
      S = min(S, red[w][1]);
      mn = min(mn, red[w][2]);
      mx = max(mx, red[w][3]);
      same &= same_red[w];
    }
    kueue_tas_level_enc e{0, 0, 0, int32_t(id0)};
    if (P == mx) {  // all values equal (:174-178)
      e.universal = 1;
    } else {
      if (P + S > mn) P = mn - S;  // no prefix/suffix overlap (:180-184)
      e.prefix_len = P;
      e.suffix_len = S;
    }
    a.out[int64_t(asg) * a.num_levels + k] = e;
    if (k == 0) a.same[asg] = same;
  }
}

// TASFlavorSnapshot.Fits (tas_flavor_snapshot.go:401-415), one thread per
// TopologyDomainRequests record: remaining = freeCapacity - tasUsage (keys of
// either map present, requests.go:84-94), then SinglePodRequests.CountIn
// (requests.go:174-217: a missing key with a non-zero request gives 0, a zero
// request MaxInt32, else max(int32(cap / req), 0); no keys gives 0).  Admission
// re-checks are a handful of records per call: plain int64 division.
__global__ void fits_kernel(DevSnap s, const kueue_tas_fits_req* reqs, int n, const kueue_tas_fits_term* terms,
                            int32_t* fits) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const kueue_tas_fits_req r = reqs[i];
  if (r.leaf < 0 || r.leaf >= s.N || leaf_out(s, r.leaf)) {
    fits[i] = 0;
    return;
  }
  const uint32_t pres = s.free_present[r.leaf] | s.usage_present[r.leaf];
  int32_t result = 0;
  bool any = false;
  for (int k = 0; k < r.num_terms; k++) {
    const kueue_tas_fits_term t = terms[r.term_begin + k];
    const bool present = t.col >= 0 && ((pres >> t.col) & 1u);
    int32_t c;
    if (!present && t.value != 0) {
      result = 0;
      any = true;
      break;
    }
    if (t.value == 0) {
      c = 0x7fffffff;
    } else {
      const int64_t cap = int64_t(uint64_t(s.free_cap[int64_t(t.col) * s.N + r.leaf]) -
                                  uint64_t(s.tas_usage[int64_t(t.col) * s.N + r.leaf]));
      const int64_t q = (cap == INT64_MIN && t.value == -1) ? INT64_MIN : cap / t.value;
      c = max(int32_t(uint32_t(uint64_t(q))), 0);
    }
    if (!any || c < result) result = c;
    any = true;
  }
  fits[i] = (any ? result : 0) >= r.count ? 1 : 0;
}

// Sequential admission over a batch of nominated workloads: the TAS half of
// Scheduler.processEntry (pkg/scheduler/scheduler.go:371-435) per workload in
// order: ClusterQueueSnapshot.Fits -> TASFlavorSnapshot.Fits
// (tas_flavor_snapshot.go:401-415: every record's SinglePodRequests.CountIn
// of free - tasUsage >= Count, no pods:1) against the usage of the workloads
// admitted before it, then AddUsage -> updateTASUsage (:257-265: per record
// single x count plus pods:count added to the leaf's tasUsage, keys created).
// One wave walks the workloads in order (the dependency chain); its lanes
// split a workload's records.  tas_usage / usage_present are read with
// L1-bypassing loads because this wave's own atomics updated them, and the
// atomics return values the wave consumes, so each admitted workload's
// updates have completed before the next workload's loads issue (no
// __threadfence: that costs microseconds per call on gfx950).
__device__ __forceinline__ int64_t load_l2(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t load_l2(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// CountIn of one record against free - usage (requests.go:174-217, no pods:1):
// terms are loaded first, then every capacity load issues at once (the loop
// Go breaks out of is evaluated on registers), kAdmitTerms per pass.
constexpr int kAdmitTerms = 8;
__device__ __forceinline__ bool admit_record_fits(const DevSnap& s, const int64_t* tas_usage,
                                                  const uint32_t* usage_present, const kueue_tas_fits_req& r,
                                                  const kueue_tas_fits_term* terms) {
  if (r.leaf < 0 || r.leaf >= s.N || leaf_out(s, r.leaf)) return false;
  const uint32_t pres = s.free_present[r.leaf] | load_l2(usage_present + r.leaf);
  int32_t result = 0;
  bool any = false;
  for (int k0 = 0; k0 < r.num_terms; k0 += kAdmitTerms) {
    int32_t col[kAdmitTerms];
    int64_t val[kAdmitTerms], fc[kAdmitTerms], us[kAdmitTerms];
#pragma unroll
    for (int u = 0; u < kAdmitTerms; u++) {
      col[u] = -1;
      val[u] = 0;
      if (k0 + u < r.num_terms) {
        const kueue_tas_fits_term t = terms[r.term_begin + k0 + u];
        col[u] = t.col;
        val[u] = t.value;
      }
    }
#pragma unroll
    for (int u = 0; u < kAdmitTerms; u++) {
      fc[u] = us[u] = 0;
      if (col[u] >= 0) {
        fc[u] = s.free_cap[int64_t(col[u]) * s.N + r.leaf];
        us[u] = load_l2(tas_usage + int64_t(col[u]) * s.N + r.leaf);
      }
    }
#pragma unroll
    for (int u = 0; u < kAdmitTerms; u++) {
      if (k0 + u >= r.num_terms) break;
      const bool present = col[u] >= 0 && ((pres >> col[u]) & 1u);
      if (!present && val[u] != 0) return 0 >= r.count;  // CountIn: a missing resource fits 0 (:200-203)
      int32_t c = 0x7fffffff;
      if (val[u] != 0) {
        const int64_t cap = int64_t(uint64_t(fc[u]) - uint64_t(us[u]));
        const int64_t q = (cap == INT64_MIN && val[u] == -1) ? INT64_MIN : cap / val[u];
        c = max(int32_t(uint32_t(uint64_t(q))), 0);
      }
      if (!any || c < result) result = c;
      any = true;
    }
  }
  return (any ? result : 0) >= r.count;
}

// One admission record as phase 1 leaves it for the in-order pass: the
// record's terms with, per term, the largest tasUsage at which it still fits
// (`lim` = free - count x value: CountIn(free - usage) >= count <=> usage <=
// lim for every term once nothing wraps and no quotient leaves int32, which
// phase 1 verifies for the whole call, else `exact`).
struct AdmitRec {
  int32_t leaf, count;
  int32_t status;  // kAdmitCheck / kAdmitAlways / kAdmitNever / kAdmitWide
  int32_t nt;
  int32_t col[kAdmitTerms];
  int64_t val[kAdmitTerms];
  int64_t lim[kAdmitTerms];
};
constexpr int32_t kAdmitCheck = 0;   // fits now; re-check (usage <= lim) once its leaf is touched
constexpr int32_t kAdmitAlways = 1;  // count <= 0: CountIn >= 0 >= count
constexpr int32_t kAdmitNever = 2;   // does not fit now, so never later in the call (usage only grows)
constexpr int32_t kAdmitWide = 3;    // more than kAdmitTerms terms: generic re-check

// Phase 1 (parallel over every record of the call): the record's fit
// against the usage at the start of the call; a workload with a record that
// does not fit cannot fit after more usage is added.  `exact` = 1 when the
// shortcuts do not hold for some record (a capacity, usage or count x value
// of 2^61 or more, a quotient outside int32 at the start or after the call's
// total additions `total[col]` to the column); the in-order pass then
// re-checks everything.
__global__ __launch_bounds__(256) void admit_fit0_kernel(DevSnap s, const int64_t* tas_usage,
                                                         const uint32_t* usage_present, const kueue_tas_fits_req* reqs,
                                                         const kueue_tas_fits_term* terms, const int32_t* rec_wl, int n,
                                                         const int64_t* total, int32_t* wl_fit0, AdmitRec* recs,
                                                         int32_t* exact) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const kueue_tas_fits_req r = reqs[i];
  const bool fits = admit_record_fits(s, tas_usage, usage_present, r, terms);
  if (!fits) atomicAnd(wl_fit0 + rec_wl[i], 0);
  AdmitRec a;
  a.leaf = r.leaf;
  a.count = r.count;
  a.nt = r.num_terms;
  a.status = r.count <= 0 ? kAdmitAlways : !fits ? kAdmitNever : r.num_terms > kAdmitTerms ? kAdmitWide : kAdmitCheck;
  bool bad = false;
  constexpr int64_t kBig = int64_t(1) << 61;
#pragma unroll
  for (int u = 0; u < kAdmitTerms; u++) {
    a.col[u] = -1;
    a.val[u] = 0;
    a.lim[u] = 0;
    if (u < r.num_terms && r.leaf >= 0 && r.leaf < s.N) {
      const kueue_tas_fits_term t = terms[r.term_begin + u];
      a.col[u] = t.col;
      a.val[u] = t.value;
      if (a.status == kAdmitCheck && t.col >= 0 && t.value > 0) {
        const int64_t f = s.free_cap[int64_t(t.col) * s.N + r.leaf], us = tas_usage[int64_t(t.col) * s.N + r.leaf];
        bad |= f >= kBig || f <= -kBig || us >= kBig || us <= -kBig || t.value > kBig / r.count;
        if (!bad) {
          const int64_t q0 = (f - us) / t.value, q1 = (f - us - total[t.col]) / t.value;
          bad |= q0 >= (int64_t(1) << 31) || q1 <= -(int64_t(1) << 31);
          a.lim[u] = f - int64_t(r.count) * t.value;
        }
      }
    }
  }
  recs[i] = a;
  if (bad) atomicOr(exact, 1);
}

// Phase 1b (parallel): the order of admission only matters between
// candidates that share a leaf.  minc[leaf] is the first phase-1 fitting
// candidate with a record on the leaf; a fitting candidate that is minc of
// every one of its leaves shares no leaf with an earlier fitting candidate,
// so no earlier admission can change its verdict (only a fitting candidate
// is ever admitted): it is admitted here — its usage added in parallel, its
// leaves marked touched for the re-checks of later candidates that share
// them — and only the other ("dependent") candidates go through the in-order
// window kernel, compacted (admit_todo_kernel).  Adding a later independent
// candidate's usage before an earlier dependent one is decided changes
// nothing for the earlier one: by construction they share no leaf.
__global__ __launch_bounds__(256) void admit_minc_kernel(const kueue_tas_fits_req* reqs, const int32_t* rec_wl, int n,
                                                         const int32_t* wl_fit0, int N, int32_t* minc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t leaf = reqs[i].leaf, w = rec_wl[i];
  if (leaf >= 0 && leaf < N && wl_fit0[w] != 0) atomicMin(minc + leaf, w);
}
__global__ __launch_bounds__(256) void admit_dep_kernel(const kueue_tas_fits_req* reqs, const int32_t* rec_wl, int n,
                                                        const int32_t* wl_fit0, int N, const int32_t* minc,
                                                        int32_t* dep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t leaf = reqs[i].leaf, w = rec_wl[i];
  if (leaf >= 0 && leaf < N && wl_fit0[w] != 0 && minc[leaf] != w) dep[w] = 1;  // (same value from every writer)
}
__global__ __launch_bounds__(256) void admit_indep_kernel(DevSnap s, int64_t* tas_usage, uint32_t* usage_present,
                                                          const kueue_tas_fits_req* reqs, const kueue_tas_fits_term* terms,
                                                          const int32_t* rec_wl, int n, const int32_t* wl_fit0,
                                                          const int32_t* dep, int pods_col, uint32_t* touched) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int w = rec_wl[i];
  if (wl_fit0[w] == 0 || dep[w] != 0) return;
  const kueue_tas_fits_req r = reqs[i];
  if (r.leaf < 0 || r.leaf >= s.N) return;  // (a fitting candidate's leaves are valid)
  uint32_t bits = 0;
  for (int q = 0; q < r.num_terms; q++) {
    const kueue_tas_fits_term t = terms[r.term_begin + q];
    if (t.col >= 0) {
      atomicAdd(reinterpret_cast<unsigned long long*>(tas_usage + int64_t(t.col) * s.N + r.leaf),
                (unsigned long long)(uint64_t(t.value) * uint64_t(int64_t(r.count))));
      bits |= 1u << t.col;
    }
  }
  if (pods_col >= 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(tas_usage + int64_t(pods_col) * s.N + r.leaf),
              (unsigned long long)int64_t(r.count));
    bits |= 1u << pods_col;
  }
  atomicOr(usage_present + r.leaf, bits);
  atomicOr(touched + (r.leaf >> 5), 1u << (r.leaf & 31));
}
// One workgroup: the verdicts decided so far (phase-1 failures 0,
// independent candidates 1) and the rest — every candidate in exact mode —
// compacted in order into todo[1 ..], todo[0] = their count, and their
// record ranges into todo_r[2 j], todo_r[2 j + 1].
__global__ __launch_bounds__(1024) void admit_todo_kernel(int n_wl, const int32_t* wl_fit0, const int32_t* dep,
                                                          int exact, int32_t* admitted, int32_t* todo,
                                                          const int64_t* wl_off, int64_t* todo_r) {
  __shared__ int32_t sh_wave[16];
  const int lane = lane_id(), wave = int(threadIdx.x) >> 6;
  int32_t base = 0;
  for (int c0 = 0; c0 < n_wl; c0 += int(blockDim.x)) {  // block-uniform
    const int w = c0 + int(threadIdx.x);
    bool flag = false;
    if (w < n_wl) {
      flag = exact != 0 || (wl_fit0[w] != 0 && dep[w] != 0);
      if (!flag) admitted[w] = wl_fit0[w] != 0 ? 1 : 0;
    }
    const uint64_t m = ballot(flag);
    const int32_t below = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) sh_wave[wave] = __popcll(m);
    __syncthreads();
    int32_t off = base, total = 0;
    for (int k = 0; k < int(blockDim.x) >> 6; k++) {
      if (k < wave) off += sh_wave[k];
      total += sh_wave[k];
    }
    if (flag) {
      const int j = off + below;
      todo[1 + j] = w;
      todo_r[2 * j] = wl_off[w];  // its record range: one load level less in the window kernel
      todo_r[2 * j + 1] = wl_off[w + 1];
    }
    base += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) todo[0] = base;
}

// Phase 2: one wave walks the workloads in order (the dependency chain), its
// lanes splitting a workload's records.  A workload whose phase-1 fit failed
// is rejected at once; one that fitted is re-checked (usage <= lim, with
// L1-bypassing loads) only on the leaves an earlier workload of this call was
// admitted onto (`touched`, one bit per leaf, in LDS when it fits).  The
// next candidate's first 64 records are fetched while the current one is
// decided.  Admission adds the usage with returning atomics (all issued, then
// consumed), so they have completed before a later re-check's loads issue
// (no __threadfence: that costs microseconds per call on gfx950).
__device__ __forceinline__ bool admit_touched(const uint32_t* lds, const uint32_t* glob, bool in_lds, int32_t leaf) {
  const uint32_t word = in_lds ? lds[leaf >> 5] : load_l2(glob + (leaf >> 5));
  return (word >> (leaf & 31)) & 1u;
}

__global__ __launch_bounds__(64) void admit_kernel(DevSnap s, int64_t* tas_usage, uint32_t* usage_present,
                                                   const kueue_tas_fits_req* reqs, const kueue_tas_fits_term* terms,
                                                   const AdmitRec* recs, const int64_t* wl_off, int n_wl, int pods_col,
                                                   const int32_t* wl_fit0, const int32_t* exact_flag,
                                                   uint32_t* touched_global, int touched_in_lds, int32_t* admitted) {
  extern __shared__ uint32_t touched_lds[];
  const int lane = lane_id();
  if (touched_in_lds) {  // (the global bitmap is cleared by the host)
    for (int k = lane; k < (s.N + 31) / 32; k += kWave) touched_lds[k] = 0;
    wave_sync();
  }
  const bool exact = *exact_flag != 0;
  const bool in_lds = touched_in_lds != 0;
  unsigned long long sink = 0;
  AdmitRec nxt;
  int nxt_w = -1;
  for (int w0 = 0; w0 < n_wl; w0 += kWave) {
    // 64 workloads' phase-1 results and offsets per load
    const int wl = min(w0 + lane, n_wl - 1);
    const bool my_cand = wl_fit0[wl] != 0 || exact;
    const int64_t my_r0 = wl_off[wl], my_r1 = wl_off[wl + 1];
    const uint64_t cands = ballot(my_cand && w0 + lane < n_wl);
    const int wend = min(w0 + kWave, n_wl);
    for (int w = w0; w < wend; w++) {
      if (!((cands >> (w - w0)) & 1ull)) {
        if (lane == 0) admitted[w] = 0;
        continue;
      }
      const int64_t r0 = int64_t(shfl_u64(uint64_t(my_r0), w - w0)), r1 = int64_t(shfl_u64(uint64_t(my_r1), w - w0));
      AdmitRec cur;
      if (nxt_w == w) cur = nxt;
      else if (r0 + lane < r1) cur = recs[r0 + lane];
      // fetch the next candidate of this block while this one is decided
      const uint64_t later = (w - w0 + 1 < kWave) ? cands & (~0ull << (w - w0 + 1)) : 0ull;
      nxt_w = -1;
      if (later) {
        const int nw = w0 + __builtin_ctzll(later);
        const int64_t n0 = int64_t(shfl_u64(uint64_t(my_r0), nw - w0)), n1 = int64_t(shfl_u64(uint64_t(my_r1), nw - w0));
        if (n0 + lane < n1) nxt = recs[n0 + lane];
        nxt_w = nw;
      }
      bool all_fit = true;
      for (int64_t base = r0; base < r1 && all_fit; base += kWave) {
        const int64_t i = base + lane;
        bool fit = true;
        if (i < r1) {
          const AdmitRec a = base == r0 ? cur : recs[i];
          if (exact || a.status == kAdmitWide) {
            fit = admit_record_fits(s, tas_usage, usage_present, reqs[i], terms);
          } else if (a.status == kAdmitNever) {
            fit = false;
          } else if (a.status == kAdmitCheck && admit_touched(touched_lds, touched_global, in_lds, a.leaf)) {
            int64_t us[kAdmitTerms];
#pragma unroll
            for (int u = 0; u < kAdmitTerms; u++)
              us[u] = (a.col[u] >= 0 && a.val[u] > 0) ? load_l2(tas_usage + int64_t(a.col[u]) * s.N + a.leaf) : 0;
#pragma unroll
            for (int u = 0; u < kAdmitTerms; u++) fit &= !(a.col[u] >= 0 && a.val[u] > 0) || us[u] <= a.lim[u];
          }
        }
        all_fit = ballot(!fit) == 0;
      }
      if (lane == 0) admitted[w] = all_fit ? 1 : 0;
      if (!all_fit) continue;
      for (int64_t base = r0; base < r1; base += kWave) {
        const int64_t i = base + lane;
        if (i >= r1) continue;
        const kueue_tas_fits_req r = reqs[i];
        uint32_t bits = 0;
        for (int k0 = 0; k0 < r.num_terms; k0 += kAdmitTerms) {
          int32_t col[kAdmitTerms];
          int64_t val[kAdmitTerms];
          unsigned long long ret[kAdmitTerms];
          if (k0 == 0 && base == r0 && !exact && cur.status != kAdmitWide) {
#pragma unroll
            for (int u = 0; u < kAdmitTerms; u++) {
              col[u] = cur.col[u];
              val[u] = cur.val[u];
            }
          } else {
#pragma unroll
            for (int u = 0; u < kAdmitTerms; u++) {
              col[u] = -1;
              val[u] = 0;
              if (k0 + u < r.num_terms) {
                const kueue_tas_fits_term t = terms[r.term_begin + k0 + u];
                col[u] = t.col;
                val[u] = t.value;
              }
            }
          }
#pragma unroll
          for (int u = 0; u < kAdmitTerms; u++) {
            ret[u] = 0;
            if (col[u] >= 0) {  // the host gives every usage resource a column first
              ret[u] = atomicAdd(reinterpret_cast<unsigned long long*>(tas_usage + int64_t(col[u]) * s.N + r.leaf),
                                 (unsigned long long)(uint64_t(val[u]) * uint64_t(int64_t(r.count))));
              bits |= 1u << col[u];
            }
          }
#pragma unroll
          for (int u = 0; u < kAdmitTerms; u++) sink += ret[u];
        }
        unsigned long long rp = 0, rb;
        if (pods_col >= 0) {
          rp = atomicAdd(reinterpret_cast<unsigned long long*>(tas_usage + int64_t(pods_col) * s.N + r.leaf),
                         (unsigned long long)int64_t(r.count));
          bits |= 1u << pods_col;
        }
        rb = atomicOr(usage_present + r.leaf, bits);
        if (in_lds) atomicOr(touched_lds + (r.leaf >> 5), 1u << (r.leaf & 31));
        else rb += atomicOr(touched_global + (r.leaf >> 5), 1u << (r.leaf & 31));
        sink += rp + rb;
      }
      wave_sync();
    }
  }
  if (lane == 0) admitted[n_wl] = int32_t(uint32_t(sink));
}

// Windowed optimistic admission (the same decisions as admit_kernel: the
// TAS half of Scheduler.processEntry, scheduler.go:371-435, per workload in
// order, Fits tas_flavor_snapshot.go:401-415 then AddUsage :257-265).  Usage
// only grows during a call, so a candidate checked against the usage of the
// workloads admitted so far keeps a failed verdict for good, and a fitting
// verdict until an admission adds usage on one of its leaves.
// One 1024-thread workgroup, one round per window of kAdmitWindow candidates:
//  1. each wave checks one candidate against the current usage (a record
//     whose leaf no admission of this call touched keeps its phase-1 verdict
//     without a load: the `touched` bitmap);
//  2. the window is decided in order: rejections are final; the first fitting
//     candidate is admitted; a later fitting one is admitted as well when none
//     of its leaves was admitted onto earlier in this round (the `round`
//     bitmap, LDS) — its check still holds — and the round stops at the first
//     fitting candidate that shares a leaf with this round's admissions (it
//     is checked again, first of the next window);
//  3. an admitted candidate's wave adds its usage with non-returning atomics;
//     the round ends with every wave's memory counters drained (s_waitcnt 0:
//     the atomics performed at L2, where the next round's loads read) and a
//     barrier.
// Rounds ~ conflicts + candidates / kAdmitWindow instead of admissions +
// rejections / kAdmitWindow.  Without room for both bitmaps in LDS the round
// admits only its first fitting candidate (the round-3 windowed kernel).
// (A variant that spread the window's records over all 1024 threads measured
// admit_device 4.1 ms vs 1.8 ms on C3 (profiles/r03_lp4, r03): a wave per candidate
// stops at the candidate's first failing record, the spread one checks all.
// An agent-scope __threadfence per admission writes the XCD's L2 back
// (buffer_wbl2): the drained counters order the atomics without it.)
constexpr int kAdmitWindow = 16;
__device__ __forceinline__ void admit_drain() {  // every outstanding memory operation of the wave completed
  __builtin_amdgcn_s_waitcnt(0);
}
// A remaining candidate checked against the current usage (the rejection
// sweep; wave-uniform): every record's Fits, the untouched leaves keeping
// their phase-1 verdict.
__device__ bool admit_sweep_fits(const DevSnap& s, const int64_t* tas_usage, const uint32_t* usage_present,
                                 const kueue_tas_fits_req* reqs, const kueue_tas_fits_term* terms, const AdmitRec* recs,
                                 const uint32_t* touched_lds, const uint32_t* touched_global, bool in_lds, int64_t r0,
                                 int64_t r1) {
  const int lane = lane_id();
  bool fit = true;
  for (int64_t base = r0; base < r1 && fit; base += kWave) {
    const int64_t i = base + lane;
    bool ok = true;
    if (i < r1) {
      const AdmitRec a = recs[i];
      if (a.status == kAdmitWide) {
        ok = admit_record_fits(s, tas_usage, usage_present, reqs[i], terms);
      } else if (a.status == kAdmitNever) {
        ok = false;
      } else if (a.status == kAdmitCheck && admit_touched(touched_lds, touched_global, in_lds, a.leaf)) {
        int64_t us[kAdmitTerms];
#pragma unroll
        for (int u = 0; u < kAdmitTerms; u++)
          us[u] = (a.col[u] >= 0 && a.val[u] > 0) ? load_l2(tas_usage + int64_t(a.col[u]) * s.N + a.leaf) : 0;
#pragma unroll
        for (int u = 0; u < kAdmitTerms; u++) ok &= !(a.col[u] >= 0 && a.val[u] > 0) || us[u] <= a.lim[u];
      }
    }
    fit = ballot(!ok) == 0;
  }
  return fit;
}
// admit_window_kernel's state across its phases (kAdmitState ints): the
// window kernel hands a rejection sweep to the grid (admit_sweep_kernel,
// then admit_compact_kernel) and the next phase resumes where it stopped.
enum AdmitState { AS_STARTED, AS_W0, AS_NTODO, AS_ROUNDS, AS_SWEEPS, AS_GATE, AS_SWEEP, AS_DONE, kAdmitState };
__global__ __launch_bounds__(64 * kAdmitWindow) void admit_window_kernel(
    DevSnap s, int64_t* tas_usage, uint32_t* usage_present, const kueue_tas_fits_req* reqs,
    const kueue_tas_fits_term* terms, const AdmitRec* recs, const int64_t* wl_off, int n_wl, int pods_col,
    const int32_t* wl_fit0, const int32_t* exact_flag, uint32_t* touched_global, int touched_in_lds,
    int32_t* admitted, int32_t* todo, int64_t* todo_r, int32_t* st, int grid_sweeps) {
  extern __shared__ uint32_t touched_lds[];  // touched bitmap [nwords] (+ the round's bitmap [nwords] when chained)
  if (st[AS_DONE]) return;  // an earlier phase finished the pass
  __shared__ int32_t sh_fit[kAdmitWindow];
  __shared__ int32_t sh_conf[2];  // per admission attempt, alternating (one barrier per attempt)
  __shared__ int32_t sh_scan[64 * kAdmitWindow];  // the sweep's compaction (a count per thread)
  const int lane = lane_id(), wave = int(threadIdx.x) >> 6;
  const int nwords = (s.N + 31) / 32;
  const bool in_lds = touched_in_lds != 0;
  const bool chain = touched_in_lds == 2;
  uint32_t* round_lds = touched_lds + nwords;
  if (in_lds)  // the leaves admit_indep_kernel admitted onto (the global bitmap, cleared by the host)
    for (int k = threadIdx.x; k < (chain ? 2 : 1) * nwords; k += blockDim.x)
      touched_lds[k] = k < nwords ? touched_global[k] : 0u;
  const bool exact = *exact_flag != 0;
  const bool resumed = st[AS_STARTED] != 0;
  int ntodo = resumed ? st[AS_NTODO] : todo[0];
  __syncthreads();
  int w0 = resumed ? st[AS_W0] : 0;  // position in the todo list
  int rounds = st[AS_ROUNDS], sweeps = st[AS_SWEEPS], nrej_since = 0;
  int sweep_gate = resumed ? st[AS_GATE] : kAdmitWindow / 4;
  int pf_pos = -1, pf_w = n_wl;  // the next window's candidate, fetched during this round
  int64_t pf_r0 = 0, pf_r1 = 0;
  while (w0 < ntodo) {  // block-uniform
    rounds++;
    const int pos = w0 + wave;
    int w = n_wl;
    int64_t r0 = 0, r1 = 0;
    if (pos < ntodo) {
      if (pf_pos == pos) {  // the previous window was decided whole
        w = pf_w;
        r0 = pf_r0;
        r1 = pf_r1;
      } else {
        w = todo[1 + pos];
        r0 = todo_r[2 * pos];
        r1 = todo_r[2 * pos + 1];
      }
    }
    pf_pos = pos + kAdmitWindow;
    if (pf_pos < ntodo) {
      pf_w = todo[1 + pf_pos];
      pf_r0 = todo_r[2 * pf_pos];
      pf_r1 = todo_r[2 * pf_pos + 1];
    }
    // the candidate's first 64 records stay in registers: the overlap check
    // and AddUsage of an admission then issue no dependent loads
    int32_t c_leaf = -1, c_count = 0, c_status = kAdmitNever;
    uint32_t c_col[kAdmitTerms / 4] = {};  // column + 1 per byte (0: none; columns < KUEUE_TAS_MAX_COLS)
    int64_t c_val[kAdmitTerms];
#pragma unroll
    for (int u = 0; u < kAdmitTerms; u++) c_val[u] = 0;
    bool fit = false;
    if (w < n_wl && (wl_fit0[w] != 0 || exact)) {
      fit = true;
      for (int64_t base = r0; base < r1 && fit; base += kWave) {
        const int64_t i = base + lane;
        bool ok = true;
        if (i < r1) {
          const AdmitRec a = recs[i];
          if (base == r0) {
            c_leaf = a.leaf;
            c_count = a.count;
            c_status = a.status;
#pragma unroll
            for (int u = 0; u < kAdmitTerms; u++) {
              c_col[u >> 2] |= uint32_t(a.col[u] + 1) << (8 * (u & 3));
              c_val[u] = a.val[u];
            }
          }
          if (exact || a.status == kAdmitWide) {
            ok = admit_record_fits(s, tas_usage, usage_present, reqs[i], terms);
          } else if (a.status == kAdmitNever) {
            ok = false;
          } else if (a.status == kAdmitCheck && admit_touched(touched_lds, touched_global, in_lds, a.leaf)) {
            int64_t us[kAdmitTerms];
#pragma unroll
            for (int u = 0; u < kAdmitTerms; u++)
              us[u] = (a.col[u] >= 0 && a.val[u] > 0) ? load_l2(tas_usage + int64_t(a.col[u]) * s.N + a.leaf) : 0;
#pragma unroll
            for (int u = 0; u < kAdmitTerms; u++) ok &= !(a.col[u] >= 0 && a.val[u] > 0) || us[u] <= a.lim[u];
          }
        }
        fit = ballot(!ok) == 0;
      }
    }
    if (lane == 0) sh_fit[wave] = fit ? 1 : 0;
    __syncthreads();
    // the window in order (block-uniform control flow)
    const int wend = min(kAdmitWindow, ntodo - w0);
    int k = 0, nadm = 0;
    for (; k < wend; k++) {
      if (!sh_fit[k]) {  // final rejection
        if (wave == k && lane == 0) admitted[w] = 0;
        continue;
      }
      if (nadm > 0 && !chain) break;  // without the round bitmap: one admission per round
      if (wave == k) {
        // a later fitting candidate's check holds unless it shares a leaf with
        // this round's admissions; if it does not, it is admitted at once
        bool hit = false;
        if (nadm > 0)
          for (int64_t base = r0; base < r1 && !hit; base += kWave) {
            const int64_t i = base + lane;
            const int32_t leaf = i >= r1 ? -1 : base == r0 ? c_leaf : recs[i].leaf;
            hit = ballot(leaf >= 0 && ((round_lds[leaf >> 5] >> (leaf & 31)) & 1u)) != 0;
          }
        if (!hit) {  // admit: AddUsage over its records, the wave's lanes a share each
          for (int64_t base = r0; base < r1; base += kWave) {
            const int64_t i = base + lane;
            if (i >= r1) continue;
            int32_t leaf;
            uint32_t bits = 0;
            int64_t count;
            if (base == r0 && !exact && c_status != kAdmitWide) {  // the record's terms are in registers
              leaf = c_leaf;
              count = c_count;
#pragma unroll
              for (int u = 0; u < kAdmitTerms; u++) {
                const int col = int((c_col[u >> 2] >> (8 * (u & 3))) & 0xffu) - 1;
                if (col >= 0) {  // the host gives every usage resource a column first
                  atomicAdd(reinterpret_cast<unsigned long long*>(tas_usage + int64_t(col) * s.N + leaf),
                            (unsigned long long)(uint64_t(c_val[u]) * uint64_t(count)));
                  bits |= 1u << col;
                }
              }
            } else {
              const kueue_tas_fits_req r = reqs[i];
              leaf = r.leaf;
              count = r.count;
              for (int q = 0; q < r.num_terms; q++) {
                const kueue_tas_fits_term t = terms[r.term_begin + q];
                if (t.col >= 0) {
                  atomicAdd(reinterpret_cast<unsigned long long*>(tas_usage + int64_t(t.col) * s.N + leaf),
                            (unsigned long long)(uint64_t(t.value) * uint64_t(count)));
                  bits |= 1u << t.col;
                }
              }
            }
            if (pods_col >= 0) {
              atomicAdd(reinterpret_cast<unsigned long long*>(tas_usage + int64_t(pods_col) * s.N + leaf),
                        (unsigned long long)count);
              bits |= 1u << pods_col;
            }
            atomicOr(usage_present + leaf, bits);
            if (in_lds) atomicOr(touched_lds + (leaf >> 5), 1u << (leaf & 31));
            else atomicOr(touched_global + (leaf >> 5), 1u << (leaf & 31));
            if (chain) atomicOr(round_lds + (leaf >> 5), 1u << (leaf & 31));
          }
          if (lane == 0) admitted[w] = 1;
        }
        if (lane == 0) sh_conf[nadm & 1] = hit ? 1 : 0;
      }
      if (chain) {  // the verdict, and the round's leaves for the next candidate's overlap check
        __syncthreads();
        if (sh_conf[nadm & 1]) break;
      }
      nadm++;
    }
    // todo[1 + w0 .. w0 + k - 1] are decided; w0 + k (if any) is checked again
    admit_drain();  // this wave's atomics performed at L2 before any wave's next loads
    if (chain && nadm > 0)
      for (int q = threadIdx.x; q < nwords; q += blockDim.x) round_lds[q] = 0;
    __syncthreads();
    w0 += k;
    // Rejection sweep: usage only grows during the pass (AddUsage), so a
    // candidate that does not fit the current usage cannot fit at its turn
    // (scheduler.go:426-435 runs Fits on usage that includes every earlier
    // admission): after a round that rejected several candidates, every
    // remaining candidate is checked against the current usage in parallel
    // (a wave per candidate), the failures rejected at once, and the todo
    // list compacted in place — nominated workloads that all target the same
    // best-fit domains (an idle, uniform cluster) leave the pass in a few
    // sweeps instead of a window round per 16 of them.
    // A sweep costs a pass over every remaining candidate's records: after one
    // that rejected under a quarter of them the next needs 4x the rejections.
    for (int q = 0; q < k; q++) nrej_since += sh_fit[q] ? 0 : 1;
    if (nrej_since >= sweep_gate && ntodo - w0 > 2 * kAdmitWindow && !exact) {  // block-uniform
      nrej_since = 0;
      if (grid_sweeps) {  // the grid sweeps (admit_sweep_kernel): this phase stops here
        if (in_lds)  // the touched bitmap back to global memory for the sweep and the next phase
          for (int q = threadIdx.x; q < nwords; q += blockDim.x) touched_global[q] = touched_lds[q];
        if (threadIdx.x == 0) {
          st[AS_STARTED] = 1;
          st[AS_W0] = w0;
          st[AS_NTODO] = ntodo;
          st[AS_ROUNDS] = rounds;
          st[AS_SWEEPS] = sweeps;
          st[AS_GATE] = sweep_gate;
          st[AS_SWEEP] = 1;
        }
        return;
      }
      sweeps++;
      const int swept_from = ntodo - w0;
      for (int pos = w0 + wave; pos < ntodo; pos += kAdmitWindow) {
        const int w = todo[1 + pos];
        const int64_t r0 = todo_r[2 * pos], r1 = todo_r[2 * pos + 1];
        const bool fit = wl_fit0[w] != 0 &&
                         admit_sweep_fits(s, tas_usage, usage_present, reqs, terms, recs, touched_lds, touched_global,
                                          in_lds, r0, r1);
        if (!fit && lane == 0) {
          admitted[w] = 0;
          todo[1 + pos] = -1;  // rejected: dropped by the compaction
        }
      }
      __syncthreads();
      // in-place stable compaction of todo[w0 .. ntodo): every thread reads its
      // contiguous share into registers, a block scan of the kept counts, then
      // the writes (to lower or equal positions, after every read)
      constexpr int kPer = 16;  // positions per thread per pass (1,024 threads: 16,384 a pass)
      int out_base = w0;
      for (int seg = w0; seg < ntodo; seg += kPer * int(blockDim.x)) {
        const int p0 = seg + int(threadIdx.x) * kPer;
        int ww[kPer];
        int64_t rr0[kPer], rr1[kPer];
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < kPer; u++) {
          const int p = p0 + u;
          ww[u] = p < ntodo ? todo[1 + p] : -1;
          rr0[u] = ww[u] >= 0 ? todo_r[2 * p] : 0;
          rr1[u] = ww[u] >= 0 ? todo_r[2 * p + 1] : 0;
          cnt += ww[u] >= 0 ? 1 : 0;
        }
        sh_scan[threadIdx.x] = cnt;
        __syncthreads();
        for (int off = 1; off < int(blockDim.x); off <<= 1) {  // Hillis-Steele inclusive scan
          const int v = threadIdx.x >= unsigned(off) ? sh_scan[threadIdx.x - off] : 0;
          __syncthreads();
          sh_scan[threadIdx.x] += v;
          __syncthreads();
        }
        int o = out_base + sh_scan[threadIdx.x] - cnt;
        const int seg_total = sh_scan[blockDim.x - 1];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kPer; u++)
          if (ww[u] >= 0) {
            todo[1 + o] = ww[u];
            todo_r[2 * o] = rr0[u];
            todo_r[2 * o + 1] = rr1[u];
            o++;
          }
        out_base += seg_total;
        __threadfence_block();
        __syncthreads();
      }
      if (4 * (swept_from - (out_base - w0)) < swept_from) sweep_gate *= 4;
      ntodo = out_base;
      pf_pos = -1;  // the prefetched candidate's position moved
    }
  }
  if (threadIdx.x == 0) {  // diagnostics after the verdicts: rounds, candidates in the in-order pass, sweeps
    admitted[n_wl] = rounds;
    admitted[n_wl + 1] = todo[0];
    admitted[n_wl + 2] = sweeps;
    st[AS_DONE] = 1;
  }
}

// The rejection sweep over the grid (a wave per remaining candidate, grid-
// stride): admit_window_kernel stopped at a sweep point; every remaining
// candidate that does not fit the current usage is rejected (final: usage
// only grows) and marked for the compaction.
__global__ __launch_bounds__(256) void admit_sweep_kernel(DevSnap s, const int64_t* tas_usage,
                                                          const uint32_t* usage_present, const kueue_tas_fits_req* reqs,
                                                          const kueue_tas_fits_term* terms, const AdmitRec* recs,
                                                          const int32_t* wl_fit0, const uint32_t* touched_global,
                                                          int32_t* admitted, int32_t* todo, const int64_t* todo_r,
                                                          const int32_t* st) {
  if (!st[AS_SWEEP] || st[AS_DONE]) return;
  const int w0 = st[AS_W0], ntodo = st[AS_NTODO];
  const int waves = int(gridDim.x * (blockDim.x >> 6));
  for (int pos = w0 + int(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); pos < ntodo; pos += waves) {
    const int w = todo[1 + pos];
    const bool fit = wl_fit0[w] != 0 && admit_sweep_fits(s, tas_usage, usage_present, reqs, terms, recs, nullptr,
                                                         touched_global, false, todo_r[2 * pos], todo_r[2 * pos + 1]);
    if (!fit && lane_id() == 0) {
      admitted[w] = 0;
      todo[1 + pos] = -1;
    }
  }
}

// The sweep's stable compaction of the todo list (one workgroup, in place:
// every thread reads its share, a block scan of the kept counts, the writes
// to lower or equal positions), then the window kernel's next phase.
__global__ __launch_bounds__(1024) void admit_compact_kernel(int32_t* todo, int64_t* todo_r, int32_t* st) {
  __shared__ int32_t sh_scan[1024];
  if (!st[AS_SWEEP] || st[AS_DONE]) return;
  const int w0 = st[AS_W0], ntodo = st[AS_NTODO];
  constexpr int kPer = 16;
  int out_base = w0;
  for (int seg = w0; seg < ntodo; seg += kPer * int(blockDim.x)) {
    const int p0 = seg + int(threadIdx.x) * kPer;
    int ww[kPer];
    int64_t rr0[kPer], rr1[kPer];
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const int p = p0 + u;
      ww[u] = p < ntodo ? todo[1 + p] : -1;
      rr0[u] = ww[u] >= 0 ? todo_r[2 * p] : 0;
      rr1[u] = ww[u] >= 0 ? todo_r[2 * p + 1] : 0;
      cnt += ww[u] >= 0 ? 1 : 0;
    }
    sh_scan[threadIdx.x] = cnt;
    __syncthreads();
    for (int off = 1; off < int(blockDim.x); off <<= 1) {
      const int v = threadIdx.x >= unsigned(off) ? sh_scan[threadIdx.x - off] : 0;
      __syncthreads();
      sh_scan[threadIdx.x] += v;
      __syncthreads();
    }
    int o = out_base + sh_scan[threadIdx.x] - cnt;
    const int seg_total = sh_scan[blockDim.x - 1];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; u++)
      if (ww[u] >= 0) {
        todo[1 + o] = ww[u];
        todo_r[2 * o] = rr0[u];
        todo_r[2 * o + 1] = rr1[u];
        o++;
      }
    out_base += seg_total;
    __threadfence_block();
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int swept_from = ntodo - w0;
    if (4 * (swept_from - (out_base - w0)) < swept_from) st[AS_GATE] *= 4;  // as the in-kernel sweep
    st[AS_NTODO] = out_base;
    st[AS_SWEEPS] += 1;
    st[AS_SWEEP] = 0;
  }
}


// ---- admission from the gathered device block (kueue_tas_admit_block) ----
// The all-gather leaves every rank's assignments in one device block, row r
// = [words, quads...] (kueue_tas_host_last_assignments' layout: a header
// (id, -1, failed, n) before each workload's n domain quads (id, podset,
// leaf, count)).  Rank 0 admits from it without a host round trip: the
// headers locate each workload's run, one workgroup orders the present
// workloads by id (processEntry's order, scheduler.go:337-339) and offsets
// their records, and the records take their PodSet's single-pod request
// terms from the compiled workloads' per-PodSet table (ComputeTASNetUsage,
// flavorassigner.go:94-130).  Error bits (AdmitBlockErr) send the host to
// its own path (a layout it does not assume) or report the record errors
// its own path reports.
constexpr int kAdmitMaxRows = 16;
struct AdmitRows {
  int64_t row_words;
  int32_t world;
  int32_t nq[kAdmitMaxRows];  // quads per row
};
enum AdmitBlockErr { ABE_ID = 1, ABE_RANGE = 2, ABE_DUP = 4, ABE_LAYOUT = 8, ABE_COL = 16 };

// One thread per quad slot of every row: a header records its workload's
// run (the row position of its first domain quad, the quad count, failed).
__global__ __launch_bounds__(256) void admit_block_headers_kernel(const int32_t* block, AdmitRows rows, int W,
                                                                  int32_t* wl_flag, int64_t* wl_pos, int32_t* wl_nd,
                                                                  int32_t* err) {
  const int r = int(blockIdx.y);
  const int q = int(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= rows.world || q >= rows.nq[r]) return;
  const int32_t* p = block + int64_t(r) * rows.row_words + 1 + 4 * int64_t(q);
  if (p[1] >= 0) return;
  const int32_t g = p[0];
  if (g < 0 || g >= W) {
    atomicOr(err, ABE_ID);
    return;
  }
  if (atomicAdd(wl_flag + g, p[2] != 0 ? 2 : 1) != 0) atomicOr(err, ABE_DUP);  // one header per workload
  wl_pos[g] = int64_t(r) * rows.row_words + 1 + 4 * (int64_t(q) + 1);
  wl_nd[g] = p[3];
  if (p[3] < 0 || q + 1 + p[3] > rows.nq[r]) atomicOr(err, ABE_LAYOUT);
}

// One workgroup: the present workloads in id order (ids, fit0 = 1) and their
// record offsets (a failed evaluation: one record that cannot fit).
// hdr[0] = workloads, hdr[1] = records.
__global__ __launch_bounds__(1024) void admit_block_offsets_kernel(int W, const int32_t* wl_flag, const int32_t* wl_nd,
                                                                   int32_t* ids, int64_t* wl_off, int32_t* fit0,
                                                                   int32_t* hdr) {
  __shared__ int32_t sh_c[16], sh_r[16];
  const int lane = lane_id(), wave = int(threadIdx.x) >> 6, nw = int(blockDim.x) >> 6;
  int32_t base_w = 0;
  int64_t base_r = 0;
  for (int c0 = 0; c0 < W; c0 += int(blockDim.x)) {  // block-uniform
    const int g = c0 + int(threadIdx.x);
    const int32_t f = g < W ? wl_flag[g] : 0;
    const int32_t present = f != 0 ? 1 : 0;
    const int32_t nrec = f == 0 ? 0 : f >= 2 ? 1 : max(wl_nd[g], 0);
    int tc, tr;
    const int ec = wave_excl_scan(present, &tc), er = wave_excl_scan(nrec, &tr);
    if (lane == 0) {
      sh_c[wave] = tc;
      sh_r[wave] = tr;
    }
    __syncthreads();
    int32_t oc = base_w, tot_c = 0;
    int64_t orr = base_r, tot_r = 0;
    for (int k = 0; k < nw; k++) {
      if (k < wave) {
        oc += sh_c[k];
        orr += sh_r[k];
      }
      tot_c += sh_c[k];
      tot_r += sh_r[k];
    }
    if (present) {
      const int j = oc + ec;
      ids[j] = g;
      wl_off[j] = orr + er;
      fit0[j] = 1;
    }
    base_w += tot_c;
    base_r += tot_r;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    wl_off[base_w] = base_r;
    hdr[0] = base_w;
    hdr[1] = int32_t(base_r);
  }
}

// One wave per present workload: its records (leaf, count, its PodSet's
// terms in the compiled table), record -> workload, and per column the
// 128-bit total of count x value this call can add (kueue_tas_admit's
// monotone shortcut precondition; tot[2 col] low, tot[2 col + 1] high words).
// ex[0] = 1 when a count or a value is negative (no shortcut).
__global__ __launch_bounds__(256) void admit_block_records_kernel(
    const int32_t* block, int N, int W, const int32_t* ids, const int64_t* wl_off, const int32_t* wl_flag,
    const int64_t* wl_pos, const int32_t* wl_nd, const int32_t* ps_base, const int32_t* ps_terms,
    const kueue_tas_fits_term* terms, int n_wl, int pods_col, kueue_tas_fits_req* reqs, int32_t* rec_wl,
    unsigned long long* tot, int32_t* ex, int32_t* err) {
  // the block's per-column totals in LDS first (one global atomic per column
  // and block: device-scope atomics on a handful of addresses from every
  // record serialize at the memory side)
  __shared__ unsigned long long sh_tot[2 * KUEUE_TAS_MAX_COLS];
  for (int q = threadIdx.x; q < 2 * KUEUE_TAS_MAX_COLS; q += blockDim.x) sh_tot[q] = 0;
  __syncthreads();
  const int k = int(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int lane = lane_id();
  int32_t bad = 0, neg = 0;
  auto add128 = [&](int col, uint64_t lo, uint64_t hi) {
    const unsigned long long old = atomicAdd(sh_tot + 2 * col, (unsigned long long)lo);
    const uint64_t carry = (old + lo < old) ? 1u : 0u;
    if (hi + carry) atomicAdd(sh_tot + 2 * col + 1, (unsigned long long)(hi + carry));
  };
  if (k < n_wl) {
    const int32_t g = ids[k];
    const int64_t base = wl_off[k];
    if (wl_flag[g] >= 2) {  // a failed evaluation is never admitted
      if (lane == 0) {
        reqs[base] = kueue_tas_fits_req{-1, 0, 0, 0};
        rec_wl[base] = k;
      }
    } else {
      const int32_t nd = wl_nd[g];
      const int64_t pos = wl_pos[g];
      const int32_t ps0 = ps_base[g], nps = ps_base[g + 1] - ps0;
      for (int j = lane; j < nd; j += kWave) {
        const int32_t* p = block + pos + 4 * int64_t(j);
        const int32_t pg = p[0], ps = p[1], leaf = p[2], count = p[3];
        if (pg != g || ps < 0) {
          bad |= ABE_LAYOUT;
          continue;
        }
        if (ps >= nps || leaf < 0 || leaf >= N) {
          bad |= ABE_RANGE;
          continue;
        }
        const int32_t tb = ps_terms[2 * (ps0 + ps)], nt = ps_terms[2 * (ps0 + ps) + 1];
        reqs[base + j] = kueue_tas_fits_req{leaf, count, tb, nt};
        rec_wl[base + j] = k;
        if (count < 0) neg = 1;
        for (int t = 0; t < nt; t++) {
          const kueue_tas_fits_term tm = terms[tb + t];
          if (tm.col < 0 || tm.col >= KUEUE_TAS_MAX_COLS) {
            bad |= ABE_COL;
            continue;
          }
          if (tm.value < 0) neg = 1;
          if (tm.value <= 0 || count <= 0) continue;
          const uint64_t a = uint64_t(tm.value), c = uint64_t(count);
          add128(tm.col, a * c, __umul64hi(a, c));
        }
        if (pods_col >= 0 && count > 0) add128(pods_col, uint64_t(count), 0);
      }
    }
  }
  if (bad) atomicOr(err, bad);
  if (neg) atomicOr(ex, 1);
  __syncthreads();
  for (int col = threadIdx.x; col < KUEUE_TAS_MAX_COLS; col += blockDim.x) {
    const uint64_t lo = sh_tot[2 * col], hi = sh_tot[2 * col + 1];
    if (!lo && !hi) continue;
    const unsigned long long old = atomicAdd(tot + 2 * col, (unsigned long long)lo);
    const uint64_t carry = (old + lo < old) ? 1u : 0u;
    if (hi + carry) atomicAdd(tot + 2 * col + 1, (unsigned long long)(hi + carry));
  }
}

// The admitted workloads' deltas (updateTASUsage per record: its terms, then
// pods), in record order — the host path's list, element for element.
// Pass 1: per block of records its delta count; pass 2 (one workgroup): the
// blocks' offsets; pass 3: each block writes its deltas.
__device__ __forceinline__ int admit_delta_count(const kueue_tas_fits_req* reqs, const int32_t* rec_wl,
                                                 const int32_t* admitted, int n, int pods_col, int i) {
  if (i >= n) return 0;
  const kueue_tas_fits_req r = reqs[i];
  if (!admitted[rec_wl[i]] || r.leaf < 0) return 0;
  return r.num_terms + (pods_col >= 0 ? 1 : 0);
}
__global__ __launch_bounds__(256) void admit_delta_blocks_kernel(const kueue_tas_fits_req* reqs, const int32_t* rec_wl,
                                                                 const int32_t* admitted, int n, int pods_col,
                                                                 int32_t* blk) {
  __shared__ int32_t sh[4];
  const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
  int tot;
  (void)wave_excl_scan(admit_delta_count(reqs, rec_wl, admitted, n, pods_col, i), &tot);
  if (lane_id() == 0) sh[threadIdx.x >> 6] = tot;
  __syncthreads();
  if (threadIdx.x == 0) blk[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}
__global__ __launch_bounds__(1024) void admit_delta_offsets_kernel(int32_t* blk, int nblk, int32_t* hdr) {
  __shared__ int32_t sh[16];
  const int lane = lane_id(), wave = int(threadIdx.x) >> 6, nw = int(blockDim.x) >> 6;
  int32_t base = 0;
  for (int c0 = 0; c0 < nblk; c0 += int(blockDim.x)) {
    const int b = c0 + int(threadIdx.x);
    const int32_t v = b < nblk ? blk[b] : 0;
    int t;
    const int e = wave_excl_scan(v, &t);
    if (lane == 0) sh[wave] = t;
    __syncthreads();
    int32_t o = base, tot = 0;
    for (int k = 0; k < nw; k++) {
      if (k < wave) o += sh[k];
      tot += sh[k];
    }
    if (b < nblk) blk[b] = o + e;
    base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) hdr[2] = base;
}
__global__ __launch_bounds__(256) void admit_delta_write_kernel(const kueue_tas_fits_req* reqs,
                                                                const kueue_tas_fits_term* terms,
                                                                const int32_t* rec_wl, const int32_t* admitted, int n,
                                                                int pods_col, const int32_t* blk, kueue_tas_delta* out) {
  __shared__ int32_t sh[4];
  const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
  const int c = admit_delta_count(reqs, rec_wl, admitted, n, pods_col, i);
  int tot;
  const int e = wave_excl_scan(c, &tot);
  if (lane_id() == 0) sh[threadIdx.x >> 6] = tot;
  __syncthreads();
  int o = blk[blockIdx.x] + e;
  for (int k = 0; k < int(threadIdx.x >> 6); k++) o += sh[k];
  if (!c) return;
  const kueue_tas_fits_req r = reqs[i];
  for (int q = 0; q < r.num_terms; q++) {
    const kueue_tas_fits_term t = terms[r.term_begin + q];
    out[o++] = kueue_tas_delta{r.leaf, t.col, int64_t(uint64_t(t.value) * uint64_t(int64_t(r.count)))};
  }
  if (pods_col >= 0) out[o] = kueue_tas_delta{r.leaf, pods_col, int64_t(r.count)};
}

}  // namespace ktas
