// tas_device.cpp — device layer of libkueue_tas.so: HBM-resident snapshot,
// batch staging and kernel launches behind the C-ABI of include/kueue_tas.h.
//
// Data layout in HBM (per context):
//   snapshot  free_cap[R][N], tas_usage[R][N] (int64 SoA), presence bitmasks
//             [N], taint-profile ids [N], label-value ids [K][N], CSR child
//             offsets per level, DomainID ranks [sum D_l]
//   per batch counters[n][5][sum D_l] int32 (state, sliceState, stateWithLeader,
//             sliceStateWithLeader, leaderState), exclusion counters, phase-2
//             scratch lists, result headers and (leaf, count) entries
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "tas_internal.h"
#include "tas_pool.h"
#include "tas_kernels.hip"

using namespace ktas;

namespace {

constexpr int kEvalsPerFillBlock = kEvalsPerBlock;

// A simple class: no leader, one-pod slices at the leaf level and no inner
// slice rounding, so sliceState == state at every level: its class row keeps
// one field (FillEvalParams::ss_alias, ctr_row).
bool simple_class(const DevEval& ev, int L) {
  bool simple = (ev.flags & KUEUE_TAS_F_LEADER) == 0 && ev.slice_level == L - 1 && ev.slice_size == 1;
  for (int l = 0; l < L && simple; l++) simple = ev.ssal[l] == 0 || ev.ssal[l] == 1;
  return simple;
}

// Device bytes per context (kueue_tas_device_bytes): every DevBuf built
// while a context is constructed links itself into that context's chain.
struct DevBufLink {
  size_t bytes = 0;
  DevBufLink* next = nullptr;
};
thread_local DevBufLink** g_devbuf_chain = nullptr;

template <typename T>
struct DevBuf : DevBufLink {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() {
    if (g_devbuf_chain) {
      next = *g_devbuf_chain;
      *g_devbuf_chain = this;
    }
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    bytes = 0;
    size_t nb = std::max<size_t>(count, 1) * sizeof(T);
    hipError_t e = hipMalloc(&p, nb);
    if (e == hipSuccess) {
      n = std::max<size_t>(count, 1);
      bytes = nb;
    }
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    bytes = 0;
  }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(bytes, o.bytes);
  }
  // ensure with 1/8 headroom when it grows (buffers that grow by a few rows at a time)
  hipError_t reserve(size_t count) { return count <= n && p ? hipSuccess : ensure(count + count / 8); }
};

template <typename T>
struct HostBuf {  // pinned host staging
  T* p = nullptr;
  size_t n = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { release(); }
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc(&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault);
    if (e == hipSuccess) n = std::max<size_t>(count, 1);
    return e;
  }
  // ensure with 1/8 headroom when it grows (a pinned allocation costs a millisecond)
  hipError_t reserve(size_t count) { return count <= n && p ? hipSuccess : ensure(count + count / 8); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
};

// Open-addressing uint64 -> int32 map (linear probing), reset per batch
// without freeing: the phase-1 class lookup of every eval.
struct FlatMap {
  std::vector<uint64_t> keys;
  std::vector<int32_t> vals;  // -1: empty
  size_t mask = 0;
  void reset(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    if (keys.size() != cap) {
      keys.assign(cap, 0);
      vals.assign(cap, -1);
    } else {
      std::fill(vals.begin(), vals.end(), -1);
    }
    mask = cap - 1;
  }
  static size_t mix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return size_t(k);
  }
  int32_t* find(uint64_t k) {  // the slot's value (-1 if absent)
    for (size_t i = mix(k) & mask;; i = (i + 1) & mask) {
      if (vals[i] < 0 || keys[i] == k) {
        keys[i] = k;
        return &vals[i];
      }
    }
  }
};

// One static part's phase-1 classes (eval_chunk): chains of local classes
// per 64-bit class hash, each local class's first member.
struct alignas(64) PartClasses {  // one per host part, on cache lines of its own
  FlatMap head;
  std::vector<int32_t> rep, next;
  std::vector<uint64_t> hcls, hsig;  // each local class's hashes, contiguous for the merge
};

// libdivide-style u64 magic for exact division by an invariant divisor d >= 1.
// 2^(64 + fl) / d and its remainder for 2^fl < d < 2^(fl + 1): the quotient
// fits 64 bits, so one 128-by-64 divq gives both (two __int128 divisions
// through the runtime library cost ~10x that per term)
static inline uint64_t div_pow2_by(int fl, uint64_t d, uint64_t* rem) {
  uint64_t q, r;
  __asm__("divq %4" : "=a"(q), "=d"(r) : "a"(uint64_t(0)), "d"(uint64_t(1) << fl), "rm"(d));
  *rem = r;
  return q;
}

void compute_magic_uncached(uint64_t d, DevTerm* t) {
  t->magic = 0;
  t->shift = 0;
  t->add = 0;
  t->pow2 = 0;
  int fl = 63 - __builtin_clzll(d);
  if ((d & (d - 1)) == 0) {
    t->pow2 = 1;
    t->shift = uint8_t(fl);
    return;
  }
  uint64_t rem;
  uint64_t proposed = div_pow2_by(fl, d, &rem);
  uint64_t e = d - rem;
  if (e < (uint64_t(1) << fl)) {
    t->shift = uint8_t(fl);
  } else {
    proposed += proposed;
    uint64_t twice = rem + rem;
    if (twice >= d || twice < rem) proposed += 1;
    t->shift = uint8_t(fl);
    t->add = 1;
  }
  t->magic = proposed + 1;
}

// the divisors of a batch repeat (a request shape per workload type): a
// direct-mapped cache of the magic numbers per host part, kept in the
// context (a thread_local here cost a __tls_get_addr call per term)
struct MagicSlot {
  uint64_t d = 0, magic = 0;
  uint8_t shift = 0, add = 0, pow2 = 0;
};
struct alignas(64) MagicCache {
  MagicSlot slot[256];
};
void compute_magic(uint64_t d, DevTerm* t, MagicCache& cache) {
  MagicSlot& c = cache.slot[(d * 0x9e3779b97f4a7c15ull) >> 56];
  if (c.d != d) {
    compute_magic_uncached(d, t);
    c.d = d;
    c.magic = t->magic;
    c.shift = t->shift;
    c.add = t->add;
    c.pow2 = t->pow2;
    return;
  }
  t->magic = c.magic;
  t->shift = c.shift;
  t->add = c.add;
  t->pow2 = c.pow2;
}

}  // namespace

struct kueue_tas_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // fast-LFC branch (tables, select, emit) beside the BestFit select
  hipStream_t stream3 = nullptr;  // ExclusionStats branch (staged fill): counts + reduce beside the roll-up/select
  hipEvent_t evs[2] = {};         // ExclusionStats branch: start, end (also the join)
  DevBuf<int8_t> d_fill_lim;
  std::vector<int32_t> cls_pos, cls_cur;
  hipEvent_t ev[8] = {};  // stage boundaries, see eval_chunk
  hipEvent_t evl[4] = {};  // fast-LFC branch: start, end (timing), join, fast select done (emit on the main stream)
  std::string err;
  int list_cap = 1024;
  bool inline_stats = true;   // ExclusionStats counted in the fill (KUEUE_TAS_CFG_SPLIT_STATS: fill_exclusion_kernel)
  bool pair_fill = true;      // fill_pair_kernel for single-run chunks (KUEUE_TAS_CFG_NO_PAIR_FILL clears it)
  bool admit_window = true;   // admit_window_kernel (KUEUE_TAS_CFG_SERIAL_ADMIT: the one-wave chain)
  int admit_grid_sweeps = [] {  // window-kernel phases (rejection sweeps over the grid between them); 1: in-kernel
    const char* e = getenv("KTAS_ADMIT_PHASES");
    return e ? std::max(1, atoi(e)) : 6;
  }();
  bool fused_top = false;     // rollup_top_kernel (KUEUE_TAS_CFG_FUSED_TOP)
  bool cat_fill = true;       // fill_pair_kernel's leaf categories (KUEUE_TAS_CFG_NO_CATEGORY_FILL clears it)
  bool labels16 = false;      // every staged label column's value ids < 2^16 (packed nodeSelector compare)
  int64_t n_loads = 0, n_splices = 0;  // kueue_tas_snapshot_load / _splice calls that succeeded (lifetime)
  bool stage_timing = true;   // record every stage event (else only the fill bracket; kueue_tas_set_stage_timing)
  int max_batch = 1024;
  int entry_cap = 512;  // per-eval device entry capacity (grows on demand)
  // snapshot
  bool loaded = false;
  DevSnap snap{};
  int maxD = 0;
  int rack_fanout = 0;  // see kueue_tas_snapshot_load
  std::vector<int32_t> h_level_sizes;
  DevBuf<int32_t> d_child_off, d_id_rank, d_taint_profile, d_labels;
  DevBuf<uint8_t> d_dead;        // leaves out of the snapshot (kueue_tas_snapshot_set_leaf_live)
  std::vector<uint8_t> h_dead;
  int64_t n_dead = 0;
  DevBuf<int64_t> d_free, d_usage;
  DevBuf<uint32_t> d_free_present, d_usage_present;
  // batch
  DevBuf<int32_t> d_counters;
  // results of a batch, one D2H: out[n] | stats (taint | res | sel counts)
  DevBuf<uint8_t> d_res;
  HostBuf<uint8_t> h_res;
  HostBuf<kueue_tas_eval_out> h_res2;  // the fast-LFC branch's own copy of the result headers (its D2H)
  kueue_tas_eval_out* res_out_h = nullptr;
  int32_t* res_stats_h = nullptr;
  DevBuf<uint64_t> d_scratch;
  DevBuf<kueue_tas_delta> d_deltas;
  DevBuf<uint8_t> d_setfree;  // set_free: leaves | rows | presence
  DevBuf<uint8_t> d_fits;  // kueue_tas_fits: requests | terms | results
  // v1beta2 encoder: parent map (leaf mode), resident names, per-call buffers
  DevBuf<int32_t> d_parent;
  DevBuf<int2> d_wave_tab;       // ragged parents: packed leaf waves (DevSnap::wave_tab)
  DevBuf<int32_t> d_leaf_parent;
  DevBuf<char> d_names;
  DevBuf<int64_t> d_name_off;
  bool names_loaded = false;
  DevBuf<char> d_enc_bytes;
  DevBuf<int64_t> d_enc_stroff, d_enc_off;
  DevBuf<int32_t> d_enc_ids, d_enc_counts, d_enc_same;
  DevBuf<kueue_tas_level_enc> d_enc_out;
  DevBuf<int32_t> d_packed;
  DevBuf<LeafPartial> d_partials;
  DevBuf<int32_t> d_fill_stats;
  HostBuf<uint8_t> h_stage;  // one pinned upload per batch: evals, terms, tables, index lists
  DevBuf<uint8_t> d_stage;
  // phase-1 class computation scratch (kept to avoid reallocation)
  std::vector<int32_t> cls_rep, cls_sig, cls_of, sig_rep, cls_next, sig_next, cls_fastrep, cls_slot, cls_order;
  std::vector<int32_t> sig_base, base_rep, cls_packed, sig_ncls;
  FlatMap cls_head, sig_head;
  DevBuf<int32_t> d_overlay, d_tags;
  DevBuf<int2> d_wave_tab2;     // 128-leaf slots of whole ragged parents (fill_pair_kernel, FC = -1)
  DevBuf<int32_t> d_wide;       // leaf parents wider than a slot (DevSnap::wide_parents)
  DevBuf<uint64_t> d_rack_pos;  // positive-child masks of the leaves' parents (fused fill)  // select's copy-on-write counters and ownership tags
  int32_t tag_epoch = 0;
  // fast-LFC leaf tables (LfcJob, tas_internal.h)
  DevBuf<uint32_t> d_lfc_ch, d_lfc_cp, d_lfc_tot;
  DevBuf<uint64_t> d_lfc_ovs, d_lfc_ovtot;
  DevBuf<uint8_t> d_lfc_u8;
  DevBuf<LfcJob> d_lfc_jobs;
  DevBuf<LfcItem> d_lfc_items;  // [0]: item count, then the items
  DevBuf<int32_t> d_prof;             // profiling build: [n][P_NCAT] select phase ticks
  DevBuf<int32_t> d_fprof;            // profiling build: fill phase stamps [blocks][8]
  std::vector<int32_t> last_fprof;
  DevBuf<int32_t> d_level_max;        // [n][kMaxLevels] level_max_kernel
  std::vector<int32_t> last_prof;
  int num_profiles = 1;
  int64_t stat_fills = 0, stat_evals = 0;  // phase-1 dedup counters (lifetime)
  std::vector<int32_t> last_ticks;    // per-eval select time (100 MHz ticks) of the last batch
  // packed (leaf, count) pairs of the last batch: pinned, device-mapped host
  // memory the pack kernel writes directly (no separate D2H copy or sync)
  int32_t* ent_host = nullptr;
  int32_t* ent_dev = nullptr;
  size_t ent_cap = 0;   // int32 capacity
  size_t ent_used = 0;  // int32 used by the last batch
  // entry tags (kueue_tas_snapshot_set_leaf_tags): per-leaf table in HBM, the
  // per-entry copies in pinned device-mapped host memory beside the entries
  DevBuf<uint64_t> d_leaf_tags;
  HostBuf<int32_t> h_admit;          // kueue_tas_admit's verdicts + its two diagnostics words (pinned D2H)
  int64_t admit_stats[3] = {-1, -1, -1};  // last kueue_tas_admit: window rounds, in-order candidates, candidates
  // kueue_tas_snapshot_splice: the gather's targets (the resident columns'
  // previous buffers after the swap, reused by the next splice) and its
  // pinned staging (leaf sources and joined rows)
  DevBuf<int64_t> sp_free, sp_usage;
  DevBuf<uint32_t> sp_fp, sp_up;
  DevBuf<int32_t> sp_prof, sp_lab, sp_src;
  DevBuf<uint64_t> sp_tags;
  DevBuf<uint8_t> sp_rows;
  HostBuf<uint8_t> h_load;
  HostBuf<uint8_t> h_tab;  // load_impl's re-derived tables (pinned arena, async copies)
  // host-mirror shadow of the usage columns and presence bits (usage_mark / usage_changes)
  DevBuf<int64_t> d_ushadow;
  DevBuf<uint32_t> d_pshadow;
  DevBuf<kueue_tas_delta> d_uchg;
  DevBuf<int32_t> d_uchg_n;
  HostBuf<int32_t> h_uchg_n;
  std::vector<kueue_tas_delta> uchg;
  bool shadow_ok = false;
  // apply_deltas stages the records in pinned memory (async copy, no sync);
  // the event guards the staging buffer's reuse
  HostBuf<kueue_tas_delta> h_deltas;
  hipEvent_t ev_deltas = nullptr;
  bool leaf_tags_on = false;
  uint64_t* tag_host = nullptr;
  uint64_t* tag_dev = nullptr;
  size_t tag_cap = 0;   // uint64 capacity (entry pairs)
  int32_t ent_stride = 0;              // pairs per eval region of the last chunk
  std::vector<int32_t> ent_count;      // pairs written per eval of the last batch (request order)
  std::vector<int64_t> ent_strided_off;  // their region offsets (pairs) in ent_host
  float last_ms[4] = {0, 0, 0, 0};
  float last_stage_ms[KUEUE_TAS_NUM_STAGES] = {};
  std::vector<MagicCache> magic_cache;  // per host part (compute_magic)
  std::vector<int32_t> h_gsrc;          // a splice's leaf sources (load_impl)
  DevBuf<int32_t> d_adm_ps;             // kueue_tas_admit_table: podset base per workload [W + 1], then (begin, n) per podset
  DevBuf<kueue_tas_fits_term> d_adm_terms;  // and the podsets' single-pod request terms
  int32_t adm_W = -1;                   // workloads of the admission table (-1: none)
  DevBuf<kueue_tas_delta> d_adm_deltas; // kueue_tas_admit_block's delta list
  HostBuf<kueue_tas_delta> h_adm_deltas;
  double admit_block_ms = 0;
  std::vector<int32_t> ctr_row_off;     // last batch: each fill position's class row offset (units of SD)
  std::vector<int32_t> level_maxfan;    // [L] the widest parent's child count per level (last load)
  std::vector<int32_t> sel_groups;      // last batch: BestFit-side slot groups (select launches), bounds
  bool scratch_full = false;            // this chunk re-runs with unbounded select lists (an eval overflowed)
  int64_t scratch_reruns = 0;           // chunks re-run so
  int64_t phase2_budget = [] {          // bytes of select lists + overlays + tags per slot group
    const char* e = getenv("KTAS_PHASE2_BUDGET");  // (tests: a small budget, many groups)
    return e ? std::max<int64_t>(atoll(e), 1) : int64_t(4096) << 20;
  }();
  bool force_scratch_rerun = getenv("KTAS_SCRATCH_TEST_RERUN") != nullptr;  // tests: every chunk re-runs once
  int64_t lcap_test_cap = [] {          // tests: bounded lists capped lower (overflows re-run unbounded)
    const char* e = getenv("KTAS_SCRATCH_TEST_CAP");
    return e ? std::max<int64_t>(atoll(e), 1) : int64_t(0);
  }();
  bool scratch_bounded = [] {           // KTAS_SCRATCH_FULL=1: every slot's lists sized for the widest level
    const char* e = getenv("KTAS_SCRATCH_FULL");
    return !(e && atoi(e) != 0);
  }();
  DevBufLink* dev_bufs = nullptr;       // every DevBuf member (kueue_tas_device_bytes)
  bool exact_merge = false;  // the next chunk merges the parts' classes with exact compares (after a collision)
  int64_t merge_reruns = 0;  // chunks re-run after a class hash collision
  size_t lfc_half = 0;        // LFC chunk-table entries per half of d_lfc_ch / d_lfc_ovs
  bool lfc_dirty[2] = {true, true};  // a half not known to be zero
  int lfc_parity = 0;         // the half the next batch with fast-LFC evals uses
  bool lfc_in_fill = [] {     // KTAS_LFC_IN_FILL=1: fast-LFC chunk tables from the pair fill (no lfc_hist_kernel);
    const char* e = getenv("KTAS_LFC_IN_FILL");  // off by default: it lengthens the fill on the main chain
    return e && atoi(e) != 0;                     // by more than it saves the side stream
  }();
  bool collide_test = false; // KUEUE_TAS_CFG_CLASS_COLLIDE
  bool emit_after_bf = [] {    // KTAS_EMIT_MAIN=1: lfc_emit on the main stream after the BestFit select
    const char* e = getenv("KTAS_EMIT_MAIN");
    return e && atoi(e) != 0;
  }();
  int32_t exp_flags = [] {     // diagnostics only (tools/probe_select.py experiments)
    const char* e = getenv("KTAS_EXP_FLAGS");
    return e ? int32_t(atoi(e)) : 0;
  }();

  double trace[24] = {};  // the last chunk's host timeline (wall ms at fixed points, kueue_tas_last_host_trace)
  double host_ms[8] = {};  // last batch host time: compile, classes, enqueue, wait, pack+D2H, copy-out, [6] of compile:
                           // validation pass, [7] of compile: records + hashes pass
  int64_t last_stats[4] = {0, 0, 0, 0};  // fill evals, leaf-partial evals, fill launches, staged columns
  int64_t last_alias_fills = 0;          // fill rows whose sliceState aliases state (FillEvalParams::ss_alias)
  uint32_t fill_paths = 0;               // KUEUE_TAS_PATH_* bits of the last kueue_tas_eval_batch
  // phase-1 counters of the last device chunk (kueue_tas_last_counters):
  // requests [chunk_base, chunk_base + chunk_rep.size()), their class counter rows
  size_t chunk_base = 0;
  std::vector<int32_t> chunk_rep;
  std::vector<uint8_t> chunk_leader;
  std::vector<uint8_t> chunk_alias;  // the class row's sliceState aliases state (FillEvalParams::ss_alias)
  std::vector<const kueue_tas_eval_req*> req_ptrs;  // kueue_tas_eval_batch's requests as kueue_tas_eval_batch_ptrs takes them
  // eval_chunk's per-request host work (kept between batches)
  std::vector<int64_t> req_term_off;
  std::vector<int32_t> req_chunk_maxt;
  std::vector<std::pair<size_t, std::string>> req_errs;
  std::vector<uint64_t> req_sig_hash, req_cls_hash;
  std::vector<uint8_t> req_fast, req_leaf;
  std::vector<int32_t> req_local_cls, part_map;
  std::vector<size_t> part_base;
  std::vector<PartClasses> part_cls;
};

// The leaf-row scatter kernels write repeated entries in no fixed order:
// the calls that take a leaf list require distinct leaves.
static bool distinct_leaves(const int32_t* leaves, size_t n) {
  std::vector<int32_t> sorted(leaves, leaves + n);
  std::sort(sorted.begin(), sorted.end());
  return std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
}

static int fail(kueue_tas_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(c, x)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess)                                                                   \
      return fail(c, KUEUE_TAS_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_));    \
  } while (0)

extern "C" {

static double wall_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int kueue_tas_abi_version(void) { return KUEUE_TAS_ABI_VERSION; }

kueue_tas_ctx* kueue_tas_ctx_create(const kueue_tas_config* cfg) {
  DevBufLink* chain = nullptr;
  g_devbuf_chain = &chain;
  auto* c = new kueue_tas_ctx();
  g_devbuf_chain = nullptr;
  c->dev_bufs = chain;
  if (cfg) {
    c->device = cfg->device;
    c->inline_stats = (cfg->flags & KUEUE_TAS_CFG_INLINE_STATS) != 0 || (cfg->flags & KUEUE_TAS_CFG_SPLIT_STATS) == 0;
    c->pair_fill = (cfg->flags & KUEUE_TAS_CFG_NO_PAIR_FILL) == 0;
    c->admit_window = (cfg->flags & KUEUE_TAS_CFG_SERIAL_ADMIT) == 0;
    c->fused_top = (cfg->flags & KUEUE_TAS_CFG_FUSED_TOP) != 0;
    c->cat_fill = (cfg->flags & KUEUE_TAS_CFG_NO_CATEGORY_FILL) == 0;
    c->collide_test = (cfg->flags & KUEUE_TAS_CFG_CLASS_COLLIDE) != 0;
    if (cfg->flags & KUEUE_TAS_CFG_LFC_IN_FILL) c->lfc_in_fill = true;
    if (cfg->list_cap > 0) {
      int lc = 64;
      while (lc < cfg->list_cap && lc < 1024) lc <<= 1;
      c->list_cap = lc;
    }
    if (cfg->max_batch > 0) c->max_batch = cfg->max_batch;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= c->device) {
    c->err = "no HIP device available";
    delete c;
    return nullptr;
  }
  // priorities: the main stream (fill -> roll-up -> BestFit select, the
  // critical path) and the fast-LFC branch high, the ExclusionStats branch
  // (off the critical path, a full-grid kernel beside select) low, so the
  // dispatcher hands CUs to select's workgroups first
  int prio_lo = 0, prio_hi = 0;
  if (hipSetDevice(c->device) != hipSuccess || hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, prio_lo) != hipSuccess) {
    delete c;
    return nullptr;
  }
  // the BestFit select launch declares more than 64 KiB of dynamic LDS
  // (kSelectWaves x kFinalWalkLds; a workgroup may use all 160 KiB of a CU)
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&select_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          kSelectWaves * std::max(kFinalWalkLds, c->list_cap * 16)) != hipSuccess) {
    c->err = "select_kernel dynamic LDS attribute";
    delete c;
    return nullptr;
  }
  // the batch's events order its streams and time its stages; the host never
  // reads memory through them (it synchronizes the streams), so no system-scope
  // release: ~1.4 us less device time per record (tools/micro/sync_cost.hip)
  for (auto& e : c->ev) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  for (auto& e : c->evl) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  for (auto& e : c->evs) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return c;
}

void kueue_tas_ctx_destroy(kueue_tas_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->stream2) (void)hipStreamSynchronize(c->stream2);
  if (c->stream3) (void)hipStreamSynchronize(c->stream3);
  c->d_child_off.release();
  c->d_id_rank.release();
  c->d_taint_profile.release();
  c->d_labels.release();
  c->d_free.release();
  c->d_usage.release();
  c->d_free_present.release();
  c->d_usage_present.release();
  c->d_counters.release();
  c->d_res.release();
  c->h_res.release();
  c->h_res2.release();
  c->d_scratch.release();
  c->d_deltas.release();
  c->d_setfree.release();
  c->d_fits.release();
  c->d_fill_lim.release();
  c->d_parent.release();
  c->d_wave_tab.release();
  c->d_leaf_parent.release();
  c->d_names.release();
  c->d_name_off.release();
  c->d_enc_bytes.release();
  c->d_enc_stroff.release();
  c->d_enc_off.release();
  c->d_enc_ids.release();
  c->d_enc_counts.release();
  c->d_enc_same.release();
  c->d_enc_out.release();
  c->d_packed.release();
  c->d_partials.release();
  c->d_fill_stats.release();
  c->h_stage.release();
  c->d_stage.release();
  c->d_overlay.release();
  c->d_rack_pos.release();
  c->d_tags.release();
  c->d_lfc_ch.release();
  c->d_lfc_cp.release();
  c->d_lfc_tot.release();
  c->d_lfc_ovs.release();
  c->d_lfc_ovtot.release();
  c->d_lfc_u8.release();
  c->d_lfc_jobs.release();
  c->d_lfc_items.release();
  c->d_prof.release();
  c->d_level_max.release();
  if (c->ent_host) (void)hipHostFree(c->ent_host);
  c->ent_host = c->ent_dev = nullptr;
  if (c->tag_host) (void)hipHostFree(c->tag_host);
  c->tag_host = c->tag_dev = nullptr;
  c->d_leaf_tags.release();
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->evl)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->evs)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_deltas) (void)hipEventDestroy(c->ev_deltas);
  if (c->stream3) (void)hipStreamDestroy(c->stream3);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* kueue_tas_last_error(kueue_tas_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

static int load_impl(kueue_tas_ctx* c, const kueue_tas_snapshot_desc* d, const kueue_tas_splice_desc* sp);

int kueue_tas_snapshot_load(kueue_tas_ctx* c, const kueue_tas_snapshot_desc* d) { return load_impl(c, d, nullptr); }

int kueue_tas_snapshot_splice(kueue_tas_ctx* c, const kueue_tas_splice_desc* sp) {
  if (!c || !sp || !sp->topo || !sp->leaf_src) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  const kueue_tas_snapshot_desc* d = sp->topo;
  if (d->num_levels != c->snap.L || d->num_cols != c->snap.R || d->num_label_cols != c->snap.K ||
      d->lowest_is_hostname != c->snap.lowest_is_hostname)
    return fail(c, KUEUE_TAS_EINVAL, "splice: the tree's levels, columns and label columns stay");
  if (d->num_levels < 1 || d->num_levels > KUEUE_TAS_MAX_LEVELS) return fail(c, KUEUE_TAS_EINVAL, "num_levels");
  const int n_new = d->level_sizes[d->num_levels - 1];
  int fresh = 0;
  for (int j = 0; j < n_new; j++) {
    const int32_t x = sp->leaf_src[j];
    if (x >= c->snap.N || x < -1) return fail(c, KUEUE_TAS_EINVAL, "splice: leaf source out of range");
    fresh += x < 0 ? 1 : 0;
  }
  if (fresh != sp->num_new) return fail(c, KUEUE_TAS_EINVAL, "splice: num_new is not the count of joined leaves");
  if (sp->num_new > 0 && (!sp->new_free_capacity || !sp->new_tas_usage || !sp->new_free_present ||
                          !sp->new_usage_present || (c->snap.K > 0 && !sp->new_label_values)))
    return fail(c, KUEUE_TAS_EINVAL, "splice: joined rows missing");
  return load_impl(c, d, sp);
}

static int load_impl(kueue_tas_ctx* c, const kueue_tas_snapshot_desc* d, const kueue_tas_splice_desc* sp) {
  if (!c || !d) return KUEUE_TAS_EINVAL;
  if (d->num_levels < 1 || d->num_levels > KUEUE_TAS_MAX_LEVELS) return fail(c, KUEUE_TAS_EINVAL, "num_levels");
  if (d->num_cols < 0 || d->num_cols > KUEUE_TAS_MAX_COLS) return fail(c, KUEUE_TAS_EINVAL, "num_cols");
  HIPCHK(c, hipSetDevice(c->device));
  DevSnap s{};
  s.L = d->num_levels;
  s.R = d->num_cols;
  s.K = d->num_label_cols;
  s.lowest_is_hostname = d->lowest_is_hostname;
  int64_t off = 0;
  int maxD = 0;
  c->h_level_sizes.assign(d->level_sizes, d->level_sizes + s.L);
  for (int l = 0; l < s.L; l++) {  // level starts 16-byte aligned (vectorized leaf scans)
    s.level_size[l] = d->level_sizes[l];
    s.level_off[l] = int32_t(off);
    off += (int64_t(d->level_sizes[l]) + 3) / 4 * 4;
    maxD = std::max(maxD, d->level_sizes[l]);
  }
  s.level_off[s.L] = int32_t(off);
  s.SD = int32_t(off);
  s.N = d->level_sizes[s.L - 1];
  const size_t N = size_t(s.N);
  s.leaf_dead = nullptr;  // a load describes live leaves only
  s.leaf_tag = nullptr;   // leaf tags describe the previous leaves
  s.tag_out = nullptr;
  s.ent_base = nullptr;
  const bool tags_were_on = c->leaf_tags_on;
  // from here on the context's tables describe the new tree: a failure below
  // leaves it unloaded (every call then reports ENOSNAPSHOT) rather than
  // holding the old snapshot beside the new dead-leaf map
  c->loaded = false;
  c->leaf_tags_on = false;
  s.n_live = s.N;
  // a splice keeps the leaves that had left out: their flags move with them
  std::vector<uint8_t> old_dead;
  const int old_N = c->snap.N;
  if (sp) old_dead.swap(c->h_dead);
  c->h_dead.assign(N, 0);
  c->n_dead = 0;
  std::vector<int32_t>& gsrc = c->h_gsrc;  // (kept: no fresh pages per splice)
  if (sp) {  // sources (joined rows numbered in order) and the dead map, in the host pool's static parts
    gsrc.resize(N);
    ktas_pool::HostPool& pool = ktas_pool::HostPool::get();
    const size_t T = pool.parts();
    std::vector<int32_t> joined(T + 1, 0);
    std::vector<int64_t> dead(T, 0);
    auto part_of = [&](size_t b) {
      size_t t = 0;
      while (t + 1 < T && ktas_pool::HostPool::part_begin(N, t + 1, T) <= b) t++;
      return t;
    };
    pool.run_static(N, [&](size_t b, size_t e) {  // pass 1: joined rows per part
      int32_t k = 0;
      for (size_t j = b; j < e; j++) k += sp->leaf_src[j] < 0 ? 1 : 0;
      joined[part_of(b) + 1] = k;
    });
    for (size_t t = 0; t < T; t++) joined[t + 1] += joined[t];
    pool.run_static(N, [&](size_t b, size_t e) {  // pass 2: the numbering and the dead leaves
      const size_t t = part_of(b);
      int32_t k = joined[t];
      int64_t nd = 0;
      for (size_t j = b; j < e; j++) {
        const int32_t x = sp->leaf_src[j];
        gsrc[j] = x >= 0 ? x : -(++k);
        if (x >= 0 && size_t(x) < old_dead.size() && old_dead[size_t(x)]) {
          c->h_dead[j] = 1;
          nd++;
        }
      }
      dead[t] = nd;
    });
    for (int64_t nd : dead) c->n_dead += nd;
  }
  // the re-derived tables go up through one pinned arena (async copies, one
  // stream synchronization at the end) instead of a synchronous copy each
  HIPCHK(c, c->h_tab.reserve(size_t(off) * 8 + N * 9 + (N + 2) * 16 + 4096));
  size_t arena_pos = 0;
  auto stage = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
    if (!bytes) return hipSuccess;
    if (arena_pos + bytes > c->h_tab.n) return hipErrorInvalidValue;  // (the bound above covers every table)
    memcpy(c->h_tab.p + arena_pos, src, bytes);
    const hipError_t e = hipMemcpyAsync(dst, c->h_tab.p + arena_pos, bytes, hipMemcpyHostToDevice, c->stream);
    arena_pos += (bytes + 255) / 256 * 256;
    return e;
  };
  // CSR offsets
  size_t nco = 0;
  for (int l = 0; l + 1 < s.L; l++) {
    s.child_base[l] = int32_t(nco);
    nco += size_t(d->level_sizes[l]) + 1;
  }
  c->level_maxfan.assign(size_t(s.L), 1);  // widest parent per level (select scratch bounds)
  for (int l = 0; l + 1 < s.L; l++) {
    const int32_t* co = d->child_offsets + s.child_base[l];
    int32_t f = 1;
    for (int p = 0; p < d->level_sizes[l]; p++) f = std::max(f, co[p + 1] - co[p]);
    c->level_maxfan[size_t(l)] = f;
  }
  HIPCHK(c, c->d_child_off.reserve(nco));
  if (nco) HIPCHK(c, hipMemcpyAsync(c->d_child_off.p, d->child_offsets, nco * 4, hipMemcpyHostToDevice, c->stream));
  s.child_off = c->d_child_off.p;
  if (sp) {  // the resident leaf columns gathered into the new numbering, the joined rows from the caller
    const int nn = std::max(sp->num_new, 1);
    const bool prof = c->snap.taint_profile != nullptr;
    const bool lab = s.K > 0 && c->snap.label_values != nullptr;
    const bool tags = tags_were_on && sp->new_leaf_tags != nullptr;
    HIPCHK(c, c->sp_free.reserve(size_t(s.R) * N));
    HIPCHK(c, c->sp_usage.reserve(size_t(s.R) * N));
    HIPCHK(c, c->sp_fp.reserve(N));
    HIPCHK(c, c->sp_up.reserve(N));
    if (prof) HIPCHK(c, c->sp_prof.reserve(N));
    if (lab) HIPCHK(c, c->sp_lab.reserve(size_t(s.K) * N));
    if (tags) HIPCHK(c, c->sp_tags.reserve(N));
    HIPCHK(c, c->sp_src.reserve(N));
    // the joined rows: free | usage | free_present | usage_present | profile | labels | tags
    const size_t o_u = size_t(s.R) * nn * 8, o_fp = 2 * o_u, o_up = o_fp + size_t(nn) * 4, o_pr = o_up + size_t(nn) * 4,
                 o_lb = o_pr + size_t(nn) * 4, o_tg = (o_lb + size_t(std::max(s.K, 1)) * nn * 4 + 7) / 8 * 8,
                 rbytes = o_tg + size_t(nn) * 8;
    HIPCHK(c, c->sp_rows.reserve(rbytes));
    // one pinned staging area: leaf sources, then the joined rows
    const size_t o_rows = (N * 4 + 255) / 256 * 256;
    HIPCHK(c, c->h_load.reserve(o_rows + rbytes));
    uint8_t* hl = c->h_load.p;
    if (N) memcpy(hl, gsrc.data(), N * 4);
    uint8_t* hr = hl + o_rows;
    if (sp->num_new > 0) {
      const size_t k = size_t(sp->num_new);
      if (s.R) {
        memcpy(hr, sp->new_free_capacity, size_t(s.R) * k * 8);
        memcpy(hr + o_u, sp->new_tas_usage, size_t(s.R) * k * 8);
      }
      memcpy(hr + o_fp, sp->new_free_present, k * 4);
      memcpy(hr + o_up, sp->new_usage_present, k * 4);
      if (prof && sp->new_taint_profile) memcpy(hr + o_pr, sp->new_taint_profile, k * 4);
      if (lab) memcpy(hr + o_lb, sp->new_label_values, size_t(s.K) * k * 4);
      if (tags) memcpy(hr + o_tg, sp->new_leaf_tags, k * 8);
      for (size_t i = 0; i < k; i++) {
        if (sp->new_taint_profile) c->num_profiles = std::max(c->num_profiles, sp->new_taint_profile[i] + 1);
        for (int q = 0; q < std::min(s.K, kStagedLabels) && sp->new_label_values; q++)
          if (uint32_t(sp->new_label_values[size_t(q) * k + i]) > 0xffffu) c->labels16 = false;
      }
    }
    if (N) HIPCHK(c, hipMemcpyAsync(c->sp_src.p, hl, N * 4, hipMemcpyHostToDevice, c->stream));
    if (sp->num_new > 0) HIPCHK(c, hipMemcpyAsync(c->sp_rows.p, hr, rbytes, hipMemcpyHostToDevice, c->stream));
    const uint8_t* rows = c->sp_rows.p;
    if (N) {
      hipLaunchKernelGGL(splice_leaves_kernel, dim3(unsigned((N + 255) / 256)), dim3(256), 0, c->stream, c->sp_src.p,
                         int(N), old_N, s.R, lab ? s.K : 0, nn, c->d_free.p, c->d_usage.p, c->d_free_present.p,
                         c->d_usage_present.p, prof ? c->d_taint_profile.p : nullptr, lab ? c->d_labels.p : nullptr,
                         reinterpret_cast<const int64_t*>(rows), reinterpret_cast<const int64_t*>(rows + o_u),
                         reinterpret_cast<const uint32_t*>(rows + o_fp), reinterpret_cast<const uint32_t*>(rows + o_up),
                         (prof && sp->new_taint_profile) ? reinterpret_cast<const int32_t*>(rows + o_pr) : nullptr,
                         reinterpret_cast<const int32_t*>(rows + o_lb), c->sp_free.p, c->sp_usage.p, c->sp_fp.p,
                         c->sp_up.p, prof ? c->sp_prof.p : nullptr, lab ? c->sp_lab.p : nullptr,
                         tags ? c->d_leaf_tags.p : nullptr, reinterpret_cast<const uint64_t*>(rows + o_tg),
                         tags ? c->sp_tags.p : nullptr);
      HIPCHK(c, hipGetLastError());
    }
    // the gathered columns go live; the previous ones become the next
    // splice's targets (stream order puts every later kernel after the gather)
    c->d_free.swap(c->sp_free);
    c->d_usage.swap(c->sp_usage);
    c->d_free_present.swap(c->sp_fp);
    c->d_usage_present.swap(c->sp_up);
    if (prof) c->d_taint_profile.swap(c->sp_prof);
    if (lab) c->d_labels.swap(c->sp_lab);
    if (tags) c->d_leaf_tags.swap(c->sp_tags);
    c->leaf_tags_on = tags;
    s.free_cap = c->d_free.p;
    s.tas_usage = c->d_usage.p;
    s.free_present = c->d_free_present.p;
    s.usage_present = c->d_usage_present.p;
    s.taint_profile = prof ? c->d_taint_profile.p : nullptr;
    s.label_values = lab ? c->d_labels.p : nullptr;
    if (c->n_dead > 0) {  // the leaves that had left, at their new indices
      HIPCHK(c, c->d_dead.reserve(N));
      HIPCHK(c, stage(c->d_dead.p, c->h_dead.data(), N));
      s.leaf_dead = c->d_dead.p;
      s.n_live = int32_t(int64_t(N) - c->n_dead);
    }
  } else {  // (leaf columns with headroom: a later splice's gather targets then fit without a reallocation)
  HIPCHK(c, c->d_free.reserve(size_t(s.R) * N));
  HIPCHK(c, c->d_usage.reserve(size_t(s.R) * N));
  if (s.R && N) {
    HIPCHK(c, hipMemcpyAsync(c->d_free.p, d->free_capacity, size_t(s.R) * N * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_usage.p, d->tas_usage, size_t(s.R) * N * 8, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(c, c->d_free_present.reserve(N));
  HIPCHK(c, c->d_usage_present.reserve(N));
  if (N) {
    HIPCHK(c, hipMemcpyAsync(c->d_free_present.p, d->free_present, N * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_usage_present.p, d->usage_present, N * 4, hipMemcpyHostToDevice, c->stream));
  }
  s.free_cap = c->d_free.p;
  s.tas_usage = c->d_usage.p;
  s.free_present = c->d_free_present.p;
  s.usage_present = c->d_usage_present.p;
  s.taint_profile = nullptr;
  c->num_profiles = 1;
  if (d->taint_profile && N) {
    for (size_t i = 0; i < N; i++) c->num_profiles = std::max(c->num_profiles, d->taint_profile[i] + 1);
    HIPCHK(c, c->d_taint_profile.reserve(N));
    HIPCHK(c, hipMemcpyAsync(c->d_taint_profile.p, d->taint_profile, N * 4, hipMemcpyHostToDevice, c->stream));
    s.taint_profile = c->d_taint_profile.p;
  }
  s.label_values = nullptr;
  c->labels16 = true;
  for (int k = 0; k < std::min(s.K, kStagedLabels) && d->label_values; k++)
    for (size_t i = 0; i < N && c->labels16; i++) c->labels16 = uint32_t(d->label_values[size_t(k) * N + i]) <= 0xffffu;
  if (s.K > 0 && d->label_values && N) {
    HIPCHK(c, c->d_labels.reserve(size_t(s.K) * N));
    HIPCHK(c, hipMemcpyAsync(c->d_labels.p, d->label_values, size_t(s.K) * N * 4, hipMemcpyHostToDevice, c->stream));
    s.label_values = c->d_labels.p;
  }
  }
  s.id_rank = nullptr;
  if (d->domain_id_rank && off) {  // re-laid out on the padded level offsets, in the pinned arena itself
    HIPCHK(c, c->d_id_rank.reserve(size_t(off)));
    const size_t bytes = size_t(off) * 4;
    if (arena_pos + bytes > c->h_tab.n) return fail(c, KUEUE_TAS_EINVAL, "load: staging arena");
    int32_t* ranks = reinterpret_cast<int32_t*>(c->h_tab.p + arena_pos);
    int64_t src = 0;
    for (int l = 0; l < s.L; l++) {
      const int32_t b = s.level_off[l], sz = d->level_sizes[l];
      memcpy(ranks + b, d->domain_id_rank + src, size_t(sz) * 4);
      for (int32_t i = b + sz; i < s.level_off[l + 1]; i++) ranks[i] = 0;
      src += sz;
    }
    HIPCHK(c, hipMemcpyAsync(c->d_id_rank.p, ranks, bytes, hipMemcpyHostToDevice, c->stream));
    arena_pos += (bytes + 255) / 256 * 256;
    s.id_rank = c->d_id_rank.p;
  }
  // leaves' parents with a uniform power-of-two fan-out F <= 64 in leaf order:
  // the staged fill rolls them up itself (one wave holds whole parents)
  c->rack_fanout = 0;
  if (s.L >= 2 && d->level_sizes[s.L - 2] > 0 && d->child_offsets) {
    const int P = d->level_sizes[s.L - 2];
    const int F = s.N / P;
    if (F > 0 && F <= kWave && (F & (F - 1)) == 0 && int64_t(F) * P == s.N) {
      const int32_t* co = d->child_offsets + s.child_base[s.L - 2];
      bool ok = true;
      for (int p = 0; p <= P && ok; p++) ok = co[p] == p * F;
      if (ok) c->rack_fanout = F;
    }
  }
  // otherwise, parents of at most 64 leaves: pack whole parents into waves
  // (first fit in leaf order) so the fill still rolls them up in the wave
  s.wave_tab = nullptr;
  s.n_wave_slots = 0;
  s.leaf_parent = nullptr;
  s.wave_tab2 = nullptr;
  s.n_wave_slots2 = 0;
  s.ragged_max_fan = 0;
  s.wide_parents = nullptr;
  s.n_wide = 0;
  // and the same packing into 128-leaf slots for fill_pair_kernel's two
  // leaves per lane (parents of at most 128 leaves; a wider parent takes
  // slots of its own, one per 128-leaf piece, flagged wide)
  if (c->rack_fanout == 0 && s.L >= 2 && d->level_sizes[s.L - 2] > 0 && d->child_offsets && s.N > 0) {
    const int P = d->level_sizes[s.L - 2];
    const int32_t* co = d->child_offsets + s.child_base[s.L - 2];
    bool ok = co[0] == 0 && co[P] == s.N;
    std::vector<int2> tab;
    std::vector<int32_t> wide;
    int cb = 0, cn = 0, fmax = 0;
    for (int p = 0; p < P && ok; p++) {
      const int f = co[p + 1] - co[p];
      if (f < 1) {
        ok = false;
        break;
      }
      fmax = std::max(fmax, f);
      if (f > 2 * kWave) {  // pieces of their own
        if (cn) tab.push_back(make_int2(cb, cn));
        for (int k = co[p]; k < co[p + 1]; k += 2 * kWave)
          tab.push_back(make_int2(k, std::min(2 * kWave, co[p + 1] - k) | (1 << 16)));
        wide.push_back(p);
        cb = co[p + 1];
        cn = 0;
        continue;
      }
      if (cn + f > 2 * kWave) {
        tab.push_back(make_int2(cb, cn));
        cb = co[p];
        cn = 0;
      }
      cn += f;
    }
    if (ok) {
      if (cn) tab.push_back(make_int2(cb, cn));
      if (!wide.empty()) {
        HIPCHK(c, c->d_wide.reserve(wide.size()));
        HIPCHK(c, stage(c->d_wide.p, wide.data(), wide.size() * 4));
        s.wide_parents = c->d_wide.p;
        s.n_wide = int32_t(wide.size());
      }
      HIPCHK(c, c->d_wave_tab2.reserve(tab.size()));
      HIPCHK(c, stage(c->d_wave_tab2.p, tab.data(), tab.size() * sizeof(int2)));
      HIPCHK(c, c->d_leaf_parent.reserve(N));  // (domain_parents_kernel below)
      s.wave_tab2 = c->d_wave_tab2.p;
      s.n_wave_slots2 = int32_t(tab.size());
      s.leaf_parent = c->d_leaf_parent.p;
      s.ragged_max_fan = fmax;
    }
  }
  if (c->rack_fanout == 0 && s.L >= 2 && d->level_sizes[s.L - 2] > 0 && d->child_offsets && s.N > 0) {
    const int P = d->level_sizes[s.L - 2];
    const int32_t* co = d->child_offsets + s.child_base[s.L - 2];
    bool ok = co[0] == 0 && co[P] == s.N;
    std::vector<int2> tab;
    int cb = 0, cn = 0;
    for (int p = 0; p < P && ok; p++) {
      const int f = co[p + 1] - co[p];
      if (f < 1 || f > kWave) {
        ok = false;
        break;
      }
      if (cn + f > kWave) {
        tab.push_back(make_int2(cb, cn));
        cb = co[p];
        cn = 0;
      }
      cn += f;
    }
    if (ok) {
      tab.push_back(make_int2(cb, cn));
      HIPCHK(c, c->d_wave_tab.reserve(tab.size()));
      HIPCHK(c, stage(c->d_wave_tab.p, tab.data(), tab.size() * sizeof(int2)));
      HIPCHK(c, c->d_leaf_parent.reserve(N));
      s.wave_tab = c->d_wave_tab.p;
      s.n_wave_slots = int32_t(tab.size());
      s.leaf_parent = c->d_leaf_parent.p;
      c->rack_fanout = -1;
    }
  }
  // parent global domain id of every domain (v1beta2 leaf-mode encoder) and
  // the ragged fills' leaf parents, derived on the device from the offsets
  // just uploaded (no O(N) host pass or upload per load / splice)
  HIPCHK(c, c->d_parent.reserve(size_t(std::max<int64_t>(off, 1))));
  if (off > 0) {
    hipLaunchKernelGGL(domain_parents_kernel, dim3(unsigned((off + 255) / 256)), dim3(256), 0, c->stream, s,
                       c->d_parent.p, s.leaf_parent ? c->d_leaf_parent.p : nullptr);
    HIPCHK(c, hipGetLastError());
  }
  c->names_loaded = false;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->snap = s;
  c->maxD = maxD;
  c->loaded = true;
  (sp ? c->n_splices : c->n_loads)++;
  return KUEUE_TAS_OK;
}

int kueue_tas_device_bytes(kueue_tas_ctx* c, int64_t* total, int64_t* phase2) {
  if (!c) return KUEUE_TAS_EINVAL;
  int64_t t = 0;
  for (const DevBufLink* b = c->dev_bufs; b; b = b->next) t += int64_t(b->bytes);
  if (total) *total = t;
  if (phase2) *phase2 = int64_t(c->d_counters.bytes + c->d_overlay.bytes + c->d_tags.bytes + c->d_scratch.bytes);
  return KUEUE_TAS_OK;
}

int kueue_tas_snapshot_counters(kueue_tas_ctx* c, int64_t* loads, int64_t* splices) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (loads) *loads = c->n_loads;
  if (splices) *splices = c->n_splices;
  return KUEUE_TAS_OK;
}

int kueue_tas_snapshot_load_names(kueue_tas_ctx* c, const char* bytes, size_t nbytes, const int64_t* offsets) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (!offsets || (nbytes && !bytes)) return fail(c, KUEUE_TAS_EINVAL, "null argument");
  size_t total = 0;
  for (int l = 0; l < c->snap.L; l++) total += size_t(c->snap.level_size[l]);
  if (offsets[0] != 0 || size_t(offsets[total]) != nbytes) return fail(c, KUEUE_TAS_EINVAL, "name offsets");
  for (size_t i = 0; i < total; i++)
    if (offsets[i + 1] < offsets[i]) return fail(c, KUEUE_TAS_EINVAL, "name offsets not monotone");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, c->d_names.ensure(nbytes));
  HIPCHK(c, c->d_name_off.ensure(total + 1));
  if (nbytes) HIPCHK(c, hipMemcpy(c->d_names.p, bytes, nbytes, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_name_off.p, offsets, (total + 1) * 8, hipMemcpyHostToDevice));
  c->names_loaded = true;
  return KUEUE_TAS_OK;
}

static int run_encode(kueue_tas_ctx* c, EncodeArgs& a, size_t n_assign, kueue_tas_level_enc* out, int32_t* same) {
  const size_t nout = n_assign * size_t(a.num_levels);
  HIPCHK(c, c->d_enc_out.ensure(nout));
  HIPCHK(c, c->d_enc_same.ensure(n_assign));
  a.out = c->d_enc_out.p;
  a.same = c->d_enc_same.p;
  a.n_assign = int32_t(n_assign);
  hipLaunchKernelGGL(encode_v1beta2_kernel, dim3(unsigned(n_assign), unsigned(a.num_levels)), dim3(256), 0, c->stream,
                     a);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, a.out, nout * sizeof(kueue_tas_level_enc), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(same, a.same, n_assign * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KUEUE_TAS_OK;
}

int kueue_tas_encode_v1beta2(kueue_tas_ctx* c, const char* bytes, size_t nbytes, const int64_t* str_off,
                             size_t num_strings, const int32_t* ids, const int32_t* counts, const int64_t* off,
                             size_t n_assign, int32_t num_levels, kueue_tas_level_enc* out, int32_t* same_counts) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (n_assign == 0) return KUEUE_TAS_OK;
  if (num_levels < 1 || num_levels > 65535 || !str_off || !off || !out || !same_counts || (nbytes && !bytes))
    return fail(c, KUEUE_TAS_EINVAL, "encode arguments");
  if (n_assign > 0x7fffffff) return fail(c, KUEUE_TAS_EINVAL, "too many assignments");
  // host-side shape checks: every id and offset the kernel will touch
  if (off[0] < 0) return fail(c, KUEUE_TAS_EINVAL, "assignment offsets");
  for (size_t i = 0; i < n_assign; i++)
    if (off[i + 1] < off[i]) return fail(c, KUEUE_TAS_EINVAL, "assignment offsets not monotone");
  const size_t ndom = size_t(off[n_assign]);
  if (ndom && (!ids || !counts)) return fail(c, KUEUE_TAS_EINVAL, "null ids/counts");
  if (str_off[0] < 0 || size_t(str_off[num_strings]) > nbytes) return fail(c, KUEUE_TAS_EINVAL, "string offsets");
  for (size_t i = 0; i < num_strings; i++)
    if (str_off[i + 1] < str_off[i]) return fail(c, KUEUE_TAS_EINVAL, "string offsets not monotone");
  for (size_t i = 0; i < ndom * size_t(num_levels); i++)
    if (ids[i] < 0 || size_t(ids[i]) >= num_strings) return fail(c, KUEUE_TAS_EINVAL, "string id out of range");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, c->d_enc_bytes.ensure(nbytes));
  HIPCHK(c, c->d_enc_stroff.ensure(num_strings + 1));
  HIPCHK(c, c->d_enc_off.ensure(n_assign + 1));
  HIPCHK(c, c->d_enc_ids.ensure(ndom * size_t(num_levels)));
  HIPCHK(c, c->d_enc_counts.ensure(ndom));
  if (nbytes) HIPCHK(c, hipMemcpyAsync(c->d_enc_bytes.p, bytes, nbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_enc_stroff.p, str_off, (num_strings + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_enc_off.p, off, (n_assign + 1) * 8, hipMemcpyHostToDevice, c->stream));
  if (ndom) {
    HIPCHK(c, hipMemcpyAsync(c->d_enc_ids.p, ids, ndom * size_t(num_levels) * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_enc_counts.p, counts, ndom * 4, hipMemcpyHostToDevice, c->stream));
  }
  EncodeArgs a{};
  a.bytes = c->d_enc_bytes.p;
  a.str_off = c->d_enc_stroff.p;
  a.ids = c->d_enc_ids.p;
  a.counts = c->d_enc_counts.p;
  a.off = c->d_enc_off.p;
  a.num_levels = num_levels;
  return run_encode(c, a, n_assign, out, same_counts);
}

int kueue_tas_encode_v1beta2_leaves(kueue_tas_ctx* c, const int32_t* pairs, const int64_t* off, size_t n_assign,
                                    int32_t first_level, kueue_tas_level_enc* out, int32_t* same_counts) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (!c->names_loaded) return fail(c, KUEUE_TAS_EINVAL, "no names loaded (kueue_tas_snapshot_load_names)");
  if (n_assign == 0) return KUEUE_TAS_OK;
  const DevSnap& s = c->snap;
  if (first_level < 0 || first_level >= s.L || !off || !out || !same_counts)
    return fail(c, KUEUE_TAS_EINVAL, "encode arguments");
  if (n_assign > 0x7fffffff) return fail(c, KUEUE_TAS_EINVAL, "too many assignments");
  if (off[0] < 0) return fail(c, KUEUE_TAS_EINVAL, "assignment offsets");
  for (size_t i = 0; i < n_assign; i++)
    if (off[i + 1] < off[i]) return fail(c, KUEUE_TAS_EINVAL, "assignment offsets not monotone");
  const size_t npairs = size_t(off[n_assign]);
  if (npairs && !pairs) return fail(c, KUEUE_TAS_EINVAL, "null pairs");
  for (size_t j = size_t(off[0]); j < npairs; j++)
    if (pairs[2 * j] < 0 || pairs[2 * j] >= s.N) return fail(c, KUEUE_TAS_EINVAL, "leaf out of range");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, c->d_enc_counts.ensure(2 * npairs));  // the pairs
  HIPCHK(c, c->d_enc_off.ensure(n_assign + 1));
  if (npairs)
    HIPCHK(c, hipMemcpyAsync(c->d_enc_counts.p, pairs, npairs * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_enc_off.p, off, (n_assign + 1) * 8, hipMemcpyHostToDevice, c->stream));
  EncodeArgs a{};
  a.bytes = c->d_names.p;
  a.str_off = c->d_name_off.p;
  a.pairs = c->d_enc_counts.p;
  a.parent = c->d_parent.p;
  a.off = c->d_enc_off.p;
  a.num_levels = s.L - first_level;
  a.first_level = first_level;
  a.L = s.L;
  int64_t base = 0;
  for (int l = 0; l < s.L; l++) {
    a.level_off[l] = s.level_off[l];
    a.name_base[l] = base;
    base += s.level_size[l];
  }
  return run_encode(c, a, n_assign, out, same_counts);
}

static int apply_deltas_impl(kueue_tas_ctx* c, const kueue_tas_delta* deltas, size_t n,
                             const uint32_t* usage_present_or_null, bool mirrored);
int kueue_tas_snapshot_apply_deltas(kueue_tas_ctx* c, const kueue_tas_delta* deltas, size_t n,
                                    const uint32_t* usage_present_or_null) {
  return apply_deltas_impl(c, deltas, n, usage_present_or_null, false);
}
int kueue_tas_snapshot_apply_deltas_mirrored(kueue_tas_ctx* c, const kueue_tas_delta* deltas, size_t n) {
  return apply_deltas_impl(c, deltas, n, nullptr, true);
}
static int apply_deltas_impl(kueue_tas_ctx* c, const kueue_tas_delta* deltas, size_t n,
                             const uint32_t* usage_present_or_null, bool mirrored) {
  if (!c || !c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot");
  HIPCHK(c, hipSetDevice(c->device));
  if (n) {
    // the records through pinned staging: an async copy, no stream sync (the
    // launches that read the usage follow on the same stream); the previous
    // call's copy must be done before its buffer is rewritten
    if (c->ev_deltas) HIPCHK(c, hipEventSynchronize(c->ev_deltas));
    else HIPCHK(c, hipEventCreateWithFlags(&c->ev_deltas, hipEventDisableTiming));
    HIPCHK(c, c->h_deltas.reserve(n));
    // range check and copy in one pass (a whole batch's admission is ~16k
    // records: over the host pool's static parts when large)
    const int32_t N = c->snap.N, R = c->snap.R;
    kueue_tas_delta* dst = c->h_deltas.p;
    std::atomic<bool> bad{false};
    auto check_copy = [&](size_t i0, size_t i1) {
      bool ok = true;
      for (size_t i = i0; i < i1; i++) {
        const kueue_tas_delta x = deltas[i];
        ok &= x.leaf >= 0 && x.leaf < N && x.col >= 0 && x.col < R;
        dst[i] = x;
      }
      if (!ok) bad.store(true, std::memory_order_relaxed);
    };
    if (n >= 8192) ktas_pool::HostPool::get().run_static(n, check_copy);
    else check_copy(0, n);
    if (bad.load()) return fail(c, KUEUE_TAS_EINVAL, "delta out of range");
    HIPCHK(c, c->d_deltas.ensure(n));
    HIPCHK(c, hipMemcpyAsync(c->d_deltas.p, c->h_deltas.p, n * sizeof(kueue_tas_delta), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_deltas, c->stream));
    int blocks = int((n + 255) / 256);
    const bool sh = mirrored && c->shadow_ok;  // no shadow yet: the next mark copies the usage whole
    hipLaunchKernelGGL(apply_deltas_kernel, dim3(blocks), dim3(256), 0, c->stream, c->d_usage.p, c->d_usage_present.p,
                       c->snap.N, c->d_deltas.p, int(n), sh ? c->d_ushadow.p : nullptr,
                       sh ? c->d_pshadow.p : nullptr);
    HIPCHK(c, hipGetLastError());
  }
  if (usage_present_or_null) {
    HIPCHK(c, hipMemcpyAsync(c->d_usage_present.p, usage_present_or_null, size_t(c->snap.N) * 4, hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // (the caller's array)
  }
  return KUEUE_TAS_OK;
}

int kueue_tas_snapshot_usage_mark(kueue_tas_ctx* c) {
  if (!c || !c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t N = size_t(c->snap.N), R = size_t(c->snap.R);
  HIPCHK(c, c->d_ushadow.reserve(N * R));  // (headroom: splices grow N a few leaves at a time)
  HIPCHK(c, c->d_pshadow.reserve(N));
  if (N * R) HIPCHK(c, hipMemcpyAsync(c->d_ushadow.p, c->d_usage.p, N * R * 8, hipMemcpyDeviceToDevice, c->stream));
  if (N) HIPCHK(c, hipMemcpyAsync(c->d_pshadow.p, c->d_usage_present.p, N * 4, hipMemcpyDeviceToDevice, c->stream));
  c->shadow_ok = true;
  return KUEUE_TAS_OK;
}

int kueue_tas_snapshot_usage_changes(kueue_tas_ctx* c, const kueue_tas_delta** changes, size_t* n) {
  if (!c || !changes || !n) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot");
  if (!c->shadow_ok) return fail(c, KUEUE_TAS_EINVAL, "usage_changes before usage_mark");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t N = size_t(c->snap.N), R = size_t(c->snap.R);
  HIPCHK(c, c->d_uchg.ensure(std::max<size_t>(N * R, 1)));
  HIPCHK(c, c->d_uchg_n.ensure(1));
  HIPCHK(c, c->h_uchg_n.ensure(1));
  HIPCHK(c, hipMemsetAsync(c->d_uchg_n.p, 0, 4, c->stream));
  if (N * R) {
    hipLaunchKernelGGL(usage_diff_kernel, dim3(unsigned((N * R + 255) / 256)), dim3(256), 0, c->stream, c->d_usage.p,
                       c->d_usage_present.p, c->d_ushadow.p, c->d_pshadow.p, int(N), int(R), c->d_uchg.p, c->d_uchg_n.p);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipMemcpyAsync(c->h_uchg_n.p, c->d_uchg_n.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t k = size_t(c->h_uchg_n.p[0]);
  c->uchg.resize(k);
  if (k) HIPCHK(c, hipMemcpy(c->uchg.data(), c->d_uchg.p, k * sizeof(kueue_tas_delta), hipMemcpyDeviceToHost));
  *changes = c->uchg.data();
  *n = k;
  return kueue_tas_snapshot_usage_mark(c);
}

int kueue_tas_snapshot_set_free(kueue_tas_ctx* c, const int32_t* leaves, size_t n, const int64_t* rows,
                                const uint32_t* free_present) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (n == 0) return KUEUE_TAS_OK;
  if (!leaves || !rows || !free_present) return fail(c, KUEUE_TAS_EINVAL, "null argument");
  for (size_t i = 0; i < n; i++)
    if (leaves[i] < 0 || leaves[i] >= c->snap.N) return fail(c, KUEUE_TAS_EINVAL, "set_free leaf out of range");
  if (!distinct_leaves(leaves, n)) return fail(c, KUEUE_TAS_EINVAL, "repeated leaf in set_free");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t R = size_t(c->snap.R);
  const size_t rows_off = (n * 4 + 7) / 8 * 8;
  const size_t pres_off = rows_off + n * R * 8;
  HIPCHK(c, c->d_setfree.ensure(pres_off + n * 4));
  uint8_t* d = c->d_setfree.p;
  HIPCHK(c, hipMemcpyAsync(d, leaves, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d + rows_off, rows, n * R * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d + pres_off, free_present, n * 4, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(set_free_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, c->stream, c->d_free.p,
                     c->d_free_present.p, c->snap.N, c->snap.R, reinterpret_cast<const int32_t*>(d),
                     reinterpret_cast<const int64_t*>(d + rows_off), reinterpret_cast<const uint32_t*>(d + pres_off),
                     int(n));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KUEUE_TAS_OK;
}

int kueue_tas_snapshot_set_leaf_live(kueue_tas_ctx* c, const int32_t* leaves, size_t n, const int32_t* live) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (n == 0) return KUEUE_TAS_OK;
  if (!leaves || !live) return fail(c, KUEUE_TAS_EINVAL, "null argument");
  for (size_t i = 0; i < n; i++)
    if (leaves[i] < 0 || leaves[i] >= c->snap.N) return fail(c, KUEUE_TAS_EINVAL, "leaf out of range");
  if (!distinct_leaves(leaves, n)) return fail(c, KUEUE_TAS_EINVAL, "repeated leaf in set_leaf_live");
  for (size_t i = 0; i < n; i++) {
    const uint8_t d = live[i] ? 0 : 1;
    c->n_dead += int64_t(d) - int64_t(c->h_dead[size_t(leaves[i])]);
    c->h_dead[size_t(leaves[i])] = d;
  }
  HIPCHK(c, hipSetDevice(c->device));
  c->snap.n_live = int32_t(int64_t(c->snap.N) - c->n_dead);
  const bool was_dense = c->snap.leaf_dead != nullptr;
  if (c->n_dead == 0) {
    c->snap.leaf_dead = nullptr;
    return KUEUE_TAS_OK;
  }
  std::vector<int32_t> lv;  // read by the async copy: lives until the synchronize below
  if (!was_dense) {  // first dead leaf: the whole map (the device copy was dropped while all leaves lived)
    HIPCHK(c, c->d_dead.reserve(size_t(c->snap.N)));
    HIPCHK(c, hipMemcpyAsync(c->d_dead.p, c->h_dead.data(), size_t(c->snap.N), hipMemcpyHostToDevice, c->stream));
  } else {  // scatter the changed leaves
    lv.resize(2 * n);
    for (size_t i = 0; i < n; i++) lv[2 * i] = leaves[i], lv[2 * i + 1] = live[i] ? 1 : 0;
    HIPCHK(c, c->d_setfree.ensure(lv.size() * 4));
    HIPCHK(c, hipMemcpyAsync(c->d_setfree.p, lv.data(), lv.size() * 4, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(set_leaf_dead_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, c->stream, c->d_dead.p,
                       reinterpret_cast<const int32_t*>(c->d_setfree.p), int(n));
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->snap.leaf_dead = c->d_dead.p;
  return KUEUE_TAS_OK;
}

int kueue_tas_snapshot_set_leaf_attrs(kueue_tas_ctx* c, const int32_t* leaves, size_t n, const int32_t* profiles,
                                      const int32_t* labels) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (n == 0) return KUEUE_TAS_OK;
  if (!leaves || !profiles) return fail(c, KUEUE_TAS_EINVAL, "null argument");
  const size_t K = size_t(c->snap.K);
  if (K && !labels) return fail(c, KUEUE_TAS_EINVAL, "labels required (snapshot has label columns)");
  if (!c->snap.taint_profile) return fail(c, KUEUE_TAS_EINVAL, "snapshot has no taint profiles");
  for (size_t i = 0; i < n; i++) {
    if (leaves[i] < 0 || leaves[i] >= c->snap.N) return fail(c, KUEUE_TAS_EINVAL, "leaf out of range");
    if (profiles[i] < 0) return fail(c, KUEUE_TAS_EINVAL, "negative taint profile");
  }
  if (!distinct_leaves(leaves, n)) return fail(c, KUEUE_TAS_EINVAL, "repeated leaf in set_leaf_attrs");
  HIPCHK(c, hipSetDevice(c->device));
  for (size_t i = 0; i < n; i++) c->num_profiles = std::max(c->num_profiles, profiles[i] + 1);
  for (size_t i = 0; i < n && K; i++)  // the packed nodeSelector compare needs 16-bit staged ids
    for (size_t k = 0; k < std::min<size_t>(K, size_t(kStagedLabels)); k++)
      if (uint32_t(labels[i * K + k]) > 0xffffu) c->labels16 = false;
  const size_t prof_off = n * 4, lab_off = 2 * n * 4;
  HIPCHK(c, c->d_setfree.ensure(lab_off + n * K * 4));
  uint8_t* d = c->d_setfree.p;
  HIPCHK(c, hipMemcpyAsync(d, leaves, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d + prof_off, profiles, n * 4, hipMemcpyHostToDevice, c->stream));
  if (K) HIPCHK(c, hipMemcpyAsync(d + lab_off, labels, n * K * 4, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(set_leaf_attrs_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, c->stream,
                     c->d_taint_profile.p, K ? c->d_labels.p : nullptr, c->snap.N, c->snap.K,
                     reinterpret_cast<const int32_t*>(d), reinterpret_cast<const int32_t*>(d + prof_off),
                     reinterpret_cast<const int32_t*>(d + lab_off), int(n));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KUEUE_TAS_OK;
}

int kueue_tas_fits(kueue_tas_ctx* c, const kueue_tas_fits_req* reqs, size_t n, const kueue_tas_fits_term* terms,
                   size_t num_terms, int32_t* fits) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (n == 0) return KUEUE_TAS_OK;
  if (!reqs || !fits || (num_terms && !terms)) return fail(c, KUEUE_TAS_EINVAL, "null argument");
  for (size_t i = 0; i < n; i++) {
    const kueue_tas_fits_req& r = reqs[i];
    if (r.leaf >= c->snap.N || r.num_terms < 0 || r.term_begin < 0 ||
        size_t(r.term_begin) + size_t(r.num_terms) > num_terms)
      return fail(c, KUEUE_TAS_EINVAL, "fits request out of range");
    for (int k = 0; k < r.num_terms; k++)
      if (terms[r.term_begin + k].col >= c->snap.R) return fail(c, KUEUE_TAS_EINVAL, "fits term column out of range");
  }
  HIPCHK(c, hipSetDevice(c->device));
  const size_t bytes = n * sizeof(kueue_tas_fits_req) + num_terms * sizeof(kueue_tas_fits_term) + n * 4;
  HIPCHK(c, c->d_fits.ensure(bytes));
  uint8_t* d = c->d_fits.p;
  auto* d_reqs = reinterpret_cast<kueue_tas_fits_req*>(d);
  auto* d_terms = reinterpret_cast<kueue_tas_fits_term*>(d + n * sizeof(kueue_tas_fits_req));
  auto* d_out = reinterpret_cast<int32_t*>(d + n * sizeof(kueue_tas_fits_req) + num_terms * sizeof(kueue_tas_fits_term));
  HIPCHK(c, hipMemcpyAsync(d_reqs, reqs, n * sizeof(kueue_tas_fits_req), hipMemcpyHostToDevice, c->stream));
  if (num_terms)
    HIPCHK(c, hipMemcpyAsync(d_terms, terms, num_terms * sizeof(kueue_tas_fits_term), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(fits_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, c->stream, c->snap, d_reqs, int(n),
                     d_terms, d_out);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(fits, d_out, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KUEUE_TAS_OK;
}

static size_t admit_al(size_t b) { return (b + 255) / 256 * 256; }
// kueue_tas_admit's device buffer (c->d_fits): the uploaded part [0, up_bytes)
// (records, terms, workload offsets, record -> workload, phase-1 flags, the
// exact flag, the per-column totals), then the verdicts (+ diagnostics), the
// phase-1 records, the window kernel's lists, the per-leaf minima, the touched
// bitmap and the window phases' state.
struct AdmitLayout {
  size_t o_terms, o_off, o_recwl, o_fit0, o_exact, o_total, up_bytes;
  size_t o_out, o_recs, o_dep, o_todo, o_todor, o_minc, o_bits, o_state, end;
};
static AdmitLayout admit_layout(size_t n, size_t num_terms, size_t n_wl, size_t N) {
  AdmitLayout L{};
  L.o_terms = admit_al(n * sizeof(kueue_tas_fits_req));
  L.o_off = L.o_terms + admit_al(num_terms * sizeof(kueue_tas_fits_term));
  L.o_recwl = L.o_off + admit_al((n_wl + 1) * 8);
  L.o_fit0 = L.o_recwl + admit_al(n * 4);
  L.o_exact = L.o_fit0 + admit_al(n_wl * 4);
  L.o_total = L.o_exact + 256;
  L.up_bytes = L.o_total + KUEUE_TAS_MAX_COLS * 8;
  L.o_out = admit_al(L.up_bytes);
  L.o_recs = L.o_out + admit_al((n_wl + 3) * 4);  // + three diagnostics words (admit_window_kernel)
  L.o_dep = L.o_recs + admit_al(n * sizeof(AdmitRec));
  L.o_todo = L.o_dep + admit_al(n_wl * 4);
  L.o_todor = L.o_todo + admit_al((n_wl + 1) * 4);
  L.o_minc = L.o_todor + admit_al(n_wl * 16);
  L.o_bits = L.o_minc + admit_al(N * 4);
  L.o_state = L.o_bits + admit_al((N + 31) / 32 * 4);  // admit_window_kernel's phase state (AdmitState)
  L.end = L.o_state + 256;
  return L;
}
static int admit_run(kueue_tas_ctx* c, const AdmitLayout& L, uint8_t* d, const kueue_tas_fits_term* d_terms, size_t n,
                     size_t n_wl, int32_t pods_col, bool exact);

int kueue_tas_admit(kueue_tas_ctx* c, const kueue_tas_fits_req* reqs, size_t n, const kueue_tas_fits_term* terms,
                    size_t num_terms, const int64_t* wl_off, size_t n_wl, int32_t pods_col, int32_t* admitted) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (n_wl == 0) return KUEUE_TAS_OK;
  if (!wl_off || !admitted || (n && !reqs) || (num_terms && !terms)) return fail(c, KUEUE_TAS_EINVAL, "null argument");
  if (pods_col < -1 || pods_col >= c->snap.R) return fail(c, KUEUE_TAS_EINVAL, "pods column out of range");
  if (wl_off[0] != 0 || size_t(wl_off[n_wl]) != n) return fail(c, KUEUE_TAS_EINVAL, "workload offsets");
  for (size_t w = 0; w < n_wl; w++)
    if (wl_off[w + 1] < wl_off[w]) return fail(c, KUEUE_TAS_EINVAL, "workload offsets not monotone");
  // per record on the host pool: the range checks, and for the monotone
  // shortcut (admit_fit0_kernel) the most usage this call can add per column
  // — the shortcut holds only for non-negative values and counts whose totals
  // stay below 2^61 (with every capacity and usage value below 2^61, checked
  // on the device, no int64 arithmetic of the call wraps)
  ktas_pool::HostPool& pool = ktas_pool::HostPool::get();
  const size_t nparts = pool.parts();
  struct alignas(64) AdmitPart {  // one per worker, on cache lines of its own
    __int128 total[KUEUE_TAS_MAX_COLS];
    bool exact;
    int err;  // 0, 1: record out of range, 2: term column out of range
  };
  std::vector<AdmitPart> parts(nparts);
  const int32_t snapN = c->snap.N, snapR = c->snap.R;
  pool.run_static(n, [&](size_t i0, size_t i1) {
    size_t t = 0;
    while (t + 1 < nparts && ktas_pool::HostPool::part_begin(n, t + 1, nparts) <= i0) t++;
    __int128 tot[KUEUE_TAS_MAX_COLS] = {};  // accumulated on the worker's stack, stored once
    bool ex = false;
    int err = 0;
    for (size_t i = i0; i < i1 && !err; i++) {
      const kueue_tas_fits_req& r = reqs[i];
      if (r.leaf >= snapN || r.num_terms < 0 || r.term_begin < 0 || size_t(r.term_begin) + size_t(r.num_terms) > num_terms) {
        err = 1;
        break;
      }
      ex = ex || r.count < 0;
      for (int k = 0; k < r.num_terms; k++) {
        const kueue_tas_fits_term& tm = terms[r.term_begin + k];
        if (tm.col < 0 || tm.col >= snapR) {
          err = 2;
          break;
        }
        ex = ex || tm.value < 0;
        if (tm.col < KUEUE_TAS_MAX_COLS) tot[tm.col] += __int128(tm.value) * r.count;
      }
      if (pods_col >= 0) tot[pods_col] += r.count;
    }
    AdmitPart& ap = parts[t];
    memcpy(ap.total, tot, sizeof tot);
    ap.exact = ex;
    ap.err = err;
  });
  bool exact = false;
  __int128 total[KUEUE_TAS_MAX_COLS] = {};  // per column: the most usage this call can add
  for (size_t t = 0; t < nparts && n > 0; t++) {
    if (parts[t].err == 1) return fail(c, KUEUE_TAS_EINVAL, "admit record out of range");
    if (parts[t].err == 2) return fail(c, KUEUE_TAS_EINVAL, "admit term column out of range");
  }
  for (size_t t = 0; t < nparts && n > 0; t++) {
    exact = exact || parts[t].exact;
    for (int k = 0; k < KUEUE_TAS_MAX_COLS; k++) total[k] += parts[t].total[k];
  }
  for (int k = 0; k < KUEUE_TAS_MAX_COLS; k++) exact = exact || total[k] >= (__int128(1) << 61);
  HIPCHK(c, hipSetDevice(c->device));
  // one pinned upload: records, terms, workload offsets, record -> workload,
  // phase-1 flags (1 = fit) and the exact flag
  const AdmitLayout L = admit_layout(n, num_terms, n_wl, size_t(c->snap.N));
  HIPCHK(c, c->d_fits.ensure(L.end));
  HIPCHK(c, c->h_stage.ensure(L.up_bytes));
  uint8_t* h = c->h_stage.p;
  if (num_terms) memcpy(h + L.o_terms, terms, num_terms * sizeof(kueue_tas_fits_term));
  memcpy(h + L.o_off, wl_off, (n_wl + 1) * 8);
  int32_t* rec_wl = reinterpret_cast<int32_t*>(h + L.o_recwl);
  pool.run_static(n_wl, [&](size_t w0, size_t w1) {  // the records and their workload, per workload range
    if (w1 > w0 && wl_off[w1] > wl_off[w0])
      memcpy(h + size_t(wl_off[w0]) * sizeof(kueue_tas_fits_req), reqs + wl_off[w0],
             size_t(wl_off[w1] - wl_off[w0]) * sizeof(kueue_tas_fits_req));
    for (size_t w = w0; w < w1; w++)
      for (int64_t i = wl_off[w]; i < wl_off[w + 1]; i++) rec_wl[i] = int32_t(w);
  });
  int32_t* fit0 = reinterpret_cast<int32_t*>(h + L.o_fit0);
  for (size_t w = 0; w < n_wl; w++) fit0[w] = 1;
  *reinterpret_cast<int32_t*>(h + L.o_exact) = exact ? 1 : 0;
  for (int k = 0; k < KUEUE_TAS_MAX_COLS; k++)
    reinterpret_cast<int64_t*>(h + L.o_total)[k] = exact ? 0 : int64_t(total[k]);
  uint8_t* d = c->d_fits.p;
  HIPCHK(c, hipMemcpyAsync(d, h, L.up_bytes, hipMemcpyHostToDevice, c->stream));
  const int rc = admit_run(c, L, d, reinterpret_cast<const kueue_tas_fits_term*>(d + L.o_terms), n, n_wl, pods_col, exact);
  if (rc) return rc;
  HIPCHK(c, c->h_admit.reserve(n_wl + 3));
  HIPCHK(c, hipMemcpyAsync(c->h_admit.p, d + L.o_out, (n_wl + 3) * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  memcpy(admitted, c->h_admit.p, n_wl * 4);
  c->admit_stats[0] = c->admit_window ? c->h_admit.p[n_wl] : -1;
  c->admit_stats[1] = c->admit_window ? c->h_admit.p[n_wl + 1] : -1;
  c->admit_stats[2] = int64_t(n_wl);
  return KUEUE_TAS_OK;
}

int kueue_tas_copy_to_host(kueue_tas_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c || (bytes && (!dst || !src))) return KUEUE_TAS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (bytes) HIPCHK(c, hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return KUEUE_TAS_OK;
}

int kueue_tas_admit_table(kueue_tas_ctx* c, const int32_t* ps_base, int32_t num_workloads, const int32_t* ps_terms,
                          const kueue_tas_fits_term* terms, size_t num_terms) {
  if (!c || num_workloads < 0 || !ps_base || (num_terms && !terms)) return KUEUE_TAS_EINVAL;
  const int32_t P = ps_base[num_workloads];
  if (P < 0 || (P && !ps_terms)) return fail(c, KUEUE_TAS_EINVAL, "admit table: podsets");
  for (int32_t w = 0; w < num_workloads; w++)
    if (ps_base[w + 1] < ps_base[w] || ps_base[0] != 0) return fail(c, KUEUE_TAS_EINVAL, "admit table: podset offsets");
  for (int32_t p = 0; p < P; p++)
    if (ps_terms[2 * p] < 0 || ps_terms[2 * p + 1] < 0 || size_t(ps_terms[2 * p]) + size_t(ps_terms[2 * p + 1]) > num_terms)
      return fail(c, KUEUE_TAS_EINVAL, "admit table: term range");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, c->d_adm_ps.ensure(size_t(num_workloads) + 1 + 2 * size_t(P)));
  HIPCHK(c, c->d_adm_terms.ensure(std::max<size_t>(num_terms, 1)));
  HIPCHK(c, hipMemcpy(c->d_adm_ps.p, ps_base, (size_t(num_workloads) + 1) * 4, hipMemcpyHostToDevice));
  if (P) HIPCHK(c, hipMemcpy(c->d_adm_ps.p + num_workloads + 1, ps_terms, 2 * size_t(P) * 4, hipMemcpyHostToDevice));
  if (num_terms)
    HIPCHK(c, hipMemcpy(c->d_adm_terms.p, terms, num_terms * sizeof(kueue_tas_fits_term), hipMemcpyHostToDevice));
  c->adm_W = num_workloads;
  return KUEUE_TAS_OK;
}

int kueue_tas_admit_block(kueue_tas_ctx* c, const int32_t* block, size_t row_words, const int64_t* lens,
                          int32_t world, int32_t pods_col, int32_t* ids, int32_t* admitted, size_t cap,
                          size_t* n_workloads, const kueue_tas_delta** deltas, size_t* n_deltas) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (!block || !lens || !ids || !admitted || !n_workloads || !deltas || !n_deltas || world < 1)
    return fail(c, KUEUE_TAS_EINVAL, "null argument");
  if (world > kAdmitMaxRows) return fail(c, KUEUE_TAS_ELAYOUT, "admit block: more rows than supported");
  if (c->adm_W < 0) return fail(c, KUEUE_TAS_EINVAL, "admit block: no admission table (kueue_tas_admit_table)");
  if (pods_col < -1 || pods_col >= c->snap.R) return fail(c, KUEUE_TAS_EINVAL, "pods column out of range");
  AdmitRows rows{};
  rows.row_words = int64_t(row_words);
  rows.world = world;
  size_t Q = 0;
  int32_t maxq = 0;
  for (int r = 0; r < world; r++) {
    if (lens[r] < 0 || lens[r] % 4 || size_t(lens[r]) + 1 > row_words) return fail(c, KUEUE_TAS_EINVAL, "admit block: row length");
    rows.nq[r] = int32_t(lens[r] / 4);
    maxq = std::max(maxq, rows.nq[r]);
    Q += size_t(rows.nq[r]);
  }
  const int W = c->adm_W;
  HIPCHK(c, hipSetDevice(c->device));
  {  // device memory only: kernels must not read a pageable host array
    hipPointerAttribute_t pa{};
    if (hipPointerGetAttributes(&pa, block) != hipSuccess || pa.type != hipMemoryTypeDevice) {
      (void)hipGetLastError();
      return fail(c, KUEUE_TAS_EHOSTMEM, "admit block: not device memory");
    }
  }
  // the layout of the host path with the bounds (records <= quads, workloads <= W)
  const AdmitLayout L = admit_layout(std::max<size_t>(Q, 1), 0, size_t(W), size_t(c->snap.N));
  // per id: flag, run position, quad count; hdr: workloads, records, deltas; errors; exact; totals (lo, hi)
  const size_t o_flag = L.end, o_pos = o_flag + admit_al(size_t(W) * 4), o_nd = o_pos + admit_al(size_t(W) * 8),
               o_ids = o_nd + admit_al(size_t(W) * 4), o_hdr = o_ids + admit_al(size_t(W) * 4),
               o_tot = o_hdr + 256, o_blk = o_tot + admit_al(KUEUE_TAS_MAX_COLS * 16),
               nblk = (std::max<size_t>(Q, 1) + 255) / 256, o_dl = o_blk + admit_al(nblk * 4);
  HIPCHK(c, c->d_fits.ensure(o_dl + 16));
  uint8_t* d = c->d_fits.p;
  int32_t* hdr = reinterpret_cast<int32_t*>(d + o_hdr);  // [0] workloads [1] records [2] deltas [3] errors [4] negative
  HIPCHK(c, hipMemsetAsync(d + o_flag, 0, size_t(W) * 4, c->stream));
  HIPCHK(c, hipMemsetAsync(d + o_hdr, 0, 256 + admit_al(KUEUE_TAS_MAX_COLS * 16), c->stream));
  const double t0 = wall_ms();
  if (maxq > 0) {
    hipLaunchKernelGGL(admit_block_headers_kernel, dim3(unsigned((maxq + 255) / 256), unsigned(world)), dim3(256), 0,
                       c->stream, block, rows, W, reinterpret_cast<int32_t*>(d + o_flag),
                       reinterpret_cast<int64_t*>(d + o_pos), reinterpret_cast<int32_t*>(d + o_nd), hdr + 3);
    HIPCHK(c, hipGetLastError());
  }
  hipLaunchKernelGGL(admit_block_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, W,
                     reinterpret_cast<const int32_t*>(d + o_flag), reinterpret_cast<const int32_t*>(d + o_nd),
                     reinterpret_cast<int32_t*>(d + o_ids), reinterpret_cast<int64_t*>(d + L.o_off),
                     reinterpret_cast<int32_t*>(d + L.o_fit0), hdr);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, c->h_admit.reserve(size_t(W) + 3 + 64 + KUEUE_TAS_MAX_COLS * 4));
  int32_t* hh = c->h_admit.p;
  HIPCHK(c, hipMemcpyAsync(hh, hdr, 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int32_t n_wl = hh[0], n = hh[1];
  if (hh[3] & (ABE_DUP | ABE_LAYOUT | ABE_ID)) return fail(c, KUEUE_TAS_ELAYOUT, "admit block: not the assignments layout");
  *n_workloads = size_t(n_wl);
  if (cap < size_t(n_wl)) return KUEUE_TAS_EOVERFLOW;
  const size_t nwl = size_t(n_wl), nr = size_t(n);
  if (nwl) {
    hipLaunchKernelGGL(admit_block_records_kernel, dim3(unsigned((nwl + 3) / 4)), dim3(256), 0, c->stream, block,
                       c->snap.N, W, reinterpret_cast<const int32_t*>(d + o_ids), reinterpret_cast<const int64_t*>(d + L.o_off),
                       reinterpret_cast<const int32_t*>(d + o_flag), reinterpret_cast<const int64_t*>(d + o_pos),
                       reinterpret_cast<const int32_t*>(d + o_nd), c->d_adm_ps.p, c->d_adm_ps.p + W + 1,
                       c->d_adm_terms.p, n_wl, pods_col, reinterpret_cast<kueue_tas_fits_req*>(d),
                       reinterpret_cast<int32_t*>(d + L.o_recwl), reinterpret_cast<unsigned long long*>(d + o_tot),
                       hdr + 4, hdr + 3);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipMemcpyAsync(hh, hdr, 32, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(hh + 8, d + o_tot, KUEUE_TAS_MAX_COLS * 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int32_t errs = hh[3];
  if (errs & ABE_LAYOUT) return fail(c, KUEUE_TAS_ELAYOUT, "admit block: not the assignments layout");
  if (errs & ABE_RANGE) return fail(c, KUEUE_TAS_EINVAL, "admit: record out of range");
  if (errs & ABE_COL) return fail(c, KUEUE_TAS_EINVAL, "admit: request resource without a column");
  bool exact = hh[4] != 0;
  const uint64_t* tot = reinterpret_cast<const uint64_t*>(hh + 8);
  int64_t tot64[KUEUE_TAS_MAX_COLS];
  for (int k = 0; k < KUEUE_TAS_MAX_COLS; k++) {
    exact = exact || tot[2 * k + 1] != 0 || tot[2 * k] >= (uint64_t(1) << 61);
    tot64[k] = int64_t(tot[2 * k]);
  }
  // the exact flag and the totals, as the host path uploads them
  HIPCHK(c, c->h_stage.ensure(8 + KUEUE_TAS_MAX_COLS * 8));
  int32_t* hx = reinterpret_cast<int32_t*>(c->h_stage.p);
  hx[0] = exact ? 1 : 0;
  HIPCHK(c, hipMemcpyAsync(d + L.o_exact, hx, 4, hipMemcpyHostToDevice, c->stream));
  int64_t* ht = reinterpret_cast<int64_t*>(c->h_stage.p + 8);
  for (int k = 0; k < KUEUE_TAS_MAX_COLS; k++) ht[k] = exact ? 0 : tot64[k];
  HIPCHK(c, hipMemcpyAsync(d + L.o_total, ht, KUEUE_TAS_MAX_COLS * 8, hipMemcpyHostToDevice, c->stream));
  const int rc = admit_run(c, L, d, c->d_adm_terms.p, nr, nwl, pods_col, exact);
  if (rc) return rc;
  // the admitted workloads' deltas on the device, in the host path's order
  const int32_t* adm_d = reinterpret_cast<const int32_t*>(d + L.o_out);
  const size_t nb = (std::max<size_t>(nr, 1) + 255) / 256;
  int32_t* blk = reinterpret_cast<int32_t*>(d + o_blk);
  if (nr) {
    hipLaunchKernelGGL(admit_delta_blocks_kernel, dim3(unsigned(nb)), dim3(256), 0, c->stream,
                       reinterpret_cast<const kueue_tas_fits_req*>(d), reinterpret_cast<const int32_t*>(d + L.o_recwl),
                       adm_d, n, pods_col, blk);
    hipLaunchKernelGGL(admit_delta_offsets_kernel, dim3(1), dim3(1024), 0, c->stream, blk, int(nb), hdr);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipMemcpyAsync(hh, d + L.o_out, (nwl + 3) * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(hh + nwl + 3, hdr, 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(ids, d + o_ids, nwl * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  memcpy(admitted, hh, nwl * 4);
  c->admit_stats[0] = c->admit_window ? hh[nwl] : -1;
  c->admit_stats[1] = c->admit_window ? hh[nwl + 1] : -1;
  c->admit_stats[2] = int64_t(nwl);
  const size_t ndl = nr ? size_t(hh[nwl + 3 + 2]) : 0;
  HIPCHK(c, c->d_adm_deltas.ensure(std::max<size_t>(ndl, 1)));
  HIPCHK(c, c->h_adm_deltas.reserve(std::max<size_t>(ndl, 1)));
  if (ndl) {
    hipLaunchKernelGGL(admit_delta_write_kernel, dim3(unsigned(nb)), dim3(256), 0, c->stream,
                       reinterpret_cast<const kueue_tas_fits_req*>(d), c->d_adm_terms.p,
                       reinterpret_cast<const int32_t*>(d + L.o_recwl), adm_d, n, pods_col, blk, c->d_adm_deltas.p);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->h_adm_deltas.p, c->d_adm_deltas.p, ndl * sizeof(kueue_tas_delta),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  *deltas = c->h_adm_deltas.p;
  *n_deltas = ndl;
  c->admit_block_ms = wall_ms() - t0;
  return KUEUE_TAS_OK;
}

// The admission pass over the records in c->d_fits (layout L): phase 1
// (admit_fit0_kernel), the order-free candidates in parallel unless exact,
// then the in-order pass (admit_window_kernel in phases with grid sweeps, or
// the one-wave chain).  Verdicts at L.o_out.
static int admit_run(kueue_tas_ctx* c, const AdmitLayout& L, uint8_t* d, const kueue_tas_fits_term* d_terms, size_t n,
                     size_t n_wl, int32_t pods_col, bool exact) {
  const size_t nwords = (size_t(c->snap.N) + 31) / 32;
  // the dynamic bitmaps share the workgroup's 64 KB of LDS with the kernel's
  // static arrays (the window kernel's fit / conflict flags and sweep scan)
  static const size_t static_lds[2] = {
      [] {
        hipFuncAttributes a{};
        return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(admit_kernel)) == hipSuccess ? size_t(a.sharedSizeBytes)
                                                                                                  : size_t(16 * 1024);
      }(),
      [] {
        hipFuncAttributes a{};
        return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(admit_window_kernel)) == hipSuccess
                   ? size_t(a.sharedSizeBytes)
                   : size_t(16 * 1024);
      }()};
  const size_t lds_budget = 64 * 1024 - static_lds[c->admit_window ? 1 : 0];
  const bool lds_bits = nwords * 4 <= lds_budget;
  // the windowed kernel's round bitmap beside the touched one: admission chains within a window
  const bool lds_chain = c->admit_window && 2 * nwords * 4 <= lds_budget;
  HIPCHK(c, hipMemsetAsync(d + L.o_bits, 0, nwords * 4, c->stream));
  HIPCHK(c, hipMemsetAsync(d + L.o_state, 0, 256, c->stream));
  // order-free candidates decided in parallel (admit_minc / dep / indep), unless exact
  const bool indep = c->admit_window && !exact && n > 0;
  if (indep) {
    HIPCHK(c, hipMemsetAsync(d + L.o_minc, 0x7f, size_t(c->snap.N) * 4, c->stream));
    HIPCHK(c, hipMemsetAsync(d + L.o_dep, 0, n_wl * 4, c->stream));
  }
  const auto* d_reqs = reinterpret_cast<const kueue_tas_fits_req*>(d);
  if (n) {
    hipLaunchKernelGGL(admit_fit0_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, c->stream, c->snap,
                       c->d_usage.p, c->d_usage_present.p, d_reqs, d_terms,
                       reinterpret_cast<const int32_t*>(d + L.o_recwl), int(n), reinterpret_cast<const int64_t*>(d + L.o_total),
                       reinterpret_cast<int32_t*>(d + L.o_fit0), reinterpret_cast<AdmitRec*>(d + L.o_recs),
                       reinterpret_cast<int32_t*>(d + L.o_exact));
    HIPCHK(c, hipGetLastError());
  }
  if (c->admit_window) {  // independent candidates in parallel, the rest windowed (one 1024-thread workgroup)
    const auto* recwl = reinterpret_cast<const int32_t*>(d + L.o_recwl);
    const auto* fit0d = reinterpret_cast<const int32_t*>(d + L.o_fit0);
    auto* depd = reinterpret_cast<int32_t*>(d + L.o_dep);
    if (indep) {
      const dim3 g(unsigned((n + 255) / 256));
      hipLaunchKernelGGL(admit_minc_kernel, g, dim3(256), 0, c->stream, d_reqs, recwl, int(n), fit0d, c->snap.N,
                         reinterpret_cast<int32_t*>(d + L.o_minc));
      hipLaunchKernelGGL(admit_dep_kernel, g, dim3(256), 0, c->stream, d_reqs, recwl, int(n), fit0d, c->snap.N,
                         reinterpret_cast<const int32_t*>(d + L.o_minc), depd);
      hipLaunchKernelGGL(admit_indep_kernel, g, dim3(256), 0, c->stream, c->snap, c->d_usage.p, c->d_usage_present.p,
                         d_reqs, d_terms, recwl, int(n), fit0d, depd, pods_col, reinterpret_cast<uint32_t*>(d + L.o_bits));
      HIPCHK(c, hipGetLastError());
    }
    hipLaunchKernelGGL(admit_todo_kernel, dim3(1), dim3(1024), 0, c->stream, int(n_wl), fit0d, depd, indep ? 0 : 1,
                       reinterpret_cast<int32_t*>(d + L.o_out), reinterpret_cast<int32_t*>(d + L.o_todo),
                       reinterpret_cast<const int64_t*>(d + L.o_off), reinterpret_cast<int64_t*>(d + L.o_todor));
    HIPCHK(c, hipGetLastError());
    // the window kernel in phases: each stops at a rejection sweep, which the
    // grid runs (a wave per remaining candidate) before the next phase
    // resumes; the last phase sweeps inside its workgroup.  A finished pass
    // leaves the later launches nothing to do.
    int32_t* st = reinterpret_cast<int32_t*>(d + L.o_state);
    int32_t* todo = reinterpret_cast<int32_t*>(d + L.o_todo);
    int64_t* todor = reinterpret_cast<int64_t*>(d + L.o_todor);
    const int phases = c->admit_grid_sweeps;
    for (int ph = 0; ph < phases; ph++) {
      if (ph > 0) {
        hipLaunchKernelGGL(admit_sweep_kernel, dim3(1024), dim3(256), 0, c->stream, c->snap, c->d_usage.p,
                           c->d_usage_present.p, d_reqs, d_terms, reinterpret_cast<const AdmitRec*>(d + L.o_recs), fit0d,
                           reinterpret_cast<const uint32_t*>(d + L.o_bits), reinterpret_cast<int32_t*>(d + L.o_out), todo,
                           todor, st);
        hipLaunchKernelGGL(admit_compact_kernel, dim3(1), dim3(1024), 0, c->stream, todo, todor, st);
      }
      hipLaunchKernelGGL(admit_window_kernel, dim3(1), dim3(64 * kAdmitWindow),
                         lds_chain ? 2 * nwords * 4 : lds_bits ? nwords * 4 : 0, c->stream, c->snap, c->d_usage.p,
                         c->d_usage_present.p, d_reqs, d_terms, reinterpret_cast<const AdmitRec*>(d + L.o_recs),
                         reinterpret_cast<const int64_t*>(d + L.o_off), int(n_wl), pods_col,
                         reinterpret_cast<const int32_t*>(d + L.o_fit0), reinterpret_cast<const int32_t*>(d + L.o_exact),
                         reinterpret_cast<uint32_t*>(d + L.o_bits), lds_chain ? 2 : lds_bits ? 1 : 0,
                         reinterpret_cast<int32_t*>(d + L.o_out), todo, todor, st, ph + 1 < phases ? 1 : 0);
      HIPCHK(c, hipGetLastError());
    }
  } else {  // one wave down the chain
    hipLaunchKernelGGL(admit_kernel, dim3(1), dim3(64), lds_bits ? nwords * 4 : 0, c->stream, c->snap, c->d_usage.p,
                       c->d_usage_present.p, d_reqs, d_terms, reinterpret_cast<const AdmitRec*>(d + L.o_recs),
                       reinterpret_cast<const int64_t*>(d + L.o_off), int(n_wl),
                       pods_col, reinterpret_cast<const int32_t*>(d + L.o_fit0), reinterpret_cast<const int32_t*>(d + L.o_exact),
                       reinterpret_cast<uint32_t*>(d + L.o_bits), lds_bits ? 1 : 0, reinterpret_cast<int32_t*>(d + L.o_out));
  }
  HIPCHK(c, hipGetLastError());
  return KUEUE_TAS_OK;
}

int kueue_tas_last_admit_stats(kueue_tas_ctx* c, int64_t* out3) {
  if (!c || !out3) return KUEUE_TAS_EINVAL;
  memcpy(out3, c->admit_stats, sizeof c->admit_stats);
  return KUEUE_TAS_OK;
}


// The longest candidate list a BestFit-side walk of `ev` can build (its
// select lists' capacity): every domain of a level at or above its requested
// level (findLevelWithFitDomains sorts whole levels, tas_flavor_snapshot.go:
// 1098-1163), and below it the children of the domains chosen one level up,
// at most one chosen domain per pod (updateCountsToMinimum takes a domain
// only while pods remain, :1236-1321); twice that, as the unbounded capacity
// is twice the widest level.  Unconstrained, multi-layer and replacement
// walks keep the unbounded lists.  An overflow still re-runs the chunk
// unbounded (eval_chunk returns 2), so the bound costs memory, never results.
static int64_t scratch_bound(const kueue_tas_ctx* c, const DevSnap& s, const DevEval& ev, int64_t full) {
  if (ev.flags & (KUEUE_TAS_F_UNCONSTRAINED | KUEUE_TAS_F_MULTILAYER | KUEUE_TAS_F_DOMAIN)) return full;
  const int r = ev.requested_level;
  if (r < 0 || r >= s.L || c->level_maxfan.size() < size_t(s.L)) return full;
  const int64_t pods = int64_t(std::max(ev.count, 0)) + ((ev.flags & KUEUE_TAS_F_LEADER) ? 1 : 0);
  int64_t top = 0, below = pods;  // whole levels at or above r (find_level's lists are unchecked there)
  for (int l = 0; l < s.L; l++) {
    if (l <= r) top = std::max<int64_t>(top, s.level_size[l]);
    else
      below = std::max<int64_t>(below, std::min<int64_t>(s.level_size[l], std::min<int64_t>(s.level_size[l - 1], pods) *
                                                                               c->level_maxfan[size_t(l - 1)]));
  }
  int64_t lc = std::min(full, 2 * std::max(top, below) + 64);
  if (c->lcap_test_cap) lc = std::min(lc, std::max(c->lcap_test_cap, std::min(full, 2 * top + 64)));  // (descent lists only)
  return lc;
}


static int eval_chunk(kueue_tas_ctx* c, const kueue_tas_eval_req* const* reqs, size_t n, const int32_t* taint_table,
                      size_t taint_table_len, int32_t num_taints, const kueue_tas_assumed* assumed, size_t num_assumed,
                      const kueue_tas_affinity_req* aff, size_t num_aff, const int32_t* aff_vals, size_t num_aff_vals,
                      kueue_tas_eval_out* out, int64_t* offsets, int32_t* taint_counts, int32_t* res_counts,
                      float* ms, float* stage_ms) {
  const int32_t entry_cap = c->entry_cap;
  const DevSnap& s = c->snap;
  double tm = wall_ms();
  auto lap = [&](int k) {
    const double t = wall_ms();
    c->host_ms[k] += t - tm;
    tm = t;
  };
  auto trace = [&](int k) { c->trace[k] = wall_ms(); };
  trace(0);
  // ---- per-request host work over the worker pool: validation and term
  // counts (pass A), then the device records, division magic and the class
  // hashes (pass B); errors are reported for the lowest request index ----
  ktas_pool::HostPool& pool = ktas_pool::HostPool::get();
  // static parts: the same thread handles the same requests in both passes
  // (and the host layer's compile and decode of the same workloads before
  // and after), so their records stay in that core's cache
  const size_t nparts = pool.parts();
  const size_t nchunk = nparts;
  auto part_of = [&](size_t i0) -> size_t {  // the static part starting at request i0
    size_t t = 0;
    while (t + 1 < nparts && ktas_pool::HostPool::part_begin(n, t + 1, nparts) <= i0) t++;
    return t;
  };
  std::vector<int64_t>& toff = c->req_term_off;  // first term slot of each request
  toff.assign(n + 1, 0);
  std::vector<int32_t>& chunk_maxt = c->req_chunk_maxt;
  chunk_maxt.assign(std::max<size_t>(nchunk, 1), 1);
  std::vector<std::pair<size_t, std::string>>& errs = c->req_errs;  // per chunk: (first bad request, message)
  errs.assign(std::max<size_t>(nchunk, 1), {SIZE_MAX, std::string()});
  auto validate = [&](size_t i, std::string* msg) -> bool {
    const auto& r = *reqs[i];
    if (r.num_req < 0 || r.num_req > KUEUE_TAS_MAX_COLS || r.num_leader_req < 0 || r.num_leader_req > KUEUE_TAS_MAX_COLS)
      return *msg = "num_req", false;
    if (r.slice_size == 0) return *msg = "slice_size == 0 (integer divide by zero)", false;
    if (r.requested_level < 0 || r.requested_level >= s.L || r.slice_level < 0 || r.slice_level >= s.L)
      return *msg = "level out of range", false;
    if (r.num_selectors < 0 || r.num_selectors > KUEUE_TAS_MAX_SELECTORS) return *msg = "num_selectors", false;
    if (r.num_selectors > 0 && s.K == 0) return *msg = "selectors without label columns", false;
    // host-side shape check of every requirement the fill will read
    auto check_reqs = [&](int32_t rb, int32_t re, bool terms, const char* what) -> bool {
      if (rb < 0 || re < rb || size_t(re) > num_aff || (re > rb && (!aff || !aff_vals)))
        return *msg = std::string(what) + " range", false;
      for (int32_t k = rb; k < re; k++) {
        const kueue_tas_affinity_req& q = aff[k];
        if (q.col < KUEUE_TAS_AFFINITY_LEAF || q.col >= s.K || q.begin < 0 || q.len < 0 ||
            size_t(q.begin) + size_t(q.len) > num_aff_vals || (terms && k > rb && q.term < aff[k - 1].term))
          return *msg = std::string(what) + " requirement", false;
        for (int32_t j = 1; j < q.len; j++)
          if (aff_vals[q.begin + j] <= aff_vals[q.begin + j - 1])
            return *msg = std::string(what) + " values not sorted", false;
      }
      return true;
    };
    if ((r.flags & KUEUE_TAS_F_AFFINITY) && !check_reqs(r.affinity_begin, r.affinity_end, true, "affinity")) return false;
    if (r.flags & KUEUE_TAS_F_SELECTOR_EXT) {
      if (r.num_selectors != KUEUE_TAS_MAX_SELECTORS)
        return *msg = "KUEUE_TAS_F_SELECTOR_EXT needs the inline selector pairs filled", false;
      if (!check_reqs(r.selector_begin, r.selector_end, false, "nodeSelector")) return false;
    }
    if (r.assumed_begin < 0 || r.assumed_end < r.assumed_begin || size_t(r.assumed_end) > num_assumed ||
        (r.assumed_end > r.assumed_begin && !assumed))
      return *msg = "assumed range", false;
    for (int32_t a = r.assumed_begin; a < r.assumed_end; a++) {  // sorted by leaf (the fill's binary search)
      const kueue_tas_assumed& x = assumed[a];
      if (x.leaf < 0 || x.leaf >= s.N || x.col < 0 || x.col >= s.R || x.col >= KUEUE_TAS_MAX_COLS ||
          (a > r.assumed_begin && x.leaf < assumed[a - 1].leaf))
        return *msg = "assumed record out of range or not sorted by leaf", false;
    }
    if ((r.flags & KUEUE_TAS_F_DOMAIN) &&
        (r.domain_begin < 0 || r.domain_end < r.domain_begin || r.domain_end > s.N))
      return *msg = "required domain leaf range", false;
    return true;
  };
  pool.run_static(n, [&](size_t i0, size_t i1) {
    const size_t ch = part_of(i0);
    std::string msg;
    int32_t mt = 1;  // this part's widest request, stored once (the parts' slots share a cache line)
    for (size_t i = i0; i < i1; i++) {
      const auto& r = *reqs[i];
      if (errs[ch].first == SIZE_MAX && !validate(i, &msg)) errs[ch] = {i, msg};
      toff[i + 1] = int64_t(std::max(r.num_req, 0)) + int64_t(std::max(r.num_leader_req, 0));
      mt = std::max(mt, std::max(r.num_req, r.num_leader_req));
    }
    chunk_maxt[ch] = mt;
  });
  for (auto& e : errs)
    if (e.first != SIZE_MAX) return fail(c, KUEUE_TAS_EINVAL, e.second);
  c->host_ms[6] += wall_ms() - tm;
  trace(1);
  for (size_t i = 0; i < n; i++) toff[i + 1] += toff[i];
  const size_t nterms = size_t(toff[n]);
  int maxt = 1;
  for (int32_t m : chunk_maxt) maxt = std::max(maxt, m);
  size_t stage_bytes = 0;
  auto seg = [&](size_t bytes) {
    const size_t o = stage_bytes;
    stage_bytes += (bytes + 255) / 256 * 256;
    return o;
  };
  const size_t o_evals = seg(n * sizeof(DevEval)), o_terms = seg(nterms * sizeof(DevTerm));
  const size_t o_taint = seg(taint_table_len * 4), o_assumed = seg(num_assumed * sizeof(kueue_tas_assumed));
  const size_t o_aff = seg(num_aff * sizeof(kueue_tas_affinity_req)), o_affv = seg(num_aff_vals * 4);
  const size_t o_fill = seg(n * 4), o_fchunks = seg(n * 8), o_pairs = seg(n * 8), o_rep = seg(n * 4);
  const size_t o_frun = seg(n * 4);
  const size_t o_slot = seg(n * 4), o_lrep = seg(n * 4), o_fast = seg(n * 4), o_leafsel = seg(n * 4);
  const size_t o_pidx = seg(n * 4), o_bf = seg(n * 4);
  const size_t o_moff = seg((n + 1) * 4), o_mem = seg(n * 4);  // class members in fill order (CSR)
  // rollup_top_kernel's level maxima (INT32_MIN) and per-class arrival counters (0)
  const size_t o_top = seg(n * (kMaxLevels + 1) * 4);
  const size_t o_sel = seg(n * sizeof(SelSlot));  // BestFit-side select slots' buffers
  // last: the per-position fill records, uploaded up to the batch's nfill
  const size_t o_fpos = seg(n * sizeof(FillPos));
  HIPCHK(c, c->h_stage.ensure(stage_bytes));
  HIPCHK(c, c->d_stage.ensure(stage_bytes));
  uint8_t* hs = c->h_stage.p;
  DevEval* hev = reinterpret_cast<DevEval*>(hs + o_evals);
  DevTerm* hterms = reinterpret_cast<DevTerm*>(hs + o_terms);
  // ---- class hashes (phase-1 classes below) ----
  const int32_t P = c->num_profiles;
  auto taint_row = [&](const DevEval& e) -> const int32_t* {
    return (taint_table && size_t(e.taint_table) + size_t(P) <= taint_table_len) ? taint_table + e.taint_table
                                                                                  : nullptr;
  };
  auto sig_hash = [&](const DevEval& e) {
    uint64_t h = 1469598103934665603ull;
    auto add = [&](uint64_t v) {
      h ^= v;
      h *= 1099511628211ull;
      h ^= h >> 31;
    };
    add(e.flags & (KUEUE_TAS_F_LEADER | KUEUE_TAS_F_SIMULATE_EMPTY));
    add(uint64_t(uint32_t(e.nreq)) | (uint64_t(uint32_t(e.nlead)) << 32));
    for (int k = 0; k < e.nreq + e.nlead; k++) {
      const DevTerm& t = hterms[k < e.nreq ? e.term_begin + k : e.lead_begin + (k - e.nreq)];
      add(uint64_t(uint32_t(t.col)));
      add(uint64_t(t.val));
    }
    for (int a = e.assumed_begin; a < e.assumed_end; a++) {
      add(uint64_t(uint32_t(assumed[a].leaf)) | (uint64_t(uint32_t(assumed[a].col)) << 32));
      add(uint64_t(assumed[a].value));
    }
    return h;
  };
  auto mask_hash = [&](const DevEval& e) {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    auto add = [&](uint64_t v) {
      h ^= v;
      h *= 1099511628211ull;
      h ^= h >> 29;
    };
    add(uint64_t(uint32_t(e.slice_size)) | (uint64_t(uint32_t(e.slice_level)) << 32));
    for (int l = 0; l < s.L; l++) add(uint64_t(uint32_t(e.ssal[l])));  // no kernel reads a level >= L
    add(uint64_t(uint32_t(e.nsel)));
    add(uint64_t(uint32_t(e.dom_begin)) | (uint64_t(uint32_t(e.dom_end)) << 32));
    for (int k = 0; k < e.nsel; k++) add(uint64_t(uint32_t(e.sel_col[k])) | (uint64_t(uint32_t(e.sel_val[k])) << 32));
    if (const int32_t* row = taint_row(e))
      for (int p = 0; p < P; p++) add(uint64_t(uint32_t(row[p])));
    auto add_reqs = [&](int32_t rb, int32_t re) {
      for (int k = rb; k < re; k++) {
        const kueue_tas_affinity_req& q = aff[k];
        add(uint64_t(uint32_t(q.term)) | (uint64_t(uint32_t(q.col)) << 32));
        add(uint64_t(uint32_t(q.negate)) | (uint64_t(uint32_t(q.len)) << 32));
        for (int j = 0; j < q.len; j++) add(uint64_t(uint32_t(aff_vals[q.begin + j])));
      }
    };
    if (e.flags & KUEUE_TAS_F_AFFINITY) {
      add(0xaff1u);
      add_reqs(e.aff_begin, e.aff_end);
    }
    if (e.sx_begin >= 0) {
      add(0x5e1eu);
      add_reqs(e.sx_begin, e.sx_end);
    }
    return h;
  };
  auto same_sig = [&](const DevEval& x, const DevEval& y) {
    if ((x.flags ^ y.flags) & (KUEUE_TAS_F_LEADER | KUEUE_TAS_F_SIMULATE_EMPTY)) return false;
    if (x.nreq != y.nreq || x.nlead != y.nlead) return false;
    for (int k = 0; k < x.nreq + x.nlead; k++) {
      const DevTerm& a = hterms[k < x.nreq ? x.term_begin + k : x.lead_begin + (k - x.nreq)];
      const DevTerm& b2 = hterms[k < y.nreq ? y.term_begin + k : y.lead_begin + (k - y.nreq)];
      if (a.col != b2.col || a.val != b2.val) return false;
    }
    if (x.assumed_end - x.assumed_begin != y.assumed_end - y.assumed_begin) return false;
    for (int a = 0; a < x.assumed_end - x.assumed_begin; a++) {
      const kueue_tas_assumed& p = assumed[x.assumed_begin + a];
      const kueue_tas_assumed& q = assumed[y.assumed_begin + a];
      if (p.leaf != q.leaf || p.col != q.col || p.value != q.value) return false;
    }
    return true;
  };
  // base signature: what the leaf's remaining capacity depends on (a fill chunk shares it)
  auto same_base = [&](const DevEval& x, const DevEval& y) {
    if ((x.flags ^ y.flags) & (KUEUE_TAS_F_LEADER | KUEUE_TAS_F_SIMULATE_EMPTY)) return false;
    if (x.assumed_end - x.assumed_begin != y.assumed_end - y.assumed_begin) return false;
    for (int a = 0; a < x.assumed_end - x.assumed_begin; a++) {
      const kueue_tas_assumed& p = assumed[x.assumed_begin + a];
      const kueue_tas_assumed& q = assumed[y.assumed_begin + a];
      if (p.leaf != q.leaf || p.col != q.col || p.value != q.value) return false;
    }
    return true;
  };
  auto same_mask = [&](const DevEval& x, const DevEval& y) {
    if (x.slice_size != y.slice_size || x.slice_level != y.slice_level || x.nsel != y.nsel) return false;
    if (x.dom_begin != y.dom_begin || x.dom_end != y.dom_end) return false;
    for (int l = 0; l < s.L; l++)
      if (x.ssal[l] != y.ssal[l]) return false;
    for (int k = 0; k < x.nsel; k++)
      if (x.sel_col[k] != y.sel_col[k] || x.sel_val[k] != y.sel_val[k]) return false;
    const int32_t *rx = taint_row(x), *ry = taint_row(y);
    if ((rx == nullptr) != (ry == nullptr)) return false;
    if (!(rx == nullptr || rx == ry || memcmp(rx, ry, size_t(P) * 4) == 0)) return false;
    auto same_reqs = [&](int32_t xb, int32_t xe, int32_t yb, int32_t ye) {
      if (xe - xb != ye - yb) return false;
      for (int k = 0; k < xe - xb; k++) {
        const kueue_tas_affinity_req& p = aff[xb + k];
        const kueue_tas_affinity_req& q = aff[yb + k];
        if (p.term != q.term || p.col != q.col || p.negate != q.negate || p.len != q.len) return false;
        if (p.begin != q.begin && memcmp(aff_vals + p.begin, aff_vals + q.begin, size_t(p.len) * 4) != 0) return false;
      }
      return true;
    };
    if ((x.sx_begin >= 0) != (y.sx_begin >= 0)) return false;
    if (x.sx_begin >= 0 && !same_reqs(x.sx_begin, x.sx_end, y.sx_begin, y.sx_end)) return false;
    const bool ax = (x.flags & KUEUE_TAS_F_AFFINITY) != 0, ay = (y.flags & KUEUE_TAS_F_AFFINITY) != 0;
    if (ax != ay) return false;
    if (!ax) return true;
    return same_reqs(x.aff_begin, x.aff_end, y.aff_begin, y.aff_end);
  };
  auto fast_lfc = [&](const DevEval& e) {
    return (e.flags & KUEUE_TAS_F_LFC) != 0 &&
           (e.flags & (KUEUE_TAS_F_LEADER | KUEUE_TAS_F_REQUIRED | KUEUE_TAS_F_MULTILAYER)) == 0 &&
           e.requested_level == s.L - 1 && e.slice_level == s.L - 1 && e.slice_size == 1 && e.count >= 0 && s.N > 0;
  };
  std::vector<uint64_t>& h_sig = c->req_sig_hash;   // signature hash per request
  std::vector<uint64_t>& h_cls = c->req_cls_hash;   // signature x mask hash per request
  h_sig.resize(n);
  h_cls.resize(n);
  std::vector<uint8_t>& req_fast = c->req_fast;     // fast-LFC eligible (fast_lfc)
  std::vector<uint8_t>& req_leaf = c->req_leaf;     // requested level == the leaf level
  std::vector<int32_t>& req_local_cls = c->req_local_cls;  // class within the request's static part
  req_fast.resize(n);
  req_leaf.resize(n);
  req_local_cls.resize(n);
  c->part_cls.resize(nparts);
  for (size_t t = 0; t < nparts; t++) {
    PartClasses& pc = c->part_cls[t];
    pc.head.reset(ktas_pool::HostPool::part_begin(n, t + 1, nparts) - ktas_pool::HostPool::part_begin(n, t, nparts));
    pc.rep.clear();
    pc.next.clear();
    pc.hcls.clear();
    pc.hsig.clear();
  }
  trace(2);
  // ---- compile requests to device form (magic numbers) ----
  const double t_b = wall_ms();
  if (c->magic_cache.size() < nparts) c->magic_cache.resize(nparts);
  pool.run_static(n, [&](size_t i0, size_t i1) {
    const size_t ch = part_of(i0);
    MagicCache& mc = c->magic_cache[ch];
    for (size_t i = i0; i < i1; i++) {
      const auto& r = *reqs[i];
      DevEval& e = hev[i];  // every field is assigned below (no memset of the record)
      e.req_mask = e.lead_mask = 0;
      e.flags = r.flags;
      e.count = r.count;
      e.slice_size = r.slice_size;
      e.requested_level = r.requested_level;
      e.slice_level = r.slice_level;
      e.nsel = r.num_selectors;
      e.taint_table = r.taint_table;
      e.assumed_begin = r.assumed_begin;
      e.assumed_end = r.assumed_end;
      e.aff_begin = r.affinity_begin;
      e.aff_end = r.affinity_end;
      e.dom_begin = (r.flags & KUEUE_TAS_F_DOMAIN) ? r.domain_begin : -1;
      e.dom_end = (r.flags & KUEUE_TAS_F_DOMAIN) ? r.domain_end : -1;
      const bool sx = (r.flags & KUEUE_TAS_F_SELECTOR_EXT) != 0 && r.selector_end > r.selector_begin;
      e.sx_begin = sx ? r.selector_begin : -1;
      e.sx_end = sx ? r.selector_end : -1;
      e.num_layers = std::min(r.num_layers, KUEUE_TAS_MAX_LAYERS);
      for (int k = 0; k < KUEUE_TAS_MAX_LAYERS; k++) {
        e.layer_level[k] = r.layer_level[k];
        e.layer_size[k] = r.layer_size[k] == 0 ? 1 : r.layer_size[k];
      }
      for (int l = 0; l < KUEUE_TAS_MAX_LEVELS; l++) e.ssal[l] = r.slice_size_at_level[l];
      for (int k = 0; k < KUEUE_TAS_MAX_SELECTORS; k++) {
        e.sel_col[k] = r.sel_col[k];
        e.sel_val[k] = r.sel_val[k];
      }
      int64_t tp = toff[i];
      auto add_terms = [&](const int32_t* cols, const int64_t* vals, int cnt, uint32_t* mask) -> int {
        int prev = -1;
        for (int k = 0; k < cnt; k++) {
          if (cols[k] < 0 || cols[k] >= s.R || cols[k] <= prev) return -1;
          prev = cols[k];
          DevTerm& t = hterms[tp++];
          t.col = cols[k];
          t.val = vals[k];
          t.neg = vals[k] < 0;
          uint64_t mag = vals[k] < 0 ? (0ull - uint64_t(vals[k])) : uint64_t(vals[k]);
          if (mag) {
            compute_magic(mag, &t, mc);
          } else {
            t.magic = 0;
            t.shift = t.add = t.pow2 = 0;
          }
          *mask |= 1u << cols[k];
        }
        return 0;
      };
      e.term_begin = int32_t(tp);
      e.nreq = r.num_req;
      if (add_terms(r.req_col, r.req_val, r.num_req, &e.req_mask)) {
        if (errs[ch].first == SIZE_MAX) errs[ch] = {i, "req columns"};
        continue;
      }
      e.lead_begin = int32_t(tp);
      e.nlead = (r.flags & KUEUE_TAS_F_LEADER) ? r.num_leader_req : 0;
      if (add_terms(r.leader_col, r.leader_val, e.nlead, &e.lead_mask)) {
        if (errs[ch].first == SIZE_MAX) errs[ch] = {i, "leader columns"};
        continue;
      }
      h_sig[i] = sig_hash(e);
      h_cls[i] = h_sig[i] ^ (mask_hash(e) * 0xff51afd7ed558ccdull);
      req_fast[i] = fast_lfc(e) ? 1 : 0;
      req_leaf[i] = e.requested_level == s.L - 1 ? 1 : 0;
      // this part's classes (first member in request order), exact compare on a hash hit
      PartClasses& pc = c->part_cls[ch];
      int32_t k = -1;
      int32_t* head = pc.head.find(h_cls[i]);
      for (int32_t q = *head; q >= 0; q = pc.next[size_t(q)]) {
        const DevEval& r = hev[pc.rep[size_t(q)]];
        if (same_sig(e, r) && same_mask(e, r)) {
          k = q;
          break;
        }
      }
      if (k < 0) {
        k = int32_t(pc.rep.size());
        pc.rep.push_back(int32_t(i));
        pc.next.push_back(*head);
        pc.hcls.push_back(h_cls[i]);
        pc.hsig.push_back(h_sig[i]);
        *head = k;
      }
      req_local_cls[i] = k;
    }
  });
  for (auto& e : errs)
    if (e.first != SIZE_MAX) return fail(c, KUEUE_TAS_EINVAL, e.second);
  c->host_ms[7] += wall_ms() - t_b;
  trace(3);
  if (taint_table_len) memcpy(hs + o_taint, taint_table, taint_table_len * 4);
  if (num_assumed) memcpy(hs + o_assumed, assumed, num_assumed * sizeof(kueue_tas_assumed));
  if (num_aff) memcpy(hs + o_aff, aff, num_aff * sizeof(kueue_tas_affinity_req));
  if (num_aff_vals) memcpy(hs + o_affv, aff_vals, num_aff_vals * 4);
  lap(0);
  trace(4);

  // Phase-1 classes: evals with identical phase-1 inputs (request terms,
  // masks, overlay, slice parameters) get identical counters; phase 1 runs
  // once per class (its representative).  Every member's select reads the
  // class counters and keeps its mutations in a private overlay; duplicates
  // only get the rep's exclusion stats.  A class's request signature (terms,
  // overlay, simulateEmpty, leader) decides which classes share a fill chunk.
  int32_t* h_fill = reinterpret_cast<int32_t*>(hs + o_fill);
  int32_t* h_fchunks = reinterpret_cast<int32_t*>(hs + o_fchunks);
  int32_t* h_pairs = reinterpret_cast<int32_t*>(hs + o_pairs);
  int32_t* h_rep = reinterpret_cast<int32_t*>(hs + o_rep);
  int32_t* h_slot = reinterpret_cast<int32_t*>(hs + o_slot);
  int32_t* h_lrep = reinterpret_cast<int32_t*>(hs + o_lrep);
  int32_t* h_fast = reinterpret_cast<int32_t*>(hs + o_fast);
  int32_t* h_leafsel = reinterpret_cast<int32_t*>(hs + o_leafsel);
  int32_t* h_pidx = reinterpret_cast<int32_t*>(hs + o_pidx);  // eval -> row of its leaf partials, -1
  int32_t* h_bf = reinterpret_cast<int32_t*>(hs + o_bf);      // evals selected on the main stream
  int nbf = 0;
  int nfill = 0, npairs = 0, nslots = 0, nfast = 0, nfchunks = 0, nleafsel = 0, nruns = 0, nsingle = 0;
  {
    // classes: open hash chains on the 64-bit (signature, mask) hash, exact compare on the rep
    std::vector<int32_t>& cls_rep = c->cls_rep;    // first member of each class
    std::vector<int32_t>& cls_sig = c->cls_sig;    // signature id of each class
    std::vector<int32_t>& cls_of = c->cls_of;      // class of each eval
    std::vector<int32_t>& sig_rep = c->sig_rep;    // first eval of each signature
    cls_rep.clear();
    cls_sig.clear();
    sig_rep.clear();
    cls_of.assign(n, -1);
    FlatMap& cls_head = c->cls_head;
    FlatMap& sig_head = c->sig_head;
    cls_head.reset(n);
    sig_head.reset(n);
    std::vector<int32_t>& cls_next = c->cls_next;  // chain of classes with the same hash
    std::vector<int32_t>& sig_next = c->sig_next;
    cls_next.clear();
    sig_next.clear();
    // the parts' classes merged in part order: a global class is numbered by
    // its first member, as a serial pass over the requests would number it
    std::vector<int32_t>& part_map = c->part_map;  // (part, local class) -> global class
    std::vector<size_t>& part_base = c->part_base;
    part_base.assign(nparts + 1, 0);
    for (size_t t = 0; t < nparts; t++) part_base[t + 1] = part_base[t] + c->part_cls[t].rep.size();
    part_map.assign(part_base[nparts], -1);
    // Speculative merge: parts' classes with equal 64-bit hashes are taken
    // as equal here, and verified exactly while the device runs (the exact
    // compares read other cores' records: ~0.2 us each on the critical path);
    // a hash collision re-runs the chunk with this exact merge (exact_merge)
    if (!c->exact_merge) {
      for (size_t t = 0; t < nparts; t++) {
        const PartClasses& pc = c->part_cls[t];
        for (size_t j = 0; j < pc.rep.size(); j++) {
          int32_t* head = cls_head.find(c->collide_test ? 0 : pc.hcls[j]);
          int32_t k = *head;
          if (k < 0) {
            k = int32_t(cls_rep.size());
            cls_rep.push_back(pc.rep[j]);
            cls_next.push_back(-1);
            *head = k;
            int32_t* shead = sig_head.find(c->collide_test ? 0 : pc.hsig[j]);
            if (*shead < 0) {
              *shead = int32_t(sig_rep.size());
              sig_rep.push_back(pc.rep[j]);
              sig_next.push_back(-1);
            }
            cls_sig.push_back(*shead);
          }
          part_map[part_base[t] + j] = k;
        }
      }
    }
    for (size_t t = 0; t < nparts && c->exact_merge; t++)
    for (size_t j = 0; j < c->part_cls[t].rep.size(); j++) {
      const size_t i = size_t(c->part_cls[t].rep[j]);
      const DevEval& e = hev[i];
      const uint64_t hs1 = h_sig[i];
      const uint64_t hc = h_cls[i];
      int32_t k = -1;
      int32_t* head = cls_head.find(hc);
      for (int32_t q = *head; q >= 0; q = cls_next[size_t(q)]) {
        const DevEval& r = hev[cls_rep[size_t(q)]];
        if (same_sig(e, r) && same_mask(e, r)) {
          k = q;
          break;
        }
      }
      if (k < 0) {
        k = int32_t(cls_rep.size());
        cls_rep.push_back(int32_t(i));
        cls_next.push_back(*head);
        *head = k;
        int32_t sg = -1;
        int32_t* shead = sig_head.find(hs1);
        for (int32_t q = *shead; q >= 0; q = sig_next[size_t(q)])
          if (same_sig(e, hev[sig_rep[size_t(q)]])) {
            sg = q;
            break;
          }
        if (sg < 0) {
          sg = int32_t(sig_rep.size());
          sig_rep.push_back(int32_t(i));
          sig_next.push_back(*shead);
          *shead = sg;
        }
        cls_sig.push_back(sg);
      }
      part_map[part_base[t] + j] = k;
    }
    for (size_t t = 0; t < nparts; t++)
      for (size_t i = ktas_pool::HostPool::part_begin(n, t, nparts); i < ktas_pool::HostPool::part_begin(n, t + 1, nparts); i++)
        cls_of[i] = part_map[part_base[t] + size_t(req_local_cls[i])];
    trace(5);
    const int ncls = int(cls_rep.size());
    // representative: the first fast-LFC member if any (its class gets an LFC table slot)
    std::vector<int32_t>& rep = c->cls_fastrep;
    rep.assign(size_t(ncls), -1);
    for (size_t i = 0; i < n; i++) {
      const int32_t k = cls_of[i];
      if (rep[size_t(k)] < 0 && req_fast[i]) rep[size_t(k)] = int32_t(i);
    }
    std::vector<int32_t>& slot_of = c->cls_slot;
    slot_of.assign(size_t(ncls), -1);
    for (int k = 0; k < ncls; k++) {
      if (rep[size_t(k)] >= 0) {
        slot_of[size_t(k)] = nslots;
        h_lrep[nslots++] = rep[size_t(k)];
      } else {
        rep[size_t(k)] = cls_rep[size_t(k)];
      }
    }
    for (size_t i = 0; i < n; i++) {
      const int32_t k = cls_of[i], r = rep[size_t(k)];
      const bool fast = slot_of[size_t(k)] >= 0 && req_fast[i];
      h_rep[i] = r;
      h_slot[i] = fast ? slot_of[size_t(k)] : -1;
      if (fast) h_fast[nfast++] = int32_t(i);
      else h_bf[nbf++] = int32_t(i);
      if (int32_t(i) != r) {
        h_pairs[2 * npairs] = r;
        h_pairs[2 * npairs + 1] = ~int32_t(i);  // exclusion stats only
        npairs++;
      }
      h_pidx[i] = -1;
      if (req_leaf[i] && !fast) {
        h_pidx[i] = nleafsel;
        h_leafsel[nleafsel++] = int32_t(i);
      }
    }
    trace(6);
    // fill chunks: classes ordered by (base signature, signature), <= kEvalsPerFillBlock
    // per chunk, one base signature each (the leaf's remaining capacity is
    // shared); a run of one signature inside a chunk shares the CountIn
    const int nsig = int(sig_rep.size());
    std::vector<int32_t>& sig_base = c->sig_base;
    sig_base.assign(size_t(nsig), -1);
    {
      std::vector<int32_t>& base_rep = c->base_rep;
      base_rep.clear();
      for (int g = 0; g < nsig; g++) {
        const DevEval& e = hev[sig_rep[size_t(g)]];
        for (size_t q = 0; q < base_rep.size() && sig_base[size_t(g)] < 0; q++)
          if (same_base(e, hev[base_rep[q]])) sig_base[size_t(g)] = int32_t(q);
        if (sig_base[size_t(g)] < 0) {
          sig_base[size_t(g)] = int32_t(base_rep.size());
          base_rep.push_back(sig_rep[size_t(g)]);
        }
        if (base_rep.size() > 64) {  // many distinct bases (assumed usage per eval): no sharing to look for
          for (int h = g + 1; h < nsig; h++) sig_base[size_t(h)] = int32_t(base_rep.size()) + (h - g - 1);
          break;
        }
      }
    }
    std::vector<int32_t>& order = c->cls_order;
    order.resize(size_t(ncls));
    for (int k = 0; k < ncls; k++) order[size_t(k)] = k;
    std::vector<int32_t>& sig_ncls = c->sig_ncls;  // classes per signature: small ones pack together
    sig_ncls.assign(size_t(nsig), 0);
    for (int k = 0; k < ncls; k++) sig_ncls[size_t(cls_sig[size_t(k)])]++;
    auto small = [&](int32_t sg) { return sig_ncls[size_t(sg)] < kEvalsPerFillBlock / 2; };
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b2) {
      const int32_t sa = cls_sig[size_t(a)], sb = cls_sig[size_t(b2)];
      const int32_t ba = sig_base[size_t(sa)], bb = sig_base[size_t(sb)];
      if (ba != bb) return ba < bb;
      if (small(sa) != small(sb)) return !small(sa);
      return sa < sb;
    });
    trace(7);
    for (int k = 0; k < ncls; k++) h_fill[k] = rep[size_t(order[size_t(k)])];
    nfill = ncls;
    {  // members other than the rep, grouped by fill position (stats written by the reduce)
      int32_t* h_moff = reinterpret_cast<int32_t*>(hs + o_moff);
      int32_t* h_mem = reinterpret_cast<int32_t*>(hs + o_mem);
      std::vector<int32_t>& pos = c->cls_pos;
      pos.resize(size_t(ncls));
      for (int k = 0; k < ncls; k++) pos[size_t(order[size_t(k)])] = k;
      for (int k = 0; k <= ncls; k++) h_moff[k] = 0;
      for (size_t i = 0; i < n; i++)
        if (int32_t(i) != rep[size_t(cls_of[i])]) h_moff[pos[size_t(cls_of[i])] + 1]++;
      for (int k = 0; k < ncls; k++) h_moff[k + 1] += h_moff[k];
      std::vector<int32_t>& cur = c->cls_cur;
      cur.assign(h_moff, h_moff + ncls);
      for (size_t i = 0; i < n; i++)
        if (int32_t(i) != rep[size_t(cls_of[i])]) h_mem[cur[size_t(pos[size_t(cls_of[i])])]++] = int32_t(i);
    }
    {  // counters are stored per class, row = fill position: evals and LFC tables refer to their class's row
      const std::vector<int32_t>& pos = c->cls_pos;
      for (size_t i = 0; i < n; i++) h_rep[i] = pos[size_t(cls_of[i])];
      for (int k = 0; k < ncls; k++)
        if (slot_of[size_t(k)] >= 0) h_lrep[slot_of[size_t(k)]] = pos[size_t(k)];
    }
    trace(8);
    int32_t* h_frun = reinterpret_cast<int32_t*>(hs + o_frun);
    // a signature with at least half a chunk of classes gets chunks of its
    // own (one run: CountIn before the eval loop); the smaller ones of a base
    // share packed chunks (several runs).  Single-run chunks first.
    std::vector<int32_t>& packed = c->cls_packed;  // [start, len) signature runs left for packing
    packed.clear();
    for (int k = 0; k < ncls;) {
      const int32_t sg = cls_sig[size_t(order[size_t(k)])];
      int e = k + 1;
      while (e < ncls && cls_sig[size_t(order[size_t(e)])] == sg) e++;
      if (e - k >= kEvalsPerFillBlock / 2) {
        for (int q = k; q < e; q += kEvalsPerFillBlock) {
          h_fchunks[2 * nfchunks] = q;
          h_fchunks[2 * nfchunks + 1] = std::min(kEvalsPerFillBlock, e - q);
          nfchunks++;
          for (int r = q; r < q + h_fchunks[2 * nfchunks - 1]; r++) h_frun[r] = nruns;
          nruns++;
        }
      } else {
        packed.push_back(k);
        packed.push_back(e - k);
      }
      k = e;
    }
    nsingle = nfchunks;
    for (size_t i = 0; i < packed.size();) {  // runs of one base, in order, up to a chunk each
      const int32_t k0 = packed[i];
      const int32_t base = sig_base[size_t(cls_sig[size_t(order[size_t(k0)])])];
      int len = 0;
      h_fchunks[2 * nfchunks] = k0;
      while (i < packed.size() && len + packed[i + 1] <= kEvalsPerFillBlock && packed[i] == k0 + len &&
             sig_base[size_t(cls_sig[size_t(order[size_t(packed[i])])])] == base) {
        for (int r = packed[i]; r < packed[i] + packed[i + 1]; r++) h_frun[r] = nruns;
        nruns++;
        len += packed[i + 1];
        i += 2;
      }
      h_fchunks[2 * nfchunks + 1] = len;
      nfchunks++;
    }
  }
  lap(1);
  trace(9);
  c->chunk_rep.assign(h_rep, h_rep + n);
  c->chunk_leader.resize(n);
  for (size_t i = 0; i < n; i++) c->chunk_leader[i] = (hev[i].flags & KUEUE_TAS_F_LEADER) ? 1 : 0;
  c->chunk_alias.assign(n, 0);  // filled with the fill records below
  // ---- device buffers ----
  const int64_t SD = s.SD;
  const int64_t full_lcap = int64_t(c->maxD) * 2 + 64;  // a list of any level's domains, twice
  const int nchunks = (s.N + kLfcChunk - 1) / kLfcChunk;
  {  // one row per class (fill position), sized by its kind (FillEvalParams::ctr_row)
    c->ctr_row_off.resize(size_t(std::max(nfill, 1)) + 1);
    int64_t at = 0;
    for (int pos = 0; pos < nfill; pos++) {
      const DevEval& ev = hev[h_fill[pos]];
      c->ctr_row_off[size_t(pos)] = int32_t(at);
      at += (ev.flags & KUEUE_TAS_F_LEADER) ? 5 : simple_class(ev, s.L) ? 1 : 2;
    }
    if (at * SD > (int64_t(1) << 40)) return fail(c, KUEUE_TAS_EINVAL, "class rows exceed the device");
    c->ctr_row_off[size_t(nfill)] = int32_t(at);
    HIPCHK(c, c->d_counters.ensure(size_t(std::max<int64_t>(at, 1)) * size_t(SD)));
  }
  // overlay, tags and scratch lists per BestFit-side select slot (fast-LFC
  // evals never mutate or walk lists): each slot's lists bounded by what its
  // walk can reach (scratch_bound), its overlay by its kind (2 fields, 5 with
  // a leader); slots run in groups whose buffers fit phase2_budget, reusing
  // one group's buffers (a fresh tag epoch per group)
  SelSlot* hsel = reinterpret_cast<SelSlot*>(hs + o_sel);
  std::vector<int32_t>& groups = c->sel_groups;
  groups.assign(1, 0);
  {
    int64_t g_scr = 0, g_ov = 0, max_scr = 2, max_ov = 1;
    int32_t g_tag = 0, max_tag = 1;
    for (int k = 0; k < nbf; k++) {
      const DevEval& ev = hev[h_bf[k]];
      const int64_t lc = (c->scratch_full || !c->scratch_bounded) ? full_lcap : scratch_bound(c, s, ev, full_lcap);
      const int64_t ovf = (ev.flags & KUEUE_TAS_F_LEADER) ? 5 : 2;
      const int64_t bytes = lc * 48 + (ovf + 1) * SD * 4;
      if (g_tag > 0 && g_scr * 8 + g_ov * 4 + int64_t(g_tag) * SD * 4 + bytes > c->phase2_budget) {
        groups.push_back(k);
        g_scr = g_ov = 0;
        g_tag = 0;
      }
      hsel[k] = SelSlot{g_scr, g_ov, g_tag, int32_t(lc)};
      g_scr += 6 * lc;
      g_ov += ovf * SD;
      g_tag++;
      max_scr = std::max(max_scr, g_scr);
      max_ov = std::max(max_ov, g_ov);
      max_tag = std::max(max_tag, g_tag);
    }
    groups.push_back(nbf);
    HIPCHK(c, c->d_scratch.ensure(size_t(max_scr)));
    HIPCHK(c, c->d_overlay.ensure(size_t(max_ov)));
    const int ngroups = int(groups.size()) - 1;
    if (c->d_tags.n < size_t(max_tag) * size_t(SD) || c->tag_epoch + ngroups >= 0x7ffffff0) {  // fresh tags: nothing owned
      HIPCHK(c, c->d_tags.ensure(size_t(max_tag) * size_t(SD)));
      HIPCHK(c, hipMemsetAsync(c->d_tags.p, 0, c->d_tags.n * 4, c->stream));
      c->tag_epoch = 0;
    }
  }
  c->tag_epoch++;
  const size_t nt = size_t(std::max(num_taints, 0));
  const size_t stats_len = n * nt + n * size_t(s.R) + 3 * n;  // taints | resources | nodeSelector | affinity | topologyDomain
  const size_t res_off_stats = (n * sizeof(kueue_tas_eval_out) + 15) / 16 * 16;
  const size_t res_bytes = res_off_stats + stats_len * 4;
  HIPCHK(c, c->d_res.ensure(res_bytes));
  HIPCHK(c, c->h_res.ensure(res_bytes));
  HIPCHK(c, c->h_res2.ensure(n));
  kueue_tas_eval_out* d_out = reinterpret_cast<kueue_tas_eval_out*>(c->d_res.p);
  int32_t* d_stats = reinterpret_cast<int32_t*>(c->d_res.p + res_off_stats);
  c->res_out_h = reinterpret_cast<kueue_tas_eval_out*>(c->h_res.p);
  c->res_stats_h = reinterpret_cast<int32_t*>(c->h_res.p + res_off_stats);
  // ExclusionStats are fully written by the fill's reduce (class reps) and the
  // replication (other members) when the staged fill counts them in LDS
  uint32_t umask = 0;
  for (size_t i = 0; i < n; i++) umask |= hev[i].req_mask | hev[i].lead_mask;
  const int ucols = __builtin_popcount(umask);
  const int nstat_all = kStatFixed + int(nt) + s.R;
  const bool lds_stats = s.N > 0 && nfchunks > 0 && ucols <= 8 && nstat_all <= kMaxFillStats;
  // per-eval entry regions [n][entry_cap] pairs in pinned, device-mapped host
  // memory: select / lfc_emit write the (leaf, count) pairs the host reads
  // after the batch's one sync (no offsets/pack kernels, no entries D2H)
  {
    const size_t need_ints = c->ent_used + size_t(n) * size_t(entry_cap) * 2;
    if (need_ints > c->ent_cap) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      size_t cap = std::max<size_t>(need_ints, 2 * c->ent_cap);
      int32_t* p = nullptr;
      HIPCHK(c, hipHostMalloc(&p, cap * 4, hipHostMallocMapped | hipHostMallocCoherent));
      if (c->ent_used) memcpy(p, c->ent_host, c->ent_used * 4);
      if (c->ent_host) (void)hipHostFree(c->ent_host);
      c->ent_host = p;
      c->ent_cap = cap;
      HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->ent_dev), p, 0));
    }
    if (c->leaf_tags_on && c->tag_cap < c->ent_cap / 2) {  // one tag per entry pair, same layout
      HIPCHK(c, hipStreamSynchronize(c->stream));
      const size_t cap = c->ent_cap / 2;
      uint64_t* p = nullptr;
      HIPCHK(c, hipHostMalloc(&p, cap * 8, hipHostMallocMapped | hipHostMallocCoherent));
      if (c->ent_used && c->tag_host) memcpy(p, c->tag_host, c->ent_used / 2 * 8);
      if (c->tag_host) (void)hipHostFree(c->tag_host);
      c->tag_host = p;
      c->tag_cap = cap;
      HIPCHK(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->tag_dev), p, 0));
    }
    if (c->leaf_tags_on) c->fill_paths |= KUEUE_TAS_PATH_ENTRY_TAGS;
    c->snap.leaf_tag = c->leaf_tags_on ? c->d_leaf_tags.p : nullptr;
    c->snap.tag_out = c->leaf_tags_on ? c->tag_dev : nullptr;
    c->snap.ent_base = c->ent_dev;
  }
  HIPCHK(c, c->d_lfc_jobs.ensure(n));
  HIPCHK(c, c->d_lfc_items.ensure(size_t(std::max(nfast, 1)) * size_t(std::max(nchunks, 1)) + 1));
  // chunk counts and overflow sums in two halves used by alternate batches:
  // the fill accumulates into zeroed tables (DevBatch::lfc_fill), and a
  // half's zeroing runs on stream2 during the batch that does not use it
  const size_t lfc_need = size_t(std::max(nslots * nchunks, 1));
  if (lfc_need > c->lfc_half) {
    c->lfc_half = lfc_need + lfc_need / 4;
    HIPCHK(c, c->d_lfc_ch.ensure(2 * c->lfc_half * kLfcBins));
    HIPCHK(c, c->d_lfc_ovs.ensure(2 * c->lfc_half));
    c->lfc_dirty[0] = c->lfc_dirty[1] = true;
  }
  const int lfc_cur = c->lfc_parity;
  HIPCHK(c, c->d_lfc_cp.ensure(size_t(std::max(nslots * nchunks, 1)) * kLfcBins));
  HIPCHK(c, c->d_lfc_tot.ensure(size_t(std::max(nslots, 1)) * kLfcBins));

  HIPCHK(c, c->d_lfc_ovtot.ensure(size_t(std::max(nslots, 1))));
  HIPCHK(c, c->d_lfc_u8.ensure(size_t(std::max(nslots, 1)) * size_t(std::max(nchunks, 1)) * kLfcChunk));
  const int nblk = (s.N + 255) / 256 * 4;  // one leaf partial per 64-leaf wave
  HIPCHK(c, c->d_partials.ensure(size_t(std::max(nleafsel, 1)) * size_t(std::max(nblk, 1))));

  if (c->fused_top) {  // rollup_top_kernel's initial level maxima and arrival counters
    int32_t* t = reinterpret_cast<int32_t*>(hs + o_top);
    for (size_t i = 0; i < size_t(nfill) * kMaxLevels; i++) t[i] = INT32_MIN;
    for (size_t i = 0; i < size_t(nfill); i++) t[n * kMaxLevels + i] = 0;
  }
  trace(10);
  // fill_pair_kernel's per-position records in fill order (FillPos)
  {
    FillPos* fp = reinterpret_cast<FillPos*>(hs + o_fpos);
    const int32_t* h_fill = reinterpret_cast<const int32_t*>(hs + o_fill);
    const int32_t* h_fch = reinterpret_cast<const int32_t*>(hs + o_fchunks);
    const int32_t* h_frun = reinterpret_cast<const int32_t*>(hs + o_frun);
    const int nsw = ucols <= 4 ? 4 : ucols <= 5 ? 5 : 8;  // the launch's NS: worker terms [0, NS), leader terms [NS, 2 NS)
    for (int ch = 0; ch < nfchunks; ch++) {
      const int e0 = h_fch[2 * ch], ne = h_fch[2 * ch + 1];
      const DevEval& base = hev[h_fill[e0]];
      for (int t = 0; t < ne; t++) {
        const int pos = e0 + t;
        const DevEval& ev = hev[h_fill[pos]];
        FillPos& r = fp[pos];
        memset(&r, 0, sizeof r);
        FillEvalParams& P = r.p;
        P.eid = h_fill[pos];
        P.lfc_slot = c->cls_slot[size_t(c->cls_order[size_t(pos)])];  // fast-LFC table slot, -1: none
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
        for (int k = 0; k < KUEUE_TAS_MAX_SELECTORS; k++) {
          P.sel_col[k] = ev.sel_col[k];
          P.sel_val[k] = ev.sel_val[k];
          if (k < ev.nsel && ev.sel_col[k] >= kStagedLabels) P.sel_far = 1;
        }
        P.sx_begin = ev.sx_begin;
        P.sx_end = ev.sx_end;
        P.ss_alias = simple_class(ev, s.L) ? 1 : 0;
        P.ctr_row = c->ctr_row_off[size_t(pos)];
        if (ev.sx_begin >= 0) P.sel_far = 1;
        {  // the packed nodeSelector compare (FillEvalParams::sel_fast)
          uint32_t m[2] = {0u, 0u}, w[2] = {0u, 0u};
          bool fast = c->labels16 && !P.sel_far, never = false;
          for (int k = 0; k < ev.nsel && fast; k++) {
            const int col = ev.sel_col[k];
            const uint32_t sh = uint32_t(col & 1) * 16u;
            const uint32_t fm = 0xffffu << sh;
            if (col < 0 || col >= kStagedLabels) {
              fast = false;
              break;
            }
            const int32_t val = ev.sel_val[k];
            if (val < 0 || val > 0xffff) {  // a value no leaf has
              never = true;
              continue;
            }
            const uint32_t fw = uint32_t(val) << sh;
            uint32_t& mm = m[col >> 1];
            uint32_t& ww = w[col >> 1];
            if ((mm & fm) && (ww & fm) != fw) never = true;  // one column, two values
            mm |= fm;
            ww = (ww & ~fm) | fw;
          }
          if (fast && never) {  // want bits outside the mask: no leaf matches
            m[0] = 0u;
            w[0] = 1u;
          }
          P.sel_fast = fast ? 1 : 0;
          P.sel_mlo = m[0];
          P.sel_mhi = m[1];
          P.sel_wlo = w[0];
          P.sel_whi = w[1];
        }
        P.run = h_frun[pos];
        P.sig_new = t == 0 || h_frun[pos - 1] != P.run;
        P.rmask = int32_t(ev.req_mask);
        P.lmask = int32_t(ev.lead_mask);
        P.pad[0] = int32_t(base.flags);  // the chunk's base signature
        P.pad[1] = base.assumed_begin;
        P.pad[2] = base.assumed_end;
        for (int q = 0; q < kStagedProfiles; q++)
          r.taint[q] = q < c->num_profiles && size_t(ev.taint_table + q) < taint_table_len ? taint_table[ev.taint_table + q] : -1;
        for (int j = 0; j < ev.nreq && j < nsw; j++) r.term[j] = hterms[ev.term_begin + j];
        for (int j = 0; j < ev.nlead && j < nsw; j++) r.term[nsw + j] = hterms[ev.lead_begin + j];
      }
    }
    for (size_t i = 0; i < n; i++) c->chunk_alias[i] = uint8_t(fp[c->chunk_rep[i]].p.ss_alias);
    for (int k = 0; k < nfill; k++) c->last_alias_fills += fp[k].p.ss_alias;
  }
  trace(11);
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_stage.p, hs, o_fpos + size_t(nfill) * sizeof(FillPos), hipMemcpyHostToDevice, c->stream));
  // the select path's descriptor (g_select_snap), ordered before both select
  // launches: stream2 joins after events recorded later on this stream.
  // Uploaded only when it differs from what the device already holds (the
  // caller serializes batches per process, and every batch drains before
  // eval_batch returns), so a steady stream of batches pays no extra copy.
  {
    static DevSnap uploaded[16];
    static bool valid[16];
    const int dev = (c->device >= 0 && c->device < 16) ? c->device : -1;
    if (dev < 0 || !valid[dev] || std::memcmp(&uploaded[dev], &c->snap, sizeof(DevSnap)) != 0) {
      HIPCHK(c, hipMemcpyToSymbolAsync(HIP_SYMBOL(g_select_snap), &c->snap, sizeof(DevSnap), 0,
                                       hipMemcpyHostToDevice, c->stream));
      if (dev >= 0) {
        std::memcpy(&uploaded[dev], &c->snap, sizeof(DevSnap));
        valid[dev] = true;
      }
    }
  }
  trace(12);
  if (!lds_stats) HIPCHK(c, hipMemsetAsync(d_stats, 0, stats_len * 4, c->stream));
  uint8_t* ds = c->d_stage.p;
  DevBatch b{};
  b.evals = reinterpret_cast<const DevEval*>(ds + o_evals);
  b.terms = reinterpret_cast<const DevTerm*>(ds + o_terms);
  b.taint_table = reinterpret_cast<const int32_t*>(ds + o_taint);
  b.assumed = reinterpret_cast<const kueue_tas_assumed*>(ds + o_assumed);
  b.aff = reinterpret_cast<const kueue_tas_affinity_req*>(ds + o_aff);
  b.aff_vals = reinterpret_cast<const int32_t*>(ds + o_affv);
  b.n = int32_t(n);
  b.num_taints = int32_t(nt);
  b.num_profiles = c->num_profiles;
  b.nstat = 0;
  b.nstat_R = s.R;
  b.fill_stats = nullptr;
  b.stats_split = 0;
  b.fill_lim = nullptr;
  b.cls_member_off = nullptr;
  b.cls_members = nullptr;
  b.rack_fanout = 0;
  b.rack_pos = nullptr;
  b.ctr_sd = SD;
  b.counters = c->d_counters.p;
  b.overlay = c->d_overlay.p;
  b.tags = c->d_tags.p;
  b.tag_epoch = c->tag_epoch;
  b.taint_counts = d_stats;
  b.res_counts = d_stats + n * nt;
  b.sel_counts = d_stats + n * nt + n * size_t(s.R);
  b.aff_counts = b.sel_counts + n;
  b.dom_counts = b.aff_counts + n;
  b.out = d_out;
  b.entries = c->ent_dev + c->ent_used;
  b.entry_cap = entry_cap;
  b.sel_slots = reinterpret_cast<const SelSlot*>(ds + o_sel);
  b.slot_base = 0;
  b.scratch = c->d_scratch.p;
  b.list_cap = c->list_cap;
  b.nblk = nblk;
  b.partials = c->d_partials.p;
  b.partial_idx = reinterpret_cast<const int32_t*>(ds + o_pidx);
  b.rep_of = reinterpret_cast<const int32_t*>(ds + o_rep);
  b.lfc_slot = reinterpret_cast<const int32_t*>(ds + o_slot);
  b.lfc_rep = reinterpret_cast<const int32_t*>(ds + o_lrep);
  b.lfc_nslots = nslots;
  b.lfc_nchunks = nchunks;
  b.lfc_ch = c->d_lfc_ch.p + size_t(lfc_cur) * c->lfc_half * kLfcBins;
  b.lfc_u8 = c->d_lfc_u8.p;
  b.exp_flags = c->exp_flags;
  b.lfc_cp = c->d_lfc_cp.p;
  b.lfc_tot = c->d_lfc_tot.p;
  b.lfc_ovs = c->d_lfc_ovs.p + size_t(lfc_cur) * c->lfc_half;
  b.lfc_ovtot = c->d_lfc_ovtot.p;
  b.lfc_jobs = c->d_lfc_jobs.p;
  b.lfc_nitems = reinterpret_cast<int32_t*>(c->d_lfc_items.p);  // item 0's slot holds the count
  b.lfc_items = c->d_lfc_items.p + 1;
  b.prof = nullptr;
  if (KTAS_PROFILE) {
    HIPCHK(c, c->d_prof.ensure(n * P_NCAT));
    HIPCHK(c, hipMemsetAsync(c->d_prof.p, 0, n * P_NCAT * 4, c->stream));
    b.prof = c->d_prof.p;
    HIPCHK(c, c->d_fprof.ensure(size_t(1) << 18));
    HIPCHK(c, hipMemsetAsync(c->d_fprof.p, 0, (size_t(1) << 18) * 4, c->stream));
    b.fill_prof = c->d_fprof.p;
  }
  c->stat_fills += nfill;
  c->stat_evals += int64_t(n);
  const int32_t* d_pairs = reinterpret_cast<const int32_t*>(ds + o_pairs);
  const int32_t* d_leafsel = reinterpret_cast<const int32_t*>(ds + o_leafsel);
  b.fill_ids = reinterpret_cast<const int32_t*>(ds + o_fill);
  b.nfill = nfill;
  b.fill_chunks = reinterpret_cast<const int32_t*>(ds + o_fchunks);
  b.fill_run = reinterpret_cast<const int32_t*>(ds + o_frun);
  b.fill_pos = reinterpret_cast<const FillPos*>(ds + o_fpos);
  // K1
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  c->last_stats[0] += nfill;
  if (s.N > 0 && nfchunks > 0) {
    dim3 grid((s.N + 255) / 256, unsigned(nfchunks));
    // the staged kernels take kFillTilesPerBlock leaf tiles per block (with
    // ragged parents a tile is 4 packed wave slots)
    const bool staged_fill = ucols <= 8;
    const unsigned stiles = ucols <= 8 && c->rack_fanout < 0 ? unsigned((s.n_wave_slots + 3) / 4) : grid.x;
    const unsigned sgx = (stiles + kFillTilesPerBlock - 1) / kFillTilesPerBlock;
    const unsigned nblk_fill = staged_fill ? sgx : grid.x;  // blocks per fill position (stats partials)
    c->last_stats[2] += 1;
    c->last_stats[3] = ucols;
    const int nstat = nstat_all;
    b.nstat = lds_stats ? nstat : 0;
    b.nstat_R = s.R;
    // single-run chunks on fill_pair_kernel (kPairLP leaves per thread): staged
    // columns, uniform fan-out >= 2 or no fused parents; it counts the
    // ExclusionStats itself, so the batch takes the inline-stats path
    // ragged leaf parents of <= 128 leaves on fill_pair_kernel (two leaves per
    // lane, segmented scans over the lanes' pairs): every class without a
    // leader (leader classes keep the one-leaf staged kernel)
    bool any_leader = false;
    for (size_t i = 0; i < n && !any_leader; i++) any_leader = (hev[i].flags & KUEUE_TAS_F_LEADER) != 0;
    const bool ragged_pair = c->pair_fill && staged_fill && s.wave_tab2 != nullptr && !any_leader;
    const bool pair = c->pair_fill && staged_fill &&
                      (ragged_pair || (c->rack_fanout >= 0 && (c->rack_fanout == 0 || c->rack_fanout >= kPairLP)));
    const unsigned pgx = ragged_pair ? unsigned((s.n_wave_slots2 + 3) / 4) : unsigned((s.N + kPairTile - 1) / kPairTile);
    if (b.nstat) {
      // sized for the tile grid: fill_exclusion_kernel (split stats) writes one partial per tile
      HIPCHK(c, c->d_fill_stats.ensure(size_t(nfill) * std::max(grid.x, nblk_fill) * size_t(nstat)));
      b.fill_stats = c->d_fill_stats.p;
      // the reduce sums every member's stats and stores them for the class's other members
      b.cls_member_off = reinterpret_cast<const int32_t*>(ds + o_moff);
      b.cls_members = reinterpret_cast<const int32_t*>(ds + o_mem);
    }
    if (b.nstat && !c->inline_stats && !pair) {  // staged fill: ExclusionStats by fill_exclusion_kernel on stream3
      HIPCHK(c, c->d_fill_lim.ensure(size_t(nruns) * size_t(s.N)));
      b.stats_split = 1;
      b.fill_lim = c->d_fill_lim.p;
    }
    // partial slots per fill position: the exclusion grid (split), else the widest fill grid
    b.nstat_blocks = int32_t(b.stats_split ? grid.x : pair ? pgx : nblk_fill);
    b.rack_fanout = ragged_pair ? -1 : ucols <= 8 ? c->rack_fanout : 0;  // the fill fuses the first roll-up level
    if (b.rack_fanout) {
      c->fill_paths |= b.rack_fanout < 0 ? KUEUE_TAS_PATH_RAGGED_ROLLUP : KUEUE_TAS_PATH_UNIFORM_ROLLUP;
      if (ragged_pair) c->fill_paths |= KUEUE_TAS_PATH_RAGGED_PAIR;
      // positive-children masks are 64-bit: none when a ragged parent is wider
      if (!ragged_pair || s.ragged_max_fan <= kWave) {
        HIPCHK(c, c->d_rack_pos.ensure(size_t(nfill) * size_t(s.level_size[s.L - 2])));
        b.rack_pos = c->d_rack_pos.p;
      }
    }
    const bool ts = b.num_profiles <= kStagedProfiles;
    // global lookups in the eval loop: a nodeSelector column beyond the
    // staged label columns, or required node affinity
    bool gl = false;
    for (size_t i = 0; i < n && !gl; i++) {
      gl = (hev[i].flags & (KUEUE_TAS_F_AFFINITY | KUEUE_TAS_F_SELECTOR_EXT)) != 0;
      for (int k = 0; k < hev[i].nsel; k++) gl = gl || hev[i].sel_col[k] >= kStagedLabels;
    }
    // leaf parents wider than a slot: zeroed before the ragged pair fill adds
    // its pieces' sums (the fill bracket and stream2's chunks start after it)
    const bool wide = ragged_pair && s.n_wide > 0;
    if (wide) {
      hipLaunchKernelGGL(wide_parents_zero_kernel, dim3(unsigned((s.n_wide + 255) / 256), unsigned(nfill)), dim3(256), 0,
                         c->stream, s, b);
      HIPCHK(c, hipGetLastError());
      HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
    }
    // leaf categories in the single-run pair fill: every filter on staged
    // data (no affinity, no far selector column: !gl), taint rows and the
    // ExclusionStats in LDS, label ids packed in 16 bits
    const bool cat = c->cat_fill && pair && !gl && ts && b.nstat > 0 && c->labels16;
    // the fast-LFC chunk tables accumulated by the fill itself (every chunk
    // runs on fill_pair_kernel: its lean loop from the block's (category,
    // value) pairs, its per-leaf loop per wave): no lfc_hist_kernel
    // re-reading the slot classes' leaf rows
    b.lfc_fill = (nfast > 0 && pair && c->lfc_in_fill) ? 1 : 0;
    if (b.lfc_fill) c->fill_paths |= KUEUE_TAS_PATH_LFC_FILL;
    if (b.lfc_fill && c->lfc_dirty[lfc_cur]) {  // (after a reallocation: zeroed before the fill)
      HIPCHK(c, hipMemsetAsync(b.lfc_ch, 0, c->lfc_half * kLfcBins * 4, c->stream));
      HIPCHK(c, hipMemsetAsync(b.lfc_ovs, 0, c->lfc_half * 8, c->stream));
      c->lfc_dirty[lfc_cur] = false;
    }
    // single-run chunks [0, nsingle) and multi-run chunks [nsingle, nfchunks): one launch each
    auto staged = [&](auto ns, auto tsv, auto mr, int first, int count, hipStream_t st) {
      if (count <= 0) return;
      constexpr int NSv = decltype(ns)::value;
      constexpr bool TSv = decltype(tsv)::value, MRv = decltype(mr)::value;
      if (pair) {  // kPairLP leaves per thread
        c->fill_paths |= KUEUE_TAS_PATH_PAIR;
        const dim3 pg(pgx, unsigned(count));
        if constexpr (TSv && !MRv) {  // single-run chunks: leaf categories
          if (cat) {
            c->fill_paths |= KUEUE_TAS_PATH_CATEGORY;
            if (b.lfc_fill) {  // (the lean loop's LFC pair lists in LDS)
              if (ragged_pair)
                hipLaunchKernelGGL((fill_pair_kernel<NSv, true, false, false, -1, true, true>), pg, dim3(256), 0, st, s, b, umask, first);
              else if (b.rack_fanout == 32)
                hipLaunchKernelGGL((fill_pair_kernel<NSv, true, false, false, 32, true, true>), pg, dim3(256), 0, st, s, b, umask, first);
              else
                hipLaunchKernelGGL((fill_pair_kernel<NSv, true, false, false, 0, true, true>), pg, dim3(256), 0, st, s, b, umask, first);
            } else if (ragged_pair) {
              hipLaunchKernelGGL((fill_pair_kernel<NSv, true, false, false, -1, true>), pg, dim3(256), 0, st, s, b, umask, first);
            } else if (b.rack_fanout == 32) {
              hipLaunchKernelGGL((fill_pair_kernel<NSv, true, false, false, 32, true>), pg, dim3(256), 0, st, s, b, umask, first);
            } else {
              hipLaunchKernelGGL((fill_pair_kernel<NSv, true, false, false, 0, true>), pg, dim3(256), 0, st, s, b, umask, first);
            }
            return;
          }
        }
        if (ragged_pair && gl)
          hipLaunchKernelGGL((fill_pair_kernel<NSv, TSv, MRv, true, -1>), pg, dim3(256), 0, st, s, b, umask, first);
        else if (ragged_pair)
          hipLaunchKernelGGL((fill_pair_kernel<NSv, TSv, MRv, false, -1>), pg, dim3(256), 0, st, s, b, umask, first);
        else if (gl && b.rack_fanout == 32)
          hipLaunchKernelGGL((fill_pair_kernel<NSv, TSv, MRv, true, 32>), pg, dim3(256), 0, st, s, b, umask, first);
        else if (gl)
          hipLaunchKernelGGL((fill_pair_kernel<NSv, TSv, MRv, true, 0>), pg, dim3(256), 0, st, s, b, umask, first);
        else if (b.rack_fanout == 32)
          hipLaunchKernelGGL((fill_pair_kernel<NSv, TSv, MRv, false, 32>), pg, dim3(256), 0, st, s, b, umask, first);
        else
          hipLaunchKernelGGL((fill_pair_kernel<NSv, TSv, MRv, false, 0>), pg, dim3(256), 0, st, s, b, umask, first);
        return;
      }
      if (gl)
        hipLaunchKernelGGL((fill_leaves_staged_kernel<NSv, TSv, MRv, true>), dim3(sgx, unsigned(count)), dim3(256), 0,
                           st, s, b, umask, first);
      else
        hipLaunchKernelGGL((fill_leaves_staged_kernel<NSv, TSv, MRv, false>), dim3(sgx, unsigned(count)), dim3(256), 0,
                           st, s, b, umask, first);
    };
    // the multi-run chunks (a few small signatures) run beside the single-run
    // chunks on stream2 (idle until the fill is done): their launch's ramp and
    // tail overlap the big launch instead of following it
    auto staged2 = [&](auto ns, auto tsv) -> int {
      const bool side = nsingle > 0 && nfchunks > nsingle;
      if (side) {
        HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev[1], 0));
        staged(ns, tsv, std::true_type(), nsingle, nfchunks - nsingle, c->stream2);
        HIPCHK(c, hipEventRecord(c->evl[2], c->stream2));
      } else {
        staged(ns, tsv, std::true_type(), nsingle, nfchunks - nsingle, c->stream);
      }
      staged(ns, tsv, std::false_type(), 0, nsingle, c->stream);
      if (side) HIPCHK(c, hipStreamWaitEvent(c->stream, c->evl[2], 0));
      return 0;
    };
    using I4 = std::integral_constant<int, 4>;
    using I5 = std::integral_constant<int, 5>;
    using I8 = std::integral_constant<int, 8>;
    int src = 0;
    c->fill_paths |= ucols <= 8 ? (ts ? KUEUE_TAS_PATH_STAGED : KUEUE_TAS_PATH_STAGED_GLOBAL_TAINTS)
                                : maxt <= 4 ? KUEUE_TAS_PATH_GENERIC4 : maxt <= 8 ? KUEUE_TAS_PATH_GENERIC8
                                : maxt <= 16 ? KUEUE_TAS_PATH_GENERIC16 : KUEUE_TAS_PATH_GENERIC32;
    if (ucols <= 8 && gl) c->fill_paths |= KUEUE_TAS_PATH_STAGED_GL;
    if (!lds_stats) c->fill_paths |= KUEUE_TAS_PATH_GLOBAL_STATS;
    if (b.stats_split) c->fill_paths |= b.num_profiles <= kStagedProfiles ? KUEUE_TAS_PATH_EXCL : KUEUE_TAS_PATH_EXCL_GLOBAL_TAINTS;
    for (size_t i = 0; i < n; i++)
      if (hev[i].sx_begin >= 0) c->fill_paths |= KUEUE_TAS_PATH_SELECTOR_EXT;
    if (ucols <= 4 && ts) src = staged2(I4(), std::true_type());
    else if (ucols <= 4) src = staged2(I4(), std::false_type());
    else if (ucols <= 5 && ts) src = staged2(I5(), std::true_type());
    else if (ucols <= 5) src = staged2(I5(), std::false_type());
    else if (ucols <= 8 && ts) src = staged2(I8(), std::true_type());
    else if (ucols <= 8) src = staged2(I8(), std::false_type());
    else if (maxt <= 4) hipLaunchKernelGGL(fill_leaves_kernel<4>, grid, dim3(256), 0, c->stream, s, b);
    else if (maxt <= 8) hipLaunchKernelGGL(fill_leaves_kernel<8>, grid, dim3(256), 0, c->stream, s, b);
    else if (maxt <= 16) hipLaunchKernelGGL(fill_leaves_kernel<16>, grid, dim3(256), 0, c->stream, s, b);
    else hipLaunchKernelGGL(fill_leaves_kernel<32>, grid, dim3(256), 0, c->stream, s, b);
    if (src) return src;
    HIPCHK(c, hipGetLastError());
    if (wide) {
      hipLaunchKernelGGL(wide_parents_finish_kernel, dim3(unsigned((s.n_wide + 255) / 256), unsigned(nfill)), dim3(256),
                         0, c->stream, s, b);
      HIPCHK(c, hipGetLastError());
    }
  }
  trace(13);
  HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
  // ExclusionStats on stream3 beside the roll-up / select, joined before the
  // D2H: the reduce of the fill's per-block partials (counted inside the
  // fill), or the split path's counting kernel + reduce
  const bool stats_branch = b.nstat > 0;
  if (stats_branch && !b.stats_split) {
    HIPCHK(c, hipStreamWaitEvent(c->stream3, c->ev[2], 0));
    if (c->stage_timing) HIPCHK(c, hipEventRecord(c->evs[0], c->stream3));
    hipLaunchKernelGGL(fill_stats_reduce_kernel, dim3(unsigned(nfill)), dim3(256), 0, c->stream3, b, int(b.nstat_blocks));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->evs[1], c->stream3));
  }
  if (b.stats_split) {  // counts, reduce and member stores beside the roll-up / select
    HIPCHK(c, hipStreamWaitEvent(c->stream3, c->ev[2], 0));
    if (c->stage_timing) HIPCHK(c, hipEventRecord(c->evs[0], c->stream3));
    dim3 grid((s.N + 255) / 256, unsigned(nfchunks));
    if (b.num_profiles <= kStagedProfiles) hipLaunchKernelGGL(fill_exclusion_kernel<true>, grid, dim3(256), 0, c->stream3, s, b);
    else hipLaunchKernelGGL(fill_exclusion_kernel<false>, grid, dim3(256), 0, c->stream3, s, b);
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(fill_stats_reduce_kernel, dim3(unsigned(nfill)), dim3(256), 0, c->stream3, b, int(grid.x));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->evs[1], c->stream3));
  }
  // K2
  const int upper = s.L - 2 - (b.rack_fanout ? 1 : 0);  // levels [0, upper] left to roll up
  int top_parents = 0;  // parents above level `upper`: the fused launch's last block rolls them up
  for (int l = 0; l < upper; l++) top_parents += s.level_size[l];
  const bool fused_top = c->fused_top && nfill > 0 && upper >= 0 && s.level_size[upper] > 0 && top_parents <= 4096 &&
                         s.level_size[upper + 1] / s.level_size[upper] >= 8;
  if (fused_top) {  // every upper level and the level maxima in one launch
    b.level_max = nbf > 0 ? reinterpret_cast<int32_t*>(ds + o_top) : nullptr;
    const int per_block = 4 * kParentsPerWave;
    dim3 grid((s.level_size[upper] + per_block - 1) / per_block, unsigned(nfill));
    hipLaunchKernelGGL(rollup_top_kernel, grid, dim3(256), 0, c->stream, s, b, upper,
                       reinterpret_cast<int32_t*>(ds + o_top) + n * kMaxLevels);
    HIPCHK(c, hipGetLastError());
  }
  // the small top levels (<= kTailParents domains) go to rollup_tail_kernel with the level maxima
  int tail_top = -1;
  if (!fused_top && nfill > 0)
    for (int l = upper; l >= 0 && tail_top < 0; l--)
      if (s.level_size[l] <= kTailParents) tail_top = l;
  for (int l = fused_top ? -1 : upper; l > tail_top; l--) {
    if (s.level_size[l] <= 0) continue;
    const int fanout = s.level_size[l + 1] / s.level_size[l];
    if (fanout >= 8) {  // wave per parent: coalesced child reads
      const int per_block = 4 * kParentsPerWave;
      dim3 grid((s.level_size[l] + per_block - 1) / per_block, unsigned(nfill));
      hipLaunchKernelGGL(rollup_level_wave_kernel, grid, dim3(256), 0, c->stream, s, b, l);
    } else {
      dim3 grid((s.level_size[l] + 255) / 256, unsigned(nfill));
      hipLaunchKernelGGL(rollup_level_kernel, grid, dim3(256), 0, c->stream, s, b, l);
    }
    HIPCHK(c, hipGetLastError());
  }
  if (!fused_top && nfill > 0 && s.L >= 2 && (nbf > 0 || tail_top >= 0)) {
    // the small top levels and the level maxima for the BestFit-side find_level
    b.level_max = nullptr;
    if (nbf > 0) {
      HIPCHK(c, c->d_level_max.ensure(size_t(nfill) * size_t(kMaxLevels)));
      b.level_max = c->d_level_max.p;
    }
    hipLaunchKernelGGL(rollup_tail_kernel, dim3(unsigned(nfill)), dim3(256), 0, c->stream, s, b, tail_top);
    HIPCHK(c, hipGetLastError());
  }
  trace(14);
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
  const bool replicated = npairs && !b.nstat;
  if (replicated) {  // exclusion stats of the class rep to the other members (global-atomic stats)
    hipLaunchKernelGGL(replicate_kernel, dim3(1, unsigned(npairs)), dim3(256), 0, c->stream, s, b, d_pairs, npairs);
    HIPCHK(c, hipGetLastError());
  }
  // an event on the main stream costs ~8 us of its device time (rocprof
  // kernel trace): recorded only when the fast-LFC branch waits for the
  // replication, or for the stage profile
  if (replicated || c->stage_timing) HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
  const int32_t* d_fast = reinterpret_cast<const int32_t*>(ds + o_fast);
  const int32_t* d_bf = reinterpret_cast<const int32_t*>(ds + o_bf);
  const int waves = kSelectWaves;  // the kernel's per-wave LDS state is sized for this
  // per-wave LDS: the sort capacity (list_cap keys); the BestFit side also
  // holds lds_level_walk's candidates (kFinalWalkLds per wave)
  const int lfc_wave_lds = c->list_cap * 16, bf_wave_lds = std::max(lfc_wave_lds, kFinalWalkLds);
  // leaf-level selection partials (non-fast evals whose requested level is the leaf level)
  if (nleafsel && s.N > 0) {
    c->last_stats[1] += nleafsel;
    dim3 grid((s.N + 255) / 256, unsigned((nleafsel + kEvalsPerFillBlock - 1) / kEvalsPerFillBlock));
    hipLaunchKernelGGL(leaf_partials_kernel, grid, dim3(256), 0, c->stream, s, b, d_leafsel, nleafsel);
    HIPCHK(c, hipGetLastError());
  }
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev[5], c->stream));
  const bool emit_main = c->emit_after_bf && nbf > 0 && nfast > 0;
  const int emit_grid = int(std::min<int64_t>(int64_t(nfast) * nchunks, 2048));
  // K3 (BestFit side and every other non-fast eval)
  if (nbf) {
    b.wave_lds = bf_wave_lds;
    const int32_t epoch0 = c->tag_epoch;
    for (size_t gi = 0; gi + 1 < c->sel_groups.size(); gi++) {  // one launch per slot group (one, within budget)
      const int g0 = c->sel_groups[gi], gn = c->sel_groups[gi + 1] - g0;
      b.slot_base = g0;
      b.tag_epoch = epoch0 + int32_t(gi);
      c->tag_epoch = b.tag_epoch;
      hipLaunchKernelGGL(select_kernel, dim3(unsigned((gn + waves - 1) / waves)), dim3(64 * waves),
                         size_t(waves) * size_t(bf_wave_lds), c->stream, s, b, d_bf + g0, gn);
      HIPCHK(c, hipGetLastError());
    }
    b.slot_base = 0;
  }
  trace(16);
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev[6], c->stream));
  // fast-LFC branch on stream2: leaf tables (after the fill), select + emit
  // (after the stats replication); the main stream runs the BestFit side.
  // Enqueued after the BestFit select: that launch is on the batch's longest
  // chain, and the host's calls for this branch would otherwise delay it
  if (nfast) {
    if (c->lfc_dirty[lfc_cur ^ 1]) {  // the next batch's half, zeroed while this batch runs
      HIPCHK(c, hipMemsetAsync(c->d_lfc_ch.p + size_t(lfc_cur ^ 1) * c->lfc_half * kLfcBins, 0,
                               c->lfc_half * kLfcBins * 4, c->stream2));
      HIPCHK(c, hipMemsetAsync(c->d_lfc_ovs.p + size_t(lfc_cur ^ 1) * c->lfc_half, 0, c->lfc_half * 8, c->stream2));
      c->lfc_dirty[lfc_cur ^ 1] = false;
    }
    c->lfc_dirty[lfc_cur] = true;  // this batch writes its half
    c->lfc_parity = lfc_cur ^ 1;
    HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev[2], 0));  // fill done
    if (c->stage_timing) HIPCHK(c, hipEventRecord(c->evl[0], c->stream2));
    if (!b.lfc_fill) {
      hipLaunchKernelGGL(lfc_hist_kernel, dim3(unsigned(nchunks), unsigned(nslots)), dim3(256), 0, c->stream2, s, b);
      HIPCHK(c, hipGetLastError());
    }
    hipLaunchKernelGGL(lfc_total_kernel, dim3(unsigned(nslots)), dim3(kLfcBins), 0, c->stream2, b);
    HIPCHK(c, hipGetLastError());
    // the fast-LFC select reads the leaf counters and the LFC tables only
    // (lfc_fast): it waits for the roll-up only when the replication wrote stats
    if (replicated) HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev[4], 0));
    b.wave_lds = lfc_wave_lds;
    const SelSlot* sel = b.sel_slots;
    b.sel_slots = nullptr;  // fast-LFC evals keep no lists or overlay
    hipLaunchKernelGGL(select_kernel, dim3(unsigned((nfast + waves - 1) / waves)), dim3(64 * waves),
                       size_t(waves) * size_t(lfc_wave_lds), c->stream2, s, b, d_fast, nfast);
    b.sel_slots = sel;
    HIPCHK(c, hipGetLastError());
    if (emit_main) {
      HIPCHK(c, hipEventRecord(c->evl[3], c->stream2));
    } else {
      hipLaunchKernelGGL(lfc_emit_kernel, dim3(unsigned(emit_grid)), dim3(256), 0, c->stream2, s, b);
      HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(c->evl[1], c->stream2));
    // the branch's result headers come back on its own stream: the host
    // waits for both streams instead of the main stream waiting for this one
    // (a cross-stream hand-off costs ~17 us of device time, sync_cost.hip)
    HIPCHK(c, hipMemcpyAsync(c->h_res2.p, d_out, n * sizeof(kueue_tas_eval_out), hipMemcpyDeviceToHost, c->stream2));
  }
  if (nfast && emit_main) {  // the emit after the BestFit select on the main stream (its chunk re-reads
    // stall the descents beside it); the fast select's items from stream2
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->evl[3], 0));
    hipLaunchKernelGGL(lfc_emit_kernel, dim3(unsigned(emit_grid)), dim3(256), 0, c->stream, s, b);
    HIPCHK(c, hipGetLastError());
  }
  trace(15);
  if (stats_branch) HIPCHK(c, hipStreamWaitEvent(c->stream, c->evs[1], 0));  // join the ExclusionStats branch
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev[7], c->stream));
  HIPCHK(c, hipMemcpyAsync(c->h_res.p, c->d_res.p, res_bytes, hipMemcpyDeviceToHost, c->stream));
  lap(2);
  trace(17);
  // the speculative class merge verified exactly while the device runs
  bool merge_ok = true;
  if (!c->exact_merge) {
    const std::vector<int32_t>& cls_rep = c->cls_rep;
    for (size_t t = 0; t < nparts && merge_ok; t++) {
      const PartClasses& pc = c->part_cls[t];
      for (size_t j = 0; j < pc.rep.size() && merge_ok; j++) {
        const int32_t r = cls_rep[size_t(c->part_map[c->part_base[t] + j])];
        if (r != pc.rep[j]) merge_ok = same_sig(hev[pc.rep[j]], hev[r]) && same_mask(hev[pc.rep[j]], hev[r]);
      }
    }
    for (size_t k = 0; k < cls_rep.size() && merge_ok; k++) {
      const int32_t g = c->sig_rep[size_t(c->cls_sig[k])];
      if (g != cls_rep[k]) merge_ok = same_sig(hev[cls_rep[k]], hev[g]);
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (nfast) {
    HIPCHK(c, hipStreamSynchronize(c->stream2));
    const int32_t* hf = reinterpret_cast<const int32_t*>(hs + o_fast);
    for (int k = 0; k < nfast; k++) c->res_out_h[hf[k]] = c->h_res2.p[hf[k]];
  }
  if (!merge_ok) {  // a 64-bit class hash collision: the caller re-runs the chunk with the exact merge
    c->exact_merge = true;
    c->merge_reruns++;
    return 2;
  }
  if (!c->scratch_full && c->scratch_bounded) {  // a bounded list overflowed: re-run with unbounded lists
    const int32_t* hb = reinterpret_cast<const int32_t*>(hs + o_bf);
    const SelSlot* hq = reinterpret_cast<const SelSlot*>(hs + o_sel);
    for (int k = 0; k < nbf; k++) {
      const kueue_tas_eval_out& o = c->res_out_h[hb[k]];
      if ((o.status == KUEUE_TAS_ST_INTERNAL && o.num_workers + o.num_leaders <= entry_cap && hq[k].lcap < full_lcap) ||
          c->force_scratch_rerun) {
        c->scratch_full = true;
        c->scratch_reruns++;
        return 2;
      }
    }
  }
  lap(3);
  trace(18);
  int32_t need = 0;
  for (size_t i = 0; i < n; i++) need = std::max(need, c->res_out_h[i].num_workers + c->res_out_h[i].num_leaders);
  if (need > entry_cap) return 1;  // caller grows entry_cap and re-runs this chunk
  const int64_t base_pairs = int64_t(c->ent_used / 2);
  for (size_t i = 0; i <= n; i++) offsets[i] = base_pairs + int64_t(i) * entry_cap;  // strided regions
  for (size_t i = 0; i < n; i++)
    c->ent_count.push_back(std::min(c->res_out_h[i].num_workers + c->res_out_h[i].num_leaders, entry_cap));
  c->ent_used += size_t(n) * size_t(entry_cap) * 2;
  c->ent_stride = entry_cap;
  lap(4);
  trace(19);
  memcpy(out, c->res_out_h, n * sizeof(kueue_tas_eval_out));
  {  // nodeSelector / affinity exclusions: counted beside select (stream3), read from the stats region after the join
    const int32_t* sel = c->res_stats_h + n * nt + n * size_t(s.R);
    for (size_t i = 0; i < n; i++) {
      out[i].excl_selector = sel[i];
      out[i].excl_affinity = sel[n + i];
      out[i].excl_topology = sel[2 * n + i];
    }
  }
  if (KTAS_PROFILE) {
    const size_t base = c->last_prof.size();
    c->last_prof.resize(base + n * P_NCAT);
    HIPCHK(c, hipMemcpy(c->last_prof.data() + base, c->d_prof.p, n * P_NCAT * 4, hipMemcpyDeviceToHost));
    c->last_fprof.resize(size_t(1) << 18);
    HIPCHK(c, hipMemcpy(c->last_fprof.data(), c->d_fprof.p, (size_t(1) << 18) * 4, hipMemcpyDeviceToHost));
  }
  for (size_t i = 0; i < n; i++) {
    c->last_ticks.push_back(c->res_out_h[i].reserved[0]);
    c->last_ticks.push_back(c->res_out_h[i].reserved[1]);
  }
  if (taint_counts && nt) memcpy(taint_counts, c->res_stats_h, n * nt * 4);
  if (res_counts && s.R) memcpy(res_counts, c->res_stats_h + n * nt, n * size_t(s.R) * 4);
  float st[KUEUE_TAS_NUM_STAGES] = {};
  if (!c->stage_timing) {  // only the fill bracket (ev1 -> ev2) was recorded
    (void)hipEventElapsedTime(&st[0], c->ev[1], c->ev[2]);
    for (int k = 0; k < KUEUE_TAS_NUM_STAGES; k++) stage_ms[k] += st[k];
    ms[0] += st[0];
    lap(5);
    return KUEUE_TAS_OK;
  }
  for (int k = 0; k < 6; k++) (void)hipEventElapsedTime(&st[k], c->ev[k + 1], c->ev[k + 2]);
  const float partials = st[3];  // ev4 -> ev5: leaf partials; stage [3] reports the concurrent fast-LFC branch
  st[3] = 0.f;
  if (nfast) (void)hipEventElapsedTime(&st[3], c->evl[0], c->evl[1]);
  if (b.nstat > 0) (void)hipEventElapsedTime(&st[2], c->evs[0], c->evs[1]);  // the concurrent stats branch
  (void)hipEventElapsedTime(&st[6], c->ev[0], c->ev[7]);
  if (nfast) {  // the fast-LFC branch may end after the main stream (its results come back on its own stream)
    float tl = 0.f;
    (void)hipEventElapsedTime(&tl, c->ev[0], c->evl[1]);
    st[6] = std::max(st[6], tl);
  }
  for (int k = 0; k < KUEUE_TAS_NUM_STAGES; k++) stage_ms[k] += st[k];
  ms[0] += st[0];                    // fill (+ exclusion stats reduce)
  ms[1] += st[1] + st[2];            // roll-up + replication
  ms[2] += partials + st[4] + st[5]; // leaf partials + select + join with the fast-LFC branch
  ms[3] += st[6];
  lap(5);
  return KUEUE_TAS_OK;
}

int kueue_tas_eval_batch(kueue_tas_ctx* c, const kueue_tas_eval_req* reqs, size_t n, const int32_t* taint_table,
                         size_t taint_table_len, int32_t num_taints, const kueue_tas_assumed* assumed,
                         size_t num_assumed, const kueue_tas_affinity_req* affinity, size_t num_affinity,
                         const int32_t* affinity_values, size_t num_affinity_values, kueue_tas_eval_out* out,
                         int64_t* entry_offsets, int32_t* entries, size_t entries_capacity, int32_t* taint_counts,
                         int32_t* res_counts) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (n && !reqs) return fail(c, KUEUE_TAS_EINVAL, "null requests");
  std::vector<const kueue_tas_eval_req*>& ptrs = c->req_ptrs;
  ptrs.resize(n);
  for (size_t i = 0; i < n; i++) ptrs[i] = reqs + i;
  return kueue_tas_eval_batch_ptrs(c, ptrs.data(), n, taint_table, taint_table_len, num_taints, assumed, num_assumed,
                                   affinity, num_affinity, affinity_values, num_affinity_values, out, entry_offsets,
                                   entries, entries_capacity, taint_counts, res_counts);
}

int kueue_tas_eval_batch_ptrs(kueue_tas_ctx* c, const kueue_tas_eval_req* const* reqs, size_t n,
                              const int32_t* taint_table, size_t taint_table_len, int32_t num_taints,
                              const kueue_tas_assumed* assumed, size_t num_assumed,
                              const kueue_tas_affinity_req* affinity, size_t num_affinity,
                              const int32_t* affinity_values, size_t num_affinity_values, kueue_tas_eval_out* out,
                              int64_t* entry_offsets, int32_t* entries, size_t entries_capacity, int32_t* taint_counts,
                              int32_t* res_counts) {
  // g_select_snap is one per device: batches of different contexts must not interleave
  static std::mutex select_snap_mu;
  std::lock_guard<std::mutex> select_snap_lock(select_snap_mu);
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  HIPCHK(c, hipSetDevice(c->device));
  float ms[4] = {0, 0, 0, 0};
  float stage_ms[KUEUE_TAS_NUM_STAGES] = {};
  c->ent_used = 0;
  c->ent_count.clear();
  c->last_ticks.clear();
  c->last_prof.clear();
  for (auto& v : c->last_stats) v = 0;
  c->last_alias_fills = 0;
  for (auto& v : c->host_ms) v = 0;
  c->fill_paths = 0;
  const size_t chunk = size_t(c->max_batch);
  std::vector<int64_t> off;
  entry_offsets[0] = 0;
  for (size_t i0 = 0; i0 < n; i0 += chunk) {
    size_t m = std::min(chunk, n - i0);
    off.assign(m + 1, 0);
    c->chunk_base = i0;
    for (;;) {
      size_t keep = c->ent_used;
      int rc = eval_chunk(c, reqs + i0, m, taint_table, taint_table_len, num_taints, assumed, num_assumed, affinity,
                          num_affinity, affinity_values, num_affinity_values, out + i0,
                          off.data(), taint_counts ? taint_counts + i0 * size_t(std::max(num_taints, 0)) : nullptr,
                          res_counts ? res_counts + i0 * size_t(c->snap.R) : nullptr, ms, stage_ms);
      if (rc == 2) {  // a class hash collision (re-run with the exact merge) or a select list overflow (unbounded lists)
        c->ent_used = keep;
        c->ent_count.resize(i0);
        c->last_ticks.resize(2 * i0);
        c->last_prof.resize(KTAS_PROFILE ? i0 * P_NCAT : 0);
        continue;
      }
      c->exact_merge = false;
      if (rc == 1) {  // an assignment exceeded the per-eval device capacity: grow and re-run
        c->ent_used = keep;
        c->ent_count.resize(i0);
        c->last_ticks.resize(2 * i0);
        c->last_prof.resize(KTAS_PROFILE ? i0 * P_NCAT : 0);
        int32_t need = 0;
        for (size_t i = 0; i < m; i++) need = std::max(need, c->res_out_h[i].num_workers + c->res_out_h[i].num_leaders);
        int cap = c->entry_cap;
        while (cap < need) cap *= 2;
        c->entry_cap = cap;
        continue;
      }
      if (rc) {
        c->scratch_full = false;
        return rc;
      }
      c->scratch_full = false;
      break;
    }
    for (size_t i = 0; i <= m; i++) entry_offsets[i0 + i] = off[i];
  }
  memcpy(c->last_ms, ms, sizeof ms);
  memcpy(c->last_stage_ms, stage_ms, sizeof stage_ms);
  c->ent_strided_off.assign(entry_offsets, entry_offsets + n + 1);
  if (!entries) return KUEUE_TAS_OK;  // strided offsets into kueue_tas_last_entries()
  // packed layout for the caller
  int64_t total = 0;
  for (size_t i = 0; i < n; i++) {
    entry_offsets[i] = total;
    total += c->ent_count[i];
  }
  entry_offsets[n] = total;
  if (size_t(total) > entries_capacity) return fail(c, KUEUE_TAS_EOVERFLOW, "entries buffer too small");
  return kueue_tas_fetch_entries(c, entries, entries_capacity);
}

int kueue_tas_last_counters(kueue_tas_ctx* c, size_t i, int32_t* out, size_t cap) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (!out) return fail(c, KUEUE_TAS_EINVAL, "null argument");
  if (i < c->chunk_base || i >= c->chunk_base + c->chunk_rep.size())
    return fail(c, KUEUE_TAS_EINVAL, "request not in the last device chunk (max_batch)");
  const DevSnap& s = c->snap;
  size_t total = 0;
  for (int l = 0; l < s.L; l++) total += size_t(s.level_size[l]);
  if (cap < 5 * total) return fail(c, KUEUE_TAS_EOVERFLOW, "counters buffer too small");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t k = i - c->chunk_base;
  const int32_t* rep = c->d_counters.p + int64_t(c->ctr_row_off[size_t(c->chunk_rep[k])]) * s.SD;
  const bool leader = c->chunk_leader[k] != 0;
  for (int f = 0; f < 5; f++) {
    // phase 1 writes the leader fields only for leader requests; otherwise
    // they equal state / sliceState and leaderState is 0 (select's Wave::get)
    int src = leader ? f : (f == 2 ? 0 : f == 3 ? 1 : f);
    if (c->chunk_alias[k] && src == 1) src = 0;  // a simple class's sliceState row aliases state
    size_t pos = size_t(f) * total;
    for (int l = 0; l < s.L; l++) {
      const size_t nl = size_t(s.level_size[l]);
      if (!leader && f == 4) std::memset(out + pos, 0, nl * 4);
      else if (nl)
        HIPCHK(c, hipMemcpyAsync(out + pos, rep + int64_t(src) * s.SD + s.level_off[l], nl * 4, hipMemcpyDeviceToHost,
                                 c->stream));
      pos += nl;
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KUEUE_TAS_OK;
}

const int32_t* kueue_tas_last_entries(kueue_tas_ctx* c, size_t* num_pairs) {
  if (!c) return nullptr;
  if (num_pairs) *num_pairs = c->ent_used / 2;
  return c->ent_host;
}

int kueue_tas_snapshot_set_leaf_tags(kueue_tas_ctx* c, const uint64_t* tags, size_t n) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (!c->loaded) return fail(c, KUEUE_TAS_ENOSNAPSHOT, "no snapshot loaded");
  if (!tags) {
    c->leaf_tags_on = false;
    return KUEUE_TAS_OK;
  }
  if (n != size_t(c->snap.N)) return fail(c, KUEUE_TAS_EINVAL, "leaf tags: n must be the snapshot's leaf count");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, c->d_leaf_tags.reserve(std::max<size_t>(n, 1)));
  if (n) HIPCHK(c, hipMemcpyAsync(c->d_leaf_tags.p, tags, n * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->leaf_tags_on = true;
  return KUEUE_TAS_OK;
}

const uint64_t* kueue_tas_last_entry_tags(kueue_tas_ctx* c) {
  return (c && c->leaf_tags_on && c->snap.tag_out) ? c->tag_host : nullptr;
}

int kueue_tas_fetch_entries(kueue_tas_ctx* c, int32_t* entries, size_t entries_capacity) {
  if (!c) return KUEUE_TAS_EINVAL;
  size_t total = 0;
  for (int32_t k : c->ent_count) total += size_t(k);
  if (total > entries_capacity) return fail(c, KUEUE_TAS_EOVERFLOW, "entries buffer too small");
  size_t pos = 0;
  for (size_t i = 0; i < c->ent_count.size(); i++) {
    const size_t k = size_t(c->ent_count[i]);
    if (k) memcpy(entries + 2 * pos, c->ent_host + 2 * size_t(c->ent_strided_off[i]), k * 8);
    pos += k;
  }
  return KUEUE_TAS_OK;
}

int kueue_tas_set_stage_timing(kueue_tas_ctx* c, int32_t on) {
  if (!c) return KUEUE_TAS_EINVAL;
  c->stage_timing = on != 0;
  return KUEUE_TAS_OK;
}

int kueue_tas_last_timings(kueue_tas_ctx* c, float* ms4) {
  if (!c || !ms4) return KUEUE_TAS_EINVAL;
  memcpy(ms4, c->last_ms, sizeof c->last_ms);
  return KUEUE_TAS_OK;
}

int kueue_tas_last_stage_times(kueue_tas_ctx* c, float* ms, int n) {
  if (!c || !ms || n < 0) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < KUEUE_TAS_NUM_STAGES; k++) ms[k] = c->last_stage_ms[k];
  return KUEUE_TAS_OK;
}

int kueue_tas_last_eval_ticks(kueue_tas_ctx* c, int32_t* ticks, size_t n) {
  if (!c || !ticks) return KUEUE_TAS_EINVAL;
  for (size_t i = 0; i < 2 * n; i++) ticks[i] = i < c->last_ticks.size() ? c->last_ticks[i] : 0;
  return KUEUE_TAS_OK;
}

int64_t kueue_tas_last_fill_profile(kueue_tas_ctx* c, int32_t* out, size_t n) {
  if (!c || !out) return 0;
  const size_t k = std::min(n, c->last_fprof.size());
  if (k) memcpy(out, c->last_fprof.data(), k * 4);
  return int64_t(k);
}

int kueue_tas_last_eval_profile(kueue_tas_ctx* c, int32_t* ticks, size_t n) {
  if (!c || !ticks) return KUEUE_TAS_EINVAL;
  for (size_t i = 0; i < n * P_NCAT; i++) ticks[i] = i < c->last_prof.size() ? c->last_prof[i] : 0;
  return KUEUE_TAS_OK;
}

int64_t kueue_tas_merge_reruns(kueue_tas_ctx* c) { return c ? c->merge_reruns : -1; }

int kueue_tas_select_groups(kueue_tas_ctx* c, int64_t* last_groups, int64_t* scratch_reruns) {
  if (!c) return KUEUE_TAS_EINVAL;
  if (last_groups) *last_groups = c->sel_groups.empty() ? 0 : int64_t(c->sel_groups.size()) - 1;
  if (scratch_reruns) *scratch_reruns = c->scratch_reruns;
  return KUEUE_TAS_OK;
}

int kueue_tas_last_host_trace(kueue_tas_ctx* c, double* ms, int n) {  // ms since the chunk's start, [0, 20)
  if (!c || !ms) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < 20; k++) ms[k] = c->trace[k] - c->trace[0];
  return KUEUE_TAS_OK;
}

int kueue_tas_last_host_times(kueue_tas_ctx* c, double* ms, int n) {  // copies min(n, 8)
  if (!c || !ms || n < 0) return KUEUE_TAS_EINVAL;
  for (int k = 0; k < n && k < 8; k++) ms[k] = c->host_ms[k];
  return KUEUE_TAS_OK;
}

uint32_t kueue_tas_last_fill_paths(kueue_tas_ctx* c) { return c ? c->fill_paths : 0u; }

int64_t kueue_tas_last_alias_fills(kueue_tas_ctx* c) { return c ? c->last_alias_fills : 0; }

int kueue_tas_last_stats(kueue_tas_ctx* c, int64_t* stats4) {
  if (!c || !stats4) return KUEUE_TAS_EINVAL;
  memcpy(stats4, c->last_stats, sizeof c->last_stats);
  return KUEUE_TAS_OK;
}

}  // extern "C"
