// tas_internal.h — device-side data structures shared by the HIP kernels and
// the C-ABI glue in tas_device.hip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kueue_tas_debug.h"

namespace ktas {

constexpr int kWave = 64;
constexpr int kMaxLevels = KUEUE_TAS_MAX_LEVELS;
constexpr int kMaxCols = KUEUE_TAS_MAX_COLS;

// One request term: requested column with its value and the exact
// unsigned-division magic for |value| (Granlund–Montgomery / libdivide u64).
struct DevTerm {
  int64_t val;       // request value (Go int64)
  uint64_t magic;    // multiplier (0 when power of two)
  int32_t col;       // resource column
  uint8_t shift;     // post shift
  uint8_t add;       // 1: "add" variant of the decode
  uint8_t pow2;      // 1: |val| is a power of two
  uint8_t neg;       // 1: val < 0
};

// Compiled evaluation (device copy of kueue_tas_eval_req).
struct DevEval {
  uint32_t flags;
  int32_t count;
  int32_t slice_size;
  int32_t requested_level;
  int32_t slice_level;
  int32_t term_begin;     // worker terms [term_begin, term_begin + nreq)
  int32_t nreq;
  int32_t lead_begin;     // leader terms
  int32_t nlead;
  int32_t nsel;
  uint32_t req_mask;
  uint32_t lead_mask;
  int32_t taint_table;
  int32_t assumed_begin;
  int32_t assumed_end;
  int32_t aff_begin;      // required node affinity requirements [aff_begin, aff_end) (KUEUE_TAS_F_AFFINITY)
  int32_t aff_end;
  int32_t dom_begin;      // required replacement domain: leaves [dom_begin, dom_end); dom_begin < 0: none
  int32_t dom_end;
  int32_t sx_begin;       // nodeSelector pairs beyond the inline ones: requirements [sx_begin, sx_end) of aff
  int32_t sx_end;         //   (KUEUE_TAS_F_SELECTOR_EXT; sx_begin < 0: none)
  int32_t num_layers;
  int32_t layer_level[KUEUE_TAS_MAX_LAYERS];
  int32_t layer_size[KUEUE_TAS_MAX_LAYERS];
  int32_t ssal[kMaxLevels];
  int32_t sel_col[KUEUE_TAS_MAX_SELECTORS];
  int32_t sel_val[KUEUE_TAS_MAX_SELECTORS];
};

// Device-resident snapshot (pointers into HBM).
struct DevSnap {
  int32_t L;
  int32_t N;               // leaves
  int32_t R;               // resource columns
  int32_t SD;              // total domains
  int32_t lowest_is_hostname;
  int32_t K;               // label columns
  int32_t level_size[kMaxLevels];
  int32_t level_off[kMaxLevels + 1];   // global domain id offsets
  int32_t child_base[kMaxLevels];      // offset of level l's child_offsets in child_off[]
  const int32_t* child_off;
  const int32_t* id_rank;              // [SD] rank of DomainID string within its level
  const int64_t* free_cap;             // [R][N]
  const int64_t* tas_usage;            // [R][N]
  const uint32_t* free_present;        // [N]
  const uint32_t* usage_present;       // [N]
  const int32_t* taint_profile;        // [N] or null
  const int32_t* label_values;         // [K][N] or null
  const uint8_t* leaf_dead;            // [N] 1: the leaf left the snapshot (kueue_tas_snapshot_set_leaf_live); null: none
  int32_t n_live;                      // leaves in the snapshot (ExclusionStats.TotalNodes)
  // Ragged leaf parents (fan-out <= 64, not uniform): the staged fill's waves
  // each take whole parents — wave slot w covers leaves [x, x + y) of
  // wave_tab[w] — so it rolls the parents up inside the wave (null: none).
  const int2* wave_tab;                // [n_wave_slots]
  int32_t n_wave_slots;
  const int32_t* leaf_parent;          // [N] parent index in level L-2 (with wave_tab or wave_tab2)
  // Ragged leaf parents for fill_pair_kernel (two leaves per lane): slot w
  // covers leaves [x, x + (y & 0xffff)) of wave_tab2[w] — whole parents of at
  // most 128 leaves, or (y >> 16 == 1) one 128-leaf piece of a wider parent,
  // whose parent sums the slots add atomically (wide_parents: those parents'
  // indices in level L-2, zeroed before the fill).  ragged_max_fan: the
  // widest leaf parent.
  const int2* wave_tab2;
  int32_t n_wave_slots2;
  int32_t ragged_max_fan;
  const int32_t* wide_parents;         // [n_wide]
  int32_t n_wide;
  // Entry tags (kueue_tas_snapshot_set_leaf_tags): every emitted entry pair k
  // of the entries region starting at ent_base also stores leaf_tag[leaf] at
  // tag_out[k] (null leaf_tag: off).  Set per batch before the descriptor upload.
  const uint64_t* leaf_tag;            // [N]
  uint64_t* tag_out;                   // [entry pairs] device view of the pinned tag region
  const int32_t* ent_base;             // device view of the pinned entries region
};

// 128-bit lexicographic sort key; lo's low 32 bits hold the domain index in its level.
struct Key {
  uint64_t hi, lo;
};

// Per-(eval, fill block) reductions over the block's leaves, for evals whose
// requested level is the leaf level: findLevelWithFitDomains (:1244-1270) then
// reduces gridDim.x partials instead of every leaf.
struct LeafPartial {
  Key top;      // min sortedDomainsWithLeader key
  Key last;     // max key
  Key lfcfit;   // min key with sliceState >= sliceCount
  Key bfkey;    // min key among st == bfst
  uint32_t bfst;   // min sortable(st) with st >= sliceCount (st: sliceState, or sliceStateWithLeader with a leader)
  int32_t minss;   // min sliceState
  int32_t pad[2];
};

// LeastFreeCapacity leaf tables (one per phase-1 class that has "fast LFC"
// evals: unconstrained, TASProfileMixed, no leader, slice size 1 at the leaf
// level, requested level = leaves).  For those evals sliceState == state at
// the leaves and the sortedDomains order (:1544-1564, LFC) is (value asc,
// leaf index asc), so findLevelWithFitDomains + updateCountsToMinimumGeneric
// reduce to bin counts: chunk histograms of the leaf values.
constexpr int kLfcBins = 128;    // values 0..126 exact; bin 127 counts values >= 127
constexpr int kLfcChunk = 2048;  // leaves per histogram chunk

// Phase-2 result of a fast-LFC greedy eval that the emit kernel expands:
// every leaf with 0 < value < t, then the first m leaves with value t (index
// order), the m-th of which gets rem_last.  t == 0: nothing to expand.
struct LfcJob {
  int32_t t, m, rem_last, pad;
};

// One (eval, chunk) piece of fast-LFC greedy output: base = output position
// of the chunk's first kept leaf, tie0 = rank of its first value-t leaf.
struct LfcItem {
  int32_t eid, chunk, base, tie0;
};

// One BestFit-side select slot's phase-2 buffers within its slot group: the
// list scratch (6 * lcap uint64 at scr_off: four int32 lists, two key
// arrays), the copy-on-write overlay (2 or 5 fields of SD int32 at ov_off)
// and the ownership tags (row tag_idx of SD int32).  lcap bounds the eval's
// candidate lists (kueue_tas_ctx::scratch_bound).
struct SelSlot {
  int64_t scr_off;
  int64_t ov_off;
  int32_t tag_idx;
  int32_t lcap;
};

// Per-batch device buffers.
struct DevBatch {
  const DevEval* evals;
  const DevTerm* terms;
  const int32_t* taint_table;
  const kueue_tas_assumed* assumed;
  const kueue_tas_affinity_req* aff;  // compiled required node affinity (kueue_tas.h)
  const int32_t* aff_vals;            // their sorted value ids
  int32_t n;
  int32_t num_taints;
  int32_t num_profiles;    // taint-profile rows per eval in taint_table
  int32_t nstat;           // kStatFixed + num_taints + R when the staged fill counts ExclusionStats in LDS, else 0
  int32_t nstat_R;         // R (resource columns) for fill_stats_reduce_kernel
  int32_t* fill_stats;     // [nfill][nstat_blocks][nstat] per-block ExclusionStats partials
  int32_t nstat_blocks;    // partial slots per fill position (the widest fill grid of the batch)
  int32_t stats_split;     // 1: the staged fill leaves ExclusionStats to fill_exclusion_kernel (fill_lim)
  int8_t* fill_lim;        // [signature runs][N] limiting resource where the run's signature gives state 0, else -1
  const int32_t* cls_member_off;  // [nfill + 1] class members other than the rep, in fill order (CSR)
  const int32_t* cls_members;     // eval ids
  int32_t rack_fanout;     // the staged fill also rolls up the leaves' parents: > 0 uniform power-of-two
                           // fan-out, -1 ragged (DevSnap::wave_tab), 0 no
  uint64_t* rack_pos;      // [nfill][D_{L-2}] with rack_fanout: bit j = child leaf j has sliceState > 0 (class rows)
  int64_t ctr_sd;          // SD: a class row's field stride (rows at FillEvalParams::ctr_row * SD)
  int32_t* counters;       // one row per phase-1 class in fill order (row = fill position), 1, 2 or 5 fields
  int32_t* taint_counts;   // [n][num_taints]
  int32_t* res_counts;     // [n][R]
  int32_t* sel_counts;     // [n]
  int32_t* aff_counts;     // [n]
  int32_t* dom_counts;     // [n] ExclusionStats.TopologyDomain
  kueue_tas_eval_out* out; // [n]
  int32_t* entries;        // [n][entry_cap][2]
  int32_t entry_cap;
  uint64_t* scratch;       // select lists per BestFit-side slot (SelSlot::scr_off, 6 * lcap uint64 each)
  const struct SelSlot* sel_slots;  // [nbf] each BestFit-side slot's phase-2 buffers (null: the fast-LFC launch)
  int32_t slot_base;       // the launch's first slot (select runs its slots in groups under a memory budget)
  int32_t list_cap;        // LDS sort capacity per wave
  int32_t wave_lds;        // select_kernel's LDS bytes per wave (>= list_cap keys; the launch's dynamic LDS / waves)
  LeafPartial* partials;   // [leaf-level evals][nblk]
  const int32_t* partial_idx; // [n] row of the eval's partials, -1 if none
  int32_t nblk;            // fill blocks per eval (partials per eval)
  const int32_t* fill_ids; // [nfill] evals whose phase 1 is computed (one per distinct phase-1 input)
  int32_t nfill;
  const int32_t* fill_chunks; // [nchunks][2] (start, len) into fill_ids: <= kEvalsPerBlock classes with one base
                              // signature (leader / simulateEmpty flags, assumed usage), request terms may differ
  const struct FillPos* fill_pos;  // [nfill] host-built per-position records (fill_pair_kernel)
  const int32_t* fill_run;    // [nfill] signature run of each fill position: consecutive positions of a chunk
                              // with the same request terms share a run (one CountIn per leaf)
  const int32_t* rep_of;   // [n] counter row (class fill position) whose phase-1 counters the eval reads
  const int32_t* lfc_slot; // [n] fast-LFC table slot, -1 if the eval is not fast LFC
  const int32_t* lfc_rep;  // [lfc_nslots] counter row whose leaf counters the table summarizes
  int32_t lfc_nslots;
  int32_t lfc_nchunks;
  uint32_t* lfc_ch;        // [nslots][nchunks][kLfcBins] per-chunk value counts
  uint32_t* lfc_cp;        // [nslots][nchunks][kLfcBins] exclusive prefix over chunks
  uint32_t* lfc_tot;       // [nslots][kLfcBins]
  uint64_t* lfc_ovs;       // [nslots][nchunks] sum of the values >= kLfcBins - 1
  uint64_t* lfc_ovtot;     // [nslots]
  uint8_t* lfc_u8;         // [nslots][nchunks * kLfcChunk] leaf values min(v, 255) (lfc_hist_kernel -> lfc_emit_kernel)
  int32_t exp_flags;       // experiment knobs (KTAS_EXP_FLAGS; 0 in the product): 1 = lfc_emit skips its stores
  int32_t lfc_fill;        // 1: fill_pair_kernel accumulates the LFC chunk tables and byte rows (no lfc_hist_kernel)
  LfcJob* lfc_jobs;        // [n]
  LfcItem* lfc_items;      // [nfast * nchunks] chunks with greedy output (appended by select)
  int32_t* lfc_nitems;     // [1] number of lfc_items
  int32_t* overlay;        // phase-2 copy-on-write counters per slot (SelSlot::ov_off: 2 or 5 fields of SD)
  int32_t* tags;           // [slots of a group][SD] overlay ownership (== tag_epoch: held)
  int32_t tag_epoch;       // the launch's (one per slot group)
  int32_t* prof;           // [n][8] select phase ticks (profiling build only, else null)
  int32_t* fill_prof;      // [blocks][8] fill_pair_kernel phase stamps (profiling build only, else null)
  int32_t* level_max;      // [nfill][kMaxLevels] max sliceState per level < L-1 of the class row's counters
                           // (level_max_kernel; rows of class reps only), null: not computed
};

}  // namespace ktas
