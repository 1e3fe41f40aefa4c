/*
 * kueue_tas_debug.h — diagnostics of libkueue_tas.so: device stage times,
 * per-eval select ticks and work counters of the last evaluation.  Not part
 * of the drop-in boundary (kueue_tas.h): the bench and the profiling tools
 * read them; a Go binding does not need them.
 */
#ifndef KUEUE_TAS_DEBUG_H_
#define KUEUE_TAS_DEBUG_H_

#include "kueue_tas.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- device layer -------------------------------------------------------- */
/* Per-stage device time of the last kueue_tas_eval_batch (milliseconds, HIP
 * events on the ctx stream): [0] fill (+ exclusion stats reduce), [1] roll-up
 * + exclusion-stats replication, [2] leaf partials + select/descend + join
 * with the fast-LFC branch, [3] total from the request upload to the join. */
int kueue_tas_last_timings(kueue_tas_ctx* ctx, float* ms4);

/* Finer per-stage device time of the last kueue_tas_eval_batch (ms, HIP
 * events, summed over its chunks): [0] fill, [1] roll-up of the remaining
 * levels, [2] ExclusionStats (staged fill: the third-stream branch of counts
 * + reduce, concurrent with [1] and [4]; else the replication), [3] the
 * fast-LFC branch on the second stream (leaf tables, select, emit; runs
 * concurrently with [1], [2], [4]), [4] select of the other evals, [5] wait
 * for the fast-LFC branch, [6] total from the request upload to the join.
 * Copies min(n, 7). */
#define KUEUE_TAS_NUM_STAGES 7
int kueue_tas_last_stage_times(kueue_tas_ctx* ctx, float* ms, int n);

/* Diagnostics: wall-clock time each eval of the last kueue_tas_eval_batch
 * spent in the select kernel (100 MHz ticks), request order: ticks[2i] total,
 * ticks[2i+1] the findLevelWithFitDomains part.  ticks holds 2n values. */
int kueue_tas_last_eval_ticks(kueue_tas_ctx* ctx, int32_t* ticks, size_t n);

/* Diagnostics (profiling build libkueue_tas_prof.so; zeros otherwise): 12
 * inclusive select-phase tick counters per eval of the last batch (LDS sort,
 * threshold walk, child gather, emit, sorted walk, global sort, count
 * update, findLevelWithFitDomains, threshold-walk keys / k-th select / emit,
 * setup).  ticks holds 12n values. */
int kueue_tas_last_eval_profile(kueue_tas_ctx* ctx, int32_t* ticks, size_t n);
/* Profiling build: fill_pair_kernel's per-block phase stamps of the last
 * device batch (100 MHz clock, 8 per block: start, records staged, CountIn,
 * categories, verdicts, class loop done); copies min(n, available) ints and
 * returns that count (0 in the product build). */
int64_t kueue_tas_last_fill_profile(kueue_tas_ctx* ctx, int32_t* out, size_t n);

/* Host wall time inside the last kueue_tas_eval_batch (ms): [0] request
 * compile, [1] phase-1 classes, [2] uploads + launches, [3] wait for the
 * select results, [4] entry packing + D2H, [5] copy-out; within [0]: [6] the
 * validation pass, [7] the records + class-hash pass.  Copies min(n, 8). */
int kueue_tas_last_host_times(kueue_tas_ctx* ctx, double* ms, int n);
/* Host timeline of the last device chunk (ms since its start) at 20 fixed
 * points: validate, staging layout, records, table copies, class merge, class
 * members, chunk order, member lists, classes done, buffers, fill records,
 * upload, fill launches, roll-up launches, LFC branch, select launch, D2H
 * enqueued, synchronized, offsets (tools/probe_host.py --trace). */
int kueue_tas_last_host_trace(kueue_tas_ctx* ctx, double* ms, int n);
/* Device chunks re-run with the exact class merge after the speculative
 * merge's verification failed (a 64-bit class hash collision, or
 * KUEUE_TAS_CFG_CLASS_COLLIDE), over the context's lifetime. */
int64_t kueue_tas_merge_reruns(kueue_tas_ctx* ctx);
/* The BestFit-side select's slot groups in the last chunk (launches whose
 * lists, overlays and tags fit the phase-2 budget; 1 within budget) and the
 * lifetime count of chunks re-run with unbounded select lists after a
 * bounded list overflowed. */
int kueue_tas_select_groups(kueue_tas_ctx* ctx, int64_t* last_groups, int64_t* scratch_reruns);

/* Work counters of the last kueue_tas_eval_batch: [0] evals whose phase 1
 * (fill + roll-up) ran (one per distinct phase-1 input), [1] evals with
 * leaf-level selection partials, [2] fill launches, [3] snapshot columns the
 * fill staged (0: generic kernel). */
int kueue_tas_last_stats(kueue_tas_ctx* ctx, int64_t* stats4);
/* Fill rows of the last eval_batch whose sliceState field aliases their state
 * (simple classes: the row's sliceState is neither stored nor read). */
int64_t kueue_tas_last_alias_fills(kueue_tas_ctx* ctx);
/* Phase-1 kernel variants the last kueue_tas_eval_batch ran (OR of the bits
 * below; tests pin that their inputs reach every variant). */
#define KUEUE_TAS_PATH_STAGED 1u                /* fill_leaves_staged_kernel, taint rows in LDS */
#define KUEUE_TAS_PATH_STAGED_GLOBAL_TAINTS 2u  /* staged fill, > 32 taint profiles: rows from global */
#define KUEUE_TAS_PATH_GENERIC4 4u              /* fill_leaves_kernel<4> (> 8 request columns) */
#define KUEUE_TAS_PATH_GENERIC8 8u
#define KUEUE_TAS_PATH_GENERIC16 16u
#define KUEUE_TAS_PATH_GENERIC32 32u
#define KUEUE_TAS_PATH_STAGED_GL 64u            /* staged fill with global lookups (far selector columns, affinity) */
#define KUEUE_TAS_PATH_GLOBAL_STATS 128u        /* ExclusionStats by global atomics (> 64 stat slots or generic fill) */
#define KUEUE_TAS_PATH_EXCL 256u                /* fill_exclusion_kernel<true> (split stats) */
#define KUEUE_TAS_PATH_EXCL_GLOBAL_TAINTS 512u  /* fill_exclusion_kernel<false> */
#define KUEUE_TAS_PATH_SELECTOR_EXT 1024u       /* nodeSelector pairs beyond the inline ones */
#define KUEUE_TAS_PATH_RAGGED_ROLLUP 2048u      /* staged fill rolls up ragged leaf parents (packed wave slots) */
#define KUEUE_TAS_PATH_UNIFORM_ROLLUP 4096u     /* staged fill rolls up uniform power-of-two leaf parents */
#define KUEUE_TAS_PATH_PAIR 8192u               /* fill_pair_kernel: two adjacent leaves per thread (kPairLP) */
#define KUEUE_TAS_PATH_ENTRY_TAGS 16384u        /* entries emitted with their leaf tags (kueue_tas_snapshot_set_leaf_tags) */
#define KUEUE_TAS_PATH_RAGGED_PAIR 32768u       /* fill_pair_kernel on ragged leaf parents (128-leaf slots, segmented scans) */
#define KUEUE_TAS_PATH_CATEGORY 65536u          /* fill_pair_kernel's single-run chunks classify leaf categories (CAT) */
#define KUEUE_TAS_PATH_LFC_FILL 131072u         /* the fast-LFC chunk tables accumulated by the fill (no lfc_hist_kernel) */
uint32_t kueue_tas_last_fill_paths(kueue_tas_ctx* ctx);
/* Stage events: on (default), every stage of kueue_tas_last_stage_times is
 * timed; off, only the fill bracket is (the other events are pure
 * instrumentation; the ones that order the streams are always recorded). */
int kueue_tas_set_stage_timing(kueue_tas_ctx* ctx, int32_t on);
/* Lifetime counts of successful kueue_tas_snapshot_load and
 * kueue_tas_snapshot_splice calls on ctx (tests pin which one an event took). */
int kueue_tas_snapshot_counters(kueue_tas_ctx* ctx, int64_t* loads, int64_t* splices);
/* Device memory held by ctx now: *total every buffer of the context,
 * *phase2 the per-batch evaluation state (class counter rows, BestFit
 * select lists, overlays and their ownership tags), which scales with the
 * batch. */
int kueue_tas_device_bytes(kueue_tas_ctx* ctx, int64_t* total, int64_t* phase2);
/* Host-mirror support (the host layer's copy of tasUsage follows the device
 * lazily): _usage_mark records the resident usage columns and presence bits
 * as the mirror's state (a device-side shadow copy); _usage_changes lists
 * every (leaf, column) whose usage or presence moved since the mark, with
 * its current value (absolute), then marks again.  The list is owned by the
 * context, valid until its next call. */
int kueue_tas_snapshot_usage_mark(kueue_tas_ctx* ctx);
int kueue_tas_snapshot_usage_changes(kueue_tas_ctx* ctx, const kueue_tas_delta** changes, size_t* n);
/* kueue_tas_snapshot_apply_deltas for deltas the host mirror already took
 * (AddUsage / RemoveUsage through the host layer): the shadow takes them as
 * well, so the mirror needs no diff for them and earlier device-only changes
 * stay pending for the next _usage_changes. */
int kueue_tas_snapshot_apply_deltas_mirrored(kueue_tas_ctx* ctx, const kueue_tas_delta* deltas, size_t n);

/* ---- host layer ---------------------------------------------------------- */
/* Device stage times of the last run (summed over its batches, ms):
 * [0] fill, [1] roll-up, [2] select, [3] total; counts[0] = device batches,
 * counts[1] = evaluations, counts[2] = evaluations with a leader. */
int kueue_tas_host_last_timings(kueue_tas_host* h, float* ms4, int64_t* counts3);
/* kueue_tas_last_stage_times summed over the last run's batches. */
int kueue_tas_host_last_stage_times(kueue_tas_host* h, float* ms, int n);
/* kueue_tas_last_host_times summed over the last run's batches. */
int kueue_tas_host_last_device_host_times(kueue_tas_host* h, double* ms, int n);
/* kueue_tas_last_eval_profile of the last device batch (diagnostics). */
int kueue_tas_host_last_eval_profile(kueue_tas_host* h, int32_t* ticks, size_t n);
/* kueue_tas_last_eval_ticks of the last device batch (diagnostics). */
int kueue_tas_host_last_eval_ticks(kueue_tas_host* h, int32_t* ticks, size_t n);
/* Host wall time of the last run_compiled (ms): [0] request staging,
 * [1] kueue_tas_eval_batch calls (device + transfers), [2] result decode, [3] total. */
int kueue_tas_host_last_profile(kueue_tas_host* h, double* ms4);
/* Finer host wall time of the last run (ms): [0] grouping + column check,
 * [1] request compile (findTopologyAssignment prelude), [2] per-pass request
 * staging (build_pass), [3] TopologyAssignment Values.  Copies min(n, 4). */
int kueue_tas_host_last_host_detail(kueue_tas_host* h, double* ms, int n);
// The last kueue_tas_host_update_nodes call's host time (ms) in n <= 13 slots:
// JSON parse, node events, flush_joins (host mirror merge), splice host rows,
// kueue_tas_snapshot_splice, leaf tags, evaluator reset, pushes, total, then
// flush_joins' parts: host-mirror fold, levels + CSR, leaf arrays, maps + ranks.
int kueue_tas_host_last_update_detail(kueue_tas_host* h, double* ms, int n);
/* kueue_tas_set_stage_timing for the host's snapshot (kept across reloads). */
int kueue_tas_host_set_stage_timing(kueue_tas_host* h, int32_t on);
/* Device stage ms (as kueue_tas_last_stage_times) summed over every
 * kueue_tas_host_run since the last reset, with the number of runs and of
 * fill launches; reset != 0 clears the sums after copying them. */
int kueue_tas_host_stage_accum(kueue_tas_host* h, float* ms, int n, int64_t* runs, int64_t* fill_launches,
                               int32_t reset);
/* Work counters of the last find/run: [0] device batches, [1] evals,
 * [2] leader evals, [3..6] kueue_tas_last_stats summed ([6]: max), [7] OR of
 * kueue_tas_last_fill_paths. */
int kueue_tas_host_last_stats(kueue_tas_host* h, int64_t* stats8);
/* kueue_tas_host_last_stats followed by [8] the fill rows whose sliceState
 * aliases state (kueue_tas_last_alias_fills summed); copies min(n, 9). */
int kueue_tas_host_last_stats_ext(kueue_tas_host* h, int64_t* out, int32_t n);
/* Host wall time of the last kueue_tas_host_admit (ms): [0] record
 * preparation, [1] kueue_tas_admit (uploads, admit_kernel, result copy),
 * [2] delta list. */
int kueue_tas_host_last_admit_times(kueue_tas_host* h, double* ms3);
// The last kueue_tas_admit: rounds of admit_window_kernel, candidates it
// walked in order (the rest were decided in parallel: phase-1 failures and
// order-free admissions), candidates in total; -1 for the serial chain.
int kueue_tas_last_admit_stats(kueue_tas_ctx* ctx, int64_t* out3);
int kueue_tas_host_last_admit_stats(kueue_tas_host* h, int64_t* out3);

#ifdef __cplusplus
}
#endif
#endif /* KUEUE_TAS_DEBUG_H_ */
