/*
 * kueue_tas.h — C-ABI of the MI355X-native TAS evaluation path.
 *
 * This is the drop-in boundary for Kueue's Topology-Aware Scheduling
 * evaluation (reference: /root/reference/pkg/cache/scheduler/).  A Go cgo shim
 * in the reference's pkg/cache/scheduler binds exactly these
 * entry points; everything here is plain C: fixed-width integers, plain
 * pointers and sizes, caller-owned buffers, 0 = OK / negative = error.
 *
 * Two layers are exported by libkueue_tas.so:
 *
 *  (1) Device layer (kueue_tas_ctx_*, kueue_tas_snapshot_*, kueue_tas_eval_*):
 *      a device-resident TAS snapshot in HBM plus batched evaluation of
 *      compiled PodSet-group requests.  Replaces, per call:
 *        TASFlavorSnapshot.findTopologyAssignment   tas_flavor_snapshot.go:804-999
 *          fillInCounts / fillInCountsHelper        :1568-1719
 *          findLevelWithFitDomains                  :1236-1321
 *          updateCountsToMinimumGeneric (+consume)  :1348-1469
 *          buildAssignment                          :1490-1501
 *        snapshot construction (domain tree)        :160-241, tas_flavor.go:118-138
 *        updateTASUsage (snapshot delta)            :257-293
 *
 *  (2) Host layer (kueue_tas_host_*): the C++ mirror of the Go API
 *      (TASFlavorSnapshot, TASPodSetRequests, TASAssignmentsResult,
 *      FindTopologyAssignmentsForFlavor :519-594 with PodSet groups,
 *      leader/worker split :596-609 and assumedUsage chaining :658-666,
 *      failure strings :1721-1793) driven by JSON documents.  It is what a
 *      Go shim would otherwise do in Go; tests drive it with the fixtures
 *      transcribed from the reference's own table tests.
 *
 * Threading: one ctx per TAS flavor snapshot; calls on one ctx are
 * serialized by the caller (the reference evaluates on the single scheduler
 * goroutine, pkg/scheduler/scheduler.go:286-365).
 */
#ifndef KUEUE_TAS_H_
#define KUEUE_TAS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KUEUE_TAS_ABI_VERSION 5
#define KUEUE_TAS_MAX_LEVELS 16    /* topology_types.go:114 (<=16 levels) */
#define KUEUE_TAS_MAX_COLS 32      /* resource columns per snapshot */
#define KUEUE_TAS_MAX_SELECTORS 8  /* nodeSelector key=value pairs held inline per request (more: KUEUE_TAS_F_SELECTOR_EXT) */
#define KUEUE_TAS_MAX_LAYERS 4     /* podsetSliceRequiredTopologyConstraints */

/* error codes */
#define KUEUE_TAS_OK 0
#define KUEUE_TAS_EINVAL -1
#define KUEUE_TAS_ENOMEM -2
#define KUEUE_TAS_EDEVICE -3
#define KUEUE_TAS_ENOSNAPSHOT -4
#define KUEUE_TAS_EOVERFLOW -5
#define KUEUE_TAS_ELAYOUT -6    /* kueue_tas_admit_block: the block is not in the assignments layout */
#define KUEUE_TAS_EHOSTMEM -7   /* kueue_tas_admit_block: the block is not device memory */

typedef struct kueue_tas_ctx kueue_tas_ctx;

/* ---- snapshot -------------------------------------------------------------
 * Domains of every level are numbered in bytewise-lexicographic order of their
 * levelValues (the tie-break of sortedDomains*, tas_flavor_snapshot.go:1532,
 * :1561, and the output order of buildAssignment :1492).  Children of a domain
 * are therefore contiguous in the next level (CSR).
 */
typedef struct {
  int32_t num_levels;             /* L */
  const int32_t* level_sizes;     /* [L] D_l */
  const int32_t* child_offsets;   /* for l in 0..L-2: D_l+1 offsets into level l+1, concatenated */
  int32_t num_cols;               /* R resource columns, numbered in sorted resource-name order */
  const int64_t* free_capacity;   /* [R][N] allocatable - non-TAS usage (leafDomain.freeCapacity) */
  const int64_t* tas_usage;       /* [R][N] leafDomain.tasUsage (incl. "pods") */
  const uint32_t* free_present;   /* [N] bit c set: column c is a key of freeCapacity */
  const uint32_t* usage_present;  /* [N] bit c set: column c is a key of tasUsage */
  int32_t lowest_is_hostname;     /* isLowestLevelNode (:155): taint/selector filters apply */
  const int32_t* taint_profile;   /* [N] taint-profile id (0..P-1) or NULL */
  int32_t num_label_cols;         /* K dictionary-encoded label columns */
  const int32_t* label_values;    /* [K][N] value id, 0 = label absent; NULL if K == 0 */
  const int32_t* domain_id_rank;  /* [sum D_l] rank of the DomainID string within its level
                                     (multiLayerNotFitMessage tie-break :1768-1769); NULL = index order */
} kueue_tas_snapshot_desc;

/* One snapshot delta record (updateTASUsage :257-265 / Sub on removal). */
typedef struct {
  int32_t leaf;                   /* leaf index */
  int32_t col;                    /* resource column */
  int64_t delta;                  /* added to tas_usage[col][leaf] */
} kueue_tas_delta;

/* ---- one PodSet-group evaluation (findTopologyAssignment) ---------------- */
#define KUEUE_TAS_F_REQUIRED 1u       /* isRequired :1140 */
#define KUEUE_TAS_F_UNCONSTRAINED 2u  /* isUnconstrained :1144 */
#define KUEUE_TAS_F_LFC 4u            /* useLeastFreeCapacityAlgorithm :1328 */
#define KUEUE_TAS_F_SIMULATE_EMPTY 8u /* WithSimulateEmpty :505 */
#define KUEUE_TAS_F_LEADER 16u        /* leaderTasPodSetRequests != nil */
#define KUEUE_TAS_F_MULTILAYER 32u    /* len(multiLayerConstraints) > 0 :873-875 */
#define KUEUE_TAS_F_AFFINITY 64u      /* requirements.affinitySelector != nil :889-897 (hostname leaves) */
#define KUEUE_TAS_F_DOMAIN 128u       /* requiredReplacementDomain != "" (node replacement, :614-678) */
#define KUEUE_TAS_F_SELECTOR_EXT 256u /* nodeSelector pairs beyond the inline sel_col/sel_val (selector_begin/end) */

typedef struct {
  uint32_t flags;
  int32_t count;                  /* workers Count */
  int32_t slice_size;             /* getSliceSizeWithSinglePodAsDefault :1162 */
  int32_t requested_level;        /* requestedLevelIdx */
  int32_t slice_level;            /* sliceLevelIdx */
  int32_t num_req;                /* worker request columns (incl. pods+1), ascending column order */
  int32_t num_leader_req;         /* leader request columns (incl. pods+1) */
  int32_t num_selectors;
  int32_t req_col[KUEUE_TAS_MAX_COLS];
  int64_t req_val[KUEUE_TAS_MAX_COLS];
  int32_t leader_col[KUEUE_TAS_MAX_COLS];
  int64_t leader_val[KUEUE_TAS_MAX_COLS];
  int32_t slice_size_at_level[KUEUE_TAS_MAX_LEVELS]; /* buildSliceSizeAtLevel :1018; 0 = absent */
  int32_t sel_col[KUEUE_TAS_MAX_SELECTORS];          /* label column */
  int32_t sel_val[KUEUE_TAS_MAX_SELECTORS];          /* required value id (-1: value never present) */
  int32_t num_layers;                                /* multi-layer constraints (for the failure message) */
  int32_t layer_level[KUEUE_TAS_MAX_LAYERS];
  int32_t layer_size[KUEUE_TAS_MAX_LAYERS];
  int32_t taint_table;            /* offset into the batch taint table: P entries, excluded taint id or -1 */
  int32_t assumed_begin;          /* [begin,end) into the batch assumed-usage records (sorted by leaf) */
  int32_t assumed_end;
  int32_t affinity_begin;         /* with KUEUE_TAS_F_AFFINITY: [begin,end) into the batch affinity */
  int32_t affinity_end;           /*   requirements; an empty range matches no leaf */
  int32_t domain_begin;           /* with KUEUE_TAS_F_DOMAIN: only leaves [begin, end) take part */
  int32_t domain_end;             /*   (belongsToRequiredDomain :1649-1656); the others count as
                                     ExclusionStats.TopologyDomain (:1613-1617) */
  int32_t selector_begin;         /* with KUEUE_TAS_F_SELECTOR_EXT: the nodeSelector pairs beyond the
                                     num_selectors inline ones, as requirements [begin, end) of the
                                     batch affinity table (col = label column, the required value id in
                                     the values table, negate 0; `term` ignored).  A leaf passes the
                                     nodeSelector when every inline pair and every such requirement
                                     matches (labels.ValidatedSelectorFromSet, selector.go:954-968: one
                                     Equals requirement per key, any number of keys); otherwise it counts
                                     as ExclusionStats.NodeSelector (:1599-1603) */
  int32_t selector_end;
} kueue_tas_eval_req;

/* One compiled requirement of required node affinity
 * (nodeaffinity.NodeSelector, vendor/k8s.io/component-helpers/scheduling/
 * corev1/nodeaffinity/nodeaffinity.go:75-201; labels.Requirement.Matches,
 * vendor/k8s.io/apimachinery/pkg/labels/selector.go:247-294).  A leaf matches
 * the requirement when its id is in values[begin, begin + len) (sorted
 * ascending) XOR negate; the id is the leaf's label value id in column `col`
 * (0 = label absent), or with col == KUEUE_TAS_AFFINITY_LEAF the leaf index
 * itself (matchFields on metadata.name).  Requirements of one
 * nodeSelectorTerm share `term` (ascending within a request): a leaf passes
 * when every requirement of some term matches. */
#define KUEUE_TAS_AFFINITY_LEAF (-1)
typedef struct {
  int32_t term;
  int32_t col;
  int32_t negate;
  int32_t begin;
  int32_t len;
} kueue_tas_affinity_req;

/* assumedUsage overlay record (addAssumedUsage :658-666), subtracted from the
 * remaining capacity of `leaf`; creates the key (presence) like Requests.Sub. */
typedef struct {
  int32_t leaf;
  int32_t col;
  int64_t value;
} kueue_tas_assumed;

#define KUEUE_TAS_ST_OK 0
#define KUEUE_TAS_ST_NO_DOMAINS 1      /* "no topology domains at level: %s" (:1242); a = level */
#define KUEUE_TAS_ST_NOT_FIT 2         /* notFitMessage(a, b, slice_size) (:1721) */
#define KUEUE_TAS_ST_MULTILAYER 3      /* multiLayerNotFitMessage (:1754); ml_fit[] */
#define KUEUE_TAS_ST_INTERNAL 4        /* device-side capacity limit hit (lists/output) */

typedef struct {
  int32_t status;
  int32_t a, b;                   /* message numbers (see status) */
  int32_t fit_level;              /* fitLevelIdx */
  int32_t num_workers;            /* worker (leaf, count) entries written */
  int32_t num_leaders;            /* leader (leaf, count) entries written after the workers */
  int32_t assignment_nil;         /* 1: updateCountsToMinimumGeneric returned nil (:1462) */
  int32_t total_nodes;            /* ExclusionStats (:423-430) */
  int32_t excl_selector;
  int32_t excl_affinity;
  int32_t excl_topology;
  int32_t ml_fit[KUEUE_TAS_MAX_LAYERS];
  int32_t ml_need[KUEUE_TAS_MAX_LAYERS];
  int32_t reserved[2];
} kueue_tas_eval_out;

typedef struct {
  int32_t list_cap;               /* LDS sort capacity per wave (test knob; 0 = default) */
  int32_t max_batch;              /* evaluations per device batch (0 = default 1024) */
  int32_t device;                 /* HIP device ordinal */
  int32_t flags;                  /* KUEUE_TAS_CFG_* */
} kueue_tas_config;
/* host layer: copy the entries through kueue_tas_eval_batch's packed buffer
 * instead of reading the zero-copy view (exercises both ABI paths) */
#define KUEUE_TAS_CFG_PACKED_ENTRIES 1
/* count ExclusionStats inside the fill (the default since round 3; kept
 * for callers that set it) */
#define KUEUE_TAS_CFG_INLINE_STATS 2
/* keep single-run fill chunks on the one-leaf-per-thread staged kernel
 * instead of fill_pair_kernel (test knob: both paths must agree) */
#define KUEUE_TAS_CFG_NO_PAIR_FILL 4
/* admit with the one-wave in-order chain (admit_kernel) instead of the
 * windowed admit_window_kernel (test knob: both must agree) */
#define KUEUE_TAS_CFG_SERIAL_ADMIT 8
/* one-leaf staged fill: ExclusionStats by the concurrent
 * fill_exclusion_kernel branch instead of inside the fill (test knob: both
 * paths must agree) */
#define KUEUE_TAS_CFG_SPLIT_STATS 16
/* roll the upper levels up and take the level maxima in one launch
 * (rollup_top_kernel: the last block of each class does the top levels)
 * instead of per-level launches and level_max_kernel.  Off by default: its
 * per-block device-scope release costs more than the launches it saves on
 * MI355X (C3 0.039 vs 0.028 ms, C3J 0.505 vs 0.087 ms; profiles/r03_lp4) */
#define KUEUE_TAS_CFG_FUSED_TOP 32
/* host layer: build TopologyAssignment Values on the host instead of taking
 * the device's entry tags (kueue_tas_snapshot_set_leaf_tags; test knob: both
 * must agree) */
#define KUEUE_TAS_CFG_HOST_VALUES 64
/* classify every leaf of fill_pair_kernel's single-run chunks per class (the
 * round-4 path) instead of once per leaf category and wave (test knob: both
 * paths must agree) */
#define KUEUE_TAS_CFG_NO_CATEGORY_FILL 128
/* test knob: the speculative merge of the host parts' phase-1 classes takes
 * every class hash as equal, so its exact verification (while the device
 * runs) fails and the chunk re-runs with the exact merge: the collision path
 * must give the same results */
#define KUEUE_TAS_CFG_CLASS_COLLIDE 256
/* fill_pair_kernel accumulates the fast-LFC chunk tables and byte rows
 * (KUEUE_TAS_PATH_LFC_FILL) instead of lfc_hist_kernel re-reading the slot
 * classes' rows; off by default (it lengthens the fill on the main chain by
 * about what it saves the side stream), also KTAS_LFC_IN_FILL=1 */
#define KUEUE_TAS_CFG_LFC_IN_FILL 512

/* ---- device layer -------------------------------------------------------- */
int kueue_tas_abi_version(void);
kueue_tas_ctx* kueue_tas_ctx_create(const kueue_tas_config* cfg);
void kueue_tas_ctx_destroy(kueue_tas_ctx* ctx);
const char* kueue_tas_last_error(kueue_tas_ctx* ctx);

/* Upload (replace) the resident snapshot. */
int kueue_tas_snapshot_load(kueue_tas_ctx* ctx, const kueue_tas_snapshot_desc* desc);
/* Apply a delta list to tas_usage on the device (rank-local replica). */
int kueue_tas_snapshot_apply_deltas(kueue_tas_ctx* ctx, const kueue_tas_delta* deltas, size_t n,
                                    const uint32_t* usage_present_or_null);

/* Replace the free-capacity rows of n leaves (rows [n][R] int64 in column
 * order, free_present [n] presence bitmasks): the device side of a non-TAS
 * pod event (nonTasUsageCache.update/delete, tas_non_tas_pod_cache.go:46-87),
 * whose leaf the host recomputes as allocatable - non-TAS usage
 * (TASFlavorCache.snapshot, tas_flavor.go:124-137) instead of rebuilding the
 * snapshot.  Leaves must be distinct. */
int kueue_tas_snapshot_set_free(kueue_tas_ctx* ctx, const int32_t* leaves, size_t n, const int64_t* rows,
                                const uint32_t* free_present);

/* Replace the taint profile (profiles [n]) and selector label ids
 * (labels [n][K], NULL when the snapshot has no label columns) of n distinct
 * hostname leaves: the device side of an in-place node update
 * (nodesCache.sync, tas_nodes_cache.go:38-50). */
int kueue_tas_snapshot_set_leaf_attrs(kueue_tas_ctx* ctx, const int32_t* leaves, size_t n, const int32_t* profiles,
                                      const int32_t* labels);

/* Take n distinct leaves out of the snapshot (live[i] = 0) or put them back
 * (live[i] = 1) without changing the tree: the device side of a node that
 * leaves (NotReady, cordoned, deleted) or returns (nodesCache.sync,
 * tas_nodes_cache.go:38-50) while its parent keeps another leaf.  A leaf out
 * of the snapshot takes part in no evaluation (zero counts, no
 * ExclusionStats, not in Total nodes) and fits nothing; it keeps its rows, so
 * usage deltas applied meanwhile are there when it returns.  The caller
 * keeps at least one live leaf under every domain (else it reloads);
 * kueue_tas_snapshot_load puts every leaf in. */
int kueue_tas_snapshot_set_leaf_live(kueue_tas_ctx* ctx, const int32_t* leaves, size_t n, const int32_t* live);

/* Evaluate n requests against the resident snapshot.
 *  taint_table:   int32 entries referenced by reqs[i].taint_table (may be NULL if no profiles)
 *  assumed:       overlay records referenced by reqs[i].assumed_begin/end
 *  affinity:      requirements referenced by reqs[i].affinity_begin/end, their
 *                 value ids in affinity_values (both may be NULL when no
 *                 request sets KUEUE_TAS_F_AFFINITY)
 *  out:           [n] result headers
 *  entry_offsets: [n+1] the (leaf, count) int32 pairs of request i are
 *                 entries[2*off[i] .. 2*off[i+1]): workers, then leaders
 *  entries:       packed pairs, capacity `entries_capacity` pairs; NULL: no
 *                 copy — entry_offsets then index (in pairs) the zero-copy
 *                 buffer of kueue_tas_last_entries(), where each request owns
 *                 a region and off[i+1] - off[i] is its capacity, not its
 *                 count (count = out[i].num_workers + out[i].num_leaders)
 *  taint_counts:  [n * num_taints] per-request taint exclusion counts (may be NULL)
 *  res_counts:    [n * num_cols]   per-request resource exclusion counts (may be NULL)
 * Returns KUEUE_TAS_OK; KUEUE_TAS_EOVERFLOW when the packed entries exceed
 * entries_capacity (out/entry_offsets are valid: grow the buffer and call
 * kueue_tas_fetch_entries); or another error. */
int kueue_tas_eval_batch(kueue_tas_ctx* ctx, const kueue_tas_eval_req* reqs, size_t n, const int32_t* taint_table,
                         size_t taint_table_len, int32_t num_taints, const kueue_tas_assumed* assumed,
                         size_t num_assumed, const kueue_tas_affinity_req* affinity, size_t num_affinity,
                         const int32_t* affinity_values, size_t num_affinity_values, kueue_tas_eval_out* out,
                         int64_t* entry_offsets, int32_t* entries, size_t entries_capacity, int32_t* taint_counts,
                         int32_t* res_counts);
/* kueue_tas_eval_batch with the requests given by address: reqs[i] points at
 * request i wherever the caller keeps it (the host layer's compiled PodSet
 * groups), so a batch is assembled without copying the records. */
int kueue_tas_eval_batch_ptrs(kueue_tas_ctx* ctx, const kueue_tas_eval_req* const* reqs, size_t n,
                              const int32_t* taint_table, size_t taint_table_len, int32_t num_taints,
                              const kueue_tas_assumed* assumed, size_t num_assumed,
                              const kueue_tas_affinity_req* affinity, size_t num_affinity,
                              const int32_t* affinity_values, size_t num_affinity_values, kueue_tas_eval_out* out,
                              int64_t* entry_offsets, int32_t* entries, size_t entries_capacity, int32_t* taint_counts,
                              int32_t* res_counts);
/* Phase-1 counters of request i of the last kueue_tas_eval_batch (its
 * fillInCounts + fillInCountsHelper result, tas_flavor_snapshot.go:1568-1719):
 * out[f * S + g] for field f = state, sliceState, stateWithLeader,
 * sliceStateWithLeader, leaderState (:71-84) and domain g in level order
 * (level 0 first, domain index order inside a level), S = sum D_l; cap >= 5 S.
 * Valid for the requests of the batch's last device chunk (all of them when
 * n <= max_batch) until the next call on ctx.  The host layer runs
 * TASBalancedPlacement (tas_balanced_placement.go) over them. */
int kueue_tas_last_counters(kueue_tas_ctx* ctx, size_t i, int32_t* out, size_t cap);
/* Copy the packed entries of the last kueue_tas_eval_batch (after EOVERFLOW). */
int kueue_tas_fetch_entries(kueue_tas_ctx* ctx, int32_t* entries, size_t entries_capacity);
/* Zero-copy view of the packed entries of the last kueue_tas_eval_batch
 * (pinned host memory the device wrote; valid until the next call on ctx).
 * Pass entries = NULL to kueue_tas_eval_batch to skip its copy. */
const int32_t* kueue_tas_last_entries(kueue_tas_ctx* ctx, size_t* num_pairs);

/* Nodes joining the snapshot (nodesCache.sync tas_nodes_cache.go:38-50 ->
 * addNode / initialize tas_flavor_snapshot.go:160-241) without a reload: the
 * leaves keep their bytewise-lexicographic numbering, so the joined leaves
 * move every later leaf; the device gathers its resident leaf columns into
 * the new numbering and takes the joined leaves' rows from the caller.
 *  topo:      the new tree (levels, CSR, DomainID ranks as in
 *             kueue_tas_snapshot_load; its leaf arrays are ignored and may
 *             be NULL); same num_cols, num_label_cols, lowest_is_hostname
 *  leaf_src:  [N_new] the leaf's index before the splice, or -1 for a joined
 *             leaf (whose row is the next of the new_* rows, in leaf order)
 *  new_*:     the joined leaves' rows, [R][num_new] / [num_new] / [K][num_new]
 *  new_leaf_tags: [num_new] the joined leaves' tags when leaf tags are set
 *             (kueue_tas_snapshot_set_leaf_tags): every resident leaf's tag
 *             moves with it; NULL clears the tags
 * Leaves that had left (kueue_tas_snapshot_set_leaf_live) stay out; names
 * must be loaded again before a v1beta2 encode. */
typedef struct {
  const kueue_tas_snapshot_desc* topo;
  const int32_t* leaf_src;
  int32_t num_new;
  const int64_t* new_free_capacity;
  const int64_t* new_tas_usage;
  const uint32_t* new_free_present;
  const uint32_t* new_usage_present;
  const int32_t* new_taint_profile;  /* NULL when the snapshot has no taint profiles */
  const int32_t* new_label_values;   /* NULL when K == 0 */
  const uint64_t* new_leaf_tags;     /* NULL: leaf tags cleared */
} kueue_tas_splice_desc;
int kueue_tas_snapshot_splice(kueue_tas_ctx* ctx, const kueue_tas_splice_desc* d);

/* Per-leaf opaque 64-bit tags that the device copies next to every entry it
 * emits (select_kernel, lfc_emit_kernel).  The host layer passes, per leaf,
 * the address of the leaf's TopologyAssignment Values (its levelValues from
 * the assignment's first level, buildAssignment tas_flavor_snapshot.go:1472-1501),
 * so an assignment's Values come back with its (leaf, count) entries instead
 * of a host pass over every domain; the Go shim can pass
 * leaf indices into its own []string table the same way.  n must be the
 * snapshot's leaf count; tags == NULL turns the copy off.  Kept across
 * batches; kueue_tas_snapshot_load clears it. */
int kueue_tas_snapshot_set_leaf_tags(kueue_tas_ctx* ctx, const uint64_t* tags, size_t n);
/* The tags of the last kueue_tas_eval_batch's entries: element k belongs to
 * entry pair k of kueue_tas_last_entries() (same strided layout, same
 * lifetime); NULL when no leaf tags are set. */
const uint64_t* kueue_tas_last_entry_tags(kueue_tas_ctx* ctx);


/* ---- admission re-check: TASFlavorSnapshot.Fits (tas_flavor_snapshot.go:401-415) ----
 * One record per workload.TopologyDomainRequests (pkg/workload/workload.go:260-269). */
typedef struct {
  int32_t leaf;        /* leaf index; -1: DomainID(values) is not a leaf of the snapshot */
  int32_t count;       /* pods placed in the domain (TopologyDomainRequests.Count) */
  int32_t term_begin;  /* single-pod requests: terms[term_begin, term_begin + num_terms) */
  int32_t num_terms;
} kueue_tas_fits_req;
typedef struct {
  int64_t value;       /* single-pod request value (Go int64) */
  int32_t col;         /* resource column; -1: a resource no leaf has (always absent) */
  int32_t pad;
} kueue_tas_fits_term;
/* fits[i] = 1 when reqs[i].leaf >= 0 and
 * SinglePodRequests.CountIn(freeCapacity - tasUsage of that leaf) >= count
 * (requests.go:174-217, no pods:1 added), else 0.  The reference's Fits is
 * the AND over a workload's records. */
int kueue_tas_fits(kueue_tas_ctx* ctx, const kueue_tas_fits_req* reqs, size_t n, const kueue_tas_fits_term* terms,
                   size_t num_terms, int32_t* fits);

/* ---- admission: the TAS half of Scheduler.processEntry ----------------------
 * (pkg/scheduler/scheduler.go:371-435).  Workload w owns the records
 * reqs[wl_off[w] .. wl_off[w+1]) (its TopologyDomainRequests, terms without
 * pods).  In order, w is admitted (admitted[w] = 1) when every record fits
 * (TASFlavorSnapshot.Fits :401-415) against the snapshot plus the usage of
 * the workloads admitted before it; its usage is then added on the device
 * (updateTASUsage :257-265: single x count per term + pods:count in
 * pods_col; -1: no pods column).  Every term's col must be >= 0. */
int kueue_tas_admit(kueue_tas_ctx* ctx, const kueue_tas_fits_req* reqs, size_t n, const kueue_tas_fits_term* terms,
                    size_t num_terms, const int64_t* wl_off, size_t n_workloads, int32_t pods_col, int32_t* admitted);
/* The same admission from the gathered block on the device (no host round
 * trip of the quads: the all-gather's receive block, rank 0's admission at 8
 * GPUs).  kueue_tas_admit_table first: for each of num_workloads compiled
 * workloads its PodSets ps_base[w] .. ps_base[w + 1], each PodSet's
 * single-pod request terms (begin, n) = ps_terms[2 p], ps_terms[2 p + 1]
 * into terms (ComputeTASNetUsage, flavorassigner.go:94-130).  block: device
 * pointer, world rows of row_words int32 = [len, quads...] with lens[r] the
 * row's len (kueue_tas_host_last_assignments' quads: every workload's header
 * followed by its domain quads, each id once); world <= 16.  Out: the present
 * workloads in ascending id in ids[0 .. *n_workloads), admitted[] their
 * verdicts (cap: KUEUE_TAS_EOVERFLOW when short, nothing admitted), and the
 * applied delta list in kueue_tas_host_admit's order (*deltas valid until the
 * next call).  KUEUE_TAS_ELAYOUT (nothing admitted) when the block is not in
 * that layout or has more than 16 rows, KUEUE_TAS_EHOSTMEM when it is not
 * device memory: the caller admits through the host path. */
/* bytes from device memory of ctx's device to host memory (synchronous) */
int kueue_tas_copy_to_host(kueue_tas_ctx* ctx, void* dst, const void* src, size_t bytes);
int kueue_tas_admit_table(kueue_tas_ctx* ctx, const int32_t* ps_base, int32_t num_workloads, const int32_t* ps_terms,
                          const kueue_tas_fits_term* terms, size_t num_terms);
int kueue_tas_admit_block(kueue_tas_ctx* ctx, const int32_t* block, size_t row_words, const int64_t* lens,
                          int32_t world, int32_t pods_col, int32_t* ids, int32_t* admitted, size_t cap,
                          size_t* n_workloads, const kueue_tas_delta** deltas, size_t* n_deltas);

/* ---- v1beta2 compact TopologyAssignment encoding -------------------------
 * V1Beta2From / singleCompactSliceEncoding (pkg/util/tas/tas_assignment.go:
 * 135-259): one slice per assignment; per level either Universal (all values
 * equal) or Individual {Prefix, Suffix, Roots} with the longest common prefix
 * and suffix of the level's values (prefix cut so the two do not overlap);
 * PodCounts Universal when every count is equal.  The device computes the
 * per-level lengths; Roots[j] = value_j[prefix_len : len_j - suffix_len]. */
typedef struct {
  int32_t universal;   /* 1: every value equals value 0 (Universal) */
  int32_t prefix_len;  /* Individual.Prefix = value0[:prefix_len]; 0: unset */
  int32_t suffix_len;  /* Individual.Suffix = value0[len0 - suffix_len:]; 0: unset */
  int32_t first;       /* string id of value 0 (-1: no domains) */
} kueue_tas_level_enc;

/* Explicit strings: assignment a owns domains [off[a], off[a+1]); domain j's
 * value at level k is string ids[j * num_levels + k] of the table
 * bytes[str_off[id] .. str_off[id+1]); counts[j] its pod count.
 * out[a * num_levels + k] is level k's encoding, same_counts[a] = 1 when
 * every count of assignment a is equal (0 for an empty assignment). */
int kueue_tas_encode_v1beta2(kueue_tas_ctx* ctx, const char* bytes, size_t nbytes, const int64_t* str_off,
                             size_t num_strings, const int32_t* ids, const int32_t* counts, const int64_t* off,
                             size_t n_assign, int32_t num_levels, kueue_tas_level_enc* out, int32_t* same_counts);

/* Resident domain names for the leaf-mode encoder: the own label value of
 * every domain, level by level in domain-index order (level 0 first), as
 * bytes[offsets[i] .. offsets[i+1]), i < sum(level_sizes).  Replaced by the
 * next kueue_tas_snapshot_load (call again after it). */
int kueue_tas_snapshot_load_names(kueue_tas_ctx* ctx, const char* bytes, size_t nbytes, const int64_t* offsets);

/* Leaf mode: assignments as (leaf, count) pairs (kueue_tas_eval_batch's
 * entries layout, pairs[2j], pairs[2j+1]); assignment a owns pairs
 * [off[a], off[a+1]).  Encoding level k is snapshot level first_level + k
 * (the leaf's ancestor there), num_levels = L - first_level; out and
 * same_counts as above, `first` indexing the resident names. */
int kueue_tas_encode_v1beta2_leaves(kueue_tas_ctx* ctx, const int32_t* pairs, const int64_t* off, size_t n_assign,
                                    int32_t first_level, kueue_tas_level_enc* out, int32_t* same_counts);

/* ---- host layer (C++ mirror of the Go API, JSON-driven) ------------------ */
typedef struct kueue_tas_host kueue_tas_host;

/* Build a TASFlavorSnapshot from a JSON case document (nodes, pods, levels,
 * nodeLabels, flavorTolerations, tasUsage, featureGates; schema in
 * tools/extract_goldens.py) and load it to the device. */
kueue_tas_host* kueue_tas_host_create(const char* snapshot_json, const kueue_tas_config* cfg);
void kueue_tas_host_destroy(kueue_tas_host* h);
const char* kueue_tas_host_last_error(kueue_tas_host* h);

/* FindTopologyAssignmentsForFlavor for one workload (podSets JSON array);
 * *out_json = {"results":[{"name","assignment","reason"}]} (free with kueue_tas_free). */
int kueue_tas_host_find(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty, char** out_json);

/* FindTopologyAssignmentsForFlavor with WithWorkload (:511-515, :519-594):
 * workload_json = {"podSets": [...], "unhealthyNodes": [node...],
 * "podSetAssignments": [{"name", "topologyAssignment": internal
 * {"levels","domains":[{"values","count"}]} or null}]}.  With unhealthy nodes
 * every PodSet with an existing assignment is repaired around
 * unhealthyNodes[0] (findReplacementAssignment :614-656: deleteDomain,
 * IsTopologyAssignmentStale, requiredReplacementDomain as a required-domain
 * leaf range (KUEUE_TAS_F_DOMAIN), the slice adjustment, mergeTopologyAssignments);
 * results carry the merged assignment.  Without unhealthy nodes it is
 * kueue_tas_host_find. */
int kueue_tas_host_find_workload(kueue_tas_host* h, const char* workload_json, int32_t simulate_empty, char** out_json);

/* Batched nominate: evaluate every workload of {"workloads":[[podset..],..]}
 * independently against the same snapshot (scheduler.go:583-619). */
int kueue_tas_host_find_batch(kueue_tas_host* h, const char* workloads_json, char** out_json);

/* Compile the workloads once; then time repeated device evaluation
 * (kueue_tas_host_run_compiled) without JSON on the timed path. */
int kueue_tas_host_compile(kueue_tas_host* h, const char* workloads_json);
int kueue_tas_host_run_compiled(kueue_tas_host* h, uint64_t* result_hash);
/* run_compiled with options: KUEUE_TAS_RUN_COMPILE groups and compiles every
 * workload's TASPodSetRequests inside the call (FindTopologyAssignmentsForFlavor
 * :528-541 + the findTopologyAssignment prelude :809-897, no cached pass);
 * KUEUE_TAS_RUN_VALUES builds each result's TopologyAssignment domains
 * (Values = the leaf's levelValues[levelIdx:], Count; buildAssignment :1472-1501). */
#define KUEUE_TAS_RUN_COMPILE 1u
#define KUEUE_TAS_RUN_VALUES 2u
int kueue_tas_host_run(kueue_tas_host* h, uint32_t flags, uint64_t* result_hash);

/* Data-parallel batches (one rank per GPU, each with a replica of the
 * snapshot).  Every rank compiles the same global workload list
 * (kueue_tas_host_compile: identical resource columns everywhere) and
 * evaluates only its shard:
 *  set_shard: run_compiled evaluates compiled workloads ids[0..n) (global
 *    indices) in that order;
 *  last_assignments: the results of the last run_compiled as int32 quads,
 *    per workload a header (id, -1, failed 0/1, number of domain quads) then
 *    one (id, podset index, leaf, count) per assigned domain;
 *    *len = quads x 4; KUEUE_TAS_EOVERFLOW when cap is too small;
 *  admit: the TAS half of processEntry over the gathered quads of every rank
 *    (workloads in ascending id): kueue_tas_admit on this replica, the host
 *    mirror updated; admitted = (id, 0/1) pairs (capacity checked first:
 *    KUEUE_TAS_EOVERFLOW before anything is admitted, *n_workloads set);
 *    *n_deltas = length of the applied delta list (updateTASUsage per domain
 *    record), copied out by last_deltas for the other replicas;
 *  apply_deltas: a replica applies those deltas (host mirror + device). */
int kueue_tas_host_set_shard(kueue_tas_host* h, const int32_t* ids, size_t n);
int kueue_tas_host_last_assignments(kueue_tas_host* h, int32_t* buf, size_t cap, size_t* len);
int kueue_tas_host_admit(kueue_tas_host* h, const int32_t* quads, size_t len, int32_t* admitted, size_t admitted_cap,
                         size_t* n_workloads, size_t* n_deltas);
int kueue_tas_host_last_deltas(kueue_tas_host* h, kueue_tas_delta* buf, size_t cap);
int kueue_tas_host_apply_deltas(kueue_tas_host* h, const kueue_tas_delta* deltas, size_t n);
/* admit from the all-gather's device block (kueue_tas_admit_block; block and
 * lens as gather_assignments leaves them): the same verdicts, admitted pairs
 * and delta list as kueue_tas_host_admit over the block's quads; a block
 * outside the assignments layout is copied to the host and admitted there,
 * one in host memory admitted there as it is. */
int kueue_tas_host_admit_block(kueue_tas_host* h, const int32_t* block, size_t row_words, const int64_t* lens,
                               int32_t world, int32_t* admitted, size_t admitted_cap, size_t* n_workloads,
                               size_t* n_deltas);

/* Every result of the last run_compiled as {"results": [[{"name",
 * "assignment","reason"}...] per compiled workload]} (kueue_tas_free). */
int kueue_tas_host_last_results(kueue_tas_host* h, char** out_json);


/* Snapshot usage updates and the admission re-check, JSON records
 * [{"values": [...], "singlePodRequests": {...}, "count": n}, ...]
 * (workload.TASFlavorUsage, pkg/workload/usage.go:24):
 *  update_usage: ClusterQueueSnapshot.AddUsage (add = 1) / RemoveUsage
 *    (add = 0) -> updateTASUsage (clusterqueue_snapshot.go:94-119,
 *    tas_flavor_snapshot.go:257-293): single x count + pods:count per leaf,
 *    applied on the device (records for unknown domains are skipped);
 *  fits: TASFlavorSnapshot.Fits (:401-415), *fits = 0 / 1. */
int kueue_tas_host_update_usage(kueue_tas_host* h, const char* usage_json, int32_t add);

/* v1beta2 wire format (apis/kueue/v1beta2 TopologyAssignment; JSON shapes in
 * oracle/tas_encoding_oracle.cpp):
 *  v1beta2_from: V1Beta2From (tas_assignment.go:251-259) of a JSON array of
 *    internal assignments ({"levels","domains":[{"values","count"}]} or null),
 *    prefix/suffix lengths computed on the device;
 *  internal_from: InternalFrom (:124-133) of a JSON array of v1beta2 values;
 *  find_v1beta2: kueue_tas_host_find whose results carry
 *    "topologyAssignment" in the v1beta2 form (Assignment.ToAPI,
 *    flavorassigner.go:355), encoded from the resident domain names;
 *  v1beta2_last: the v1beta2 form of every result of the last run_compiled
 *    ([[...] per workload]; out_json may be NULL to encode only). */
int kueue_tas_host_v1beta2_from(kueue_tas_host* h, const char* assignments_json, char** out_json);
int kueue_tas_host_internal_from(kueue_tas_host* h, const char* v1beta2_json, char** out_json);
int kueue_tas_host_find_v1beta2(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty, char** out_json);
int kueue_tas_host_v1beta2_last(kueue_tas_host* h, char** out_json);
int kueue_tas_host_fits(kueue_tas_host* h, const char* usage_json, int32_t* fits);

/* Non-TAS pod events on the resident snapshot, in order: JSON array of pods
 * as in the snapshot document ({"namespace","name","nodeName","phase",
 * "requests"}; phase Succeeded/Failed or "delete": true removes the pod),
 * nonTasUsageCache.update/delete (tas_non_tas_pod_cache.go:46-116).  Only
 * the touched leaves are recomputed and replaced on the device
 * (kueue_tas_snapshot_set_free) — no snapshot rebuild. */
int kueue_tas_host_update_pods(kueue_tas_host* h, const char* pods_json);

/* Node events, in order: JSON array of node objects as in the snapshot
 * document (a node with the same name replaces it; not Ready or
 * unschedulable removes it; nodesCache.sync, tas_nodes_cache.go:38-72).
 * Updates that keep a node in place in the topology with an existing taint
 * profile and existing label values (allocatable, taints, labels) are
 * applied to the touched leaves only (kueue_tas_snapshot_set_free +
 * kueue_tas_snapshot_set_leaf_attrs); any other event rebuilds the snapshot
 * from the document and every event since (*rebuilt = 1; may be NULL). */
int kueue_tas_host_update_nodes(kueue_tas_host* h, const char* nodes_json, int32_t* rebuilt);

/* Batched preemption search: the TAS part of preemption's `minimal`
 * (pkg/scheduler/preemption/preemption.go:307-345; workloadFits :614-625 with
 * the quota checks left to the caller).  candidates_json = [[usage records of
 * candidate 0], ...] in candidate order (records as in update_usage; the
 * candidates' usage is in the snapshot).  Every prefix {0..i} is evaluated in
 * ONE device batch as the workload under RemoveUsage of the prefix (a removal
 * overlay, the snapshot itself is not modified); then fillBackWorkloads runs
 * on the first fitting prefix.  *out_json = {"prefixFits":[bool per prefix],
 * "firstFit": i or -1, "targets": [candidate indices in the reference's final
 * order] or null, "fillBackEvals": n}. */
int kueue_tas_host_preemption_search(kueue_tas_host* h, const char* podsets_json, const char* candidates_json,
                                     char** out_json);

/* Batched partial-admission search: PodSetReducer.Search
 * (pkg/scheduler/flavorassigner/podset_reducer.go:37-86, called from
 * Scheduler.getInitialAssignments, pkg/scheduler/scheduler.go:720-739) over
 * the TAS fit of the workload: podsets_json as for kueue_tas_host_find, each
 * PodSet with its "count" and optional "minCount" (absent = count) and
 * "tas": false for a PodSet that only takes part in the count arithmetic
 * (no TAS request).  A probe's counts fit when FindTopologyAssignmentsForWorkload
 * with those counts (count-0 PodSets skipped, tas_flavorassigner.go:52-55)
 * reports no failure; quota and preemption targets are the caller's.
 * sort.Search's decision tree is evaluated `max_batch` probes (<= 0: 1023)
 * per device batch, speculatively, so the probes and the answer are the
 * reference's.  *out_json = {"found": bool, "counts": [per PodSet] or null,
 * "results": [PodSet results of the found counts] or null, "probes": the
 * reference's fits() calls, "evaluations", "batches", "profileMs"}. */
int kueue_tas_host_partial_admission_search(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty,
                                            int32_t max_batch, char** out_json);

/* ---- the snapshot queries of the scheduler's other callers ---------------
 *  has_level: TASFlavorSnapshot.HasLevel (tas_flavor_snapshot.go:1065-1088;
 *    caller tas_flavorassigner.go:195) for a kueue.PodSetTopologyRequest in
 *    its JSON shape (null -> 0): the level key and the slice level key (and,
 *    with TASMultiLayerTopology, every layer's topology) are levels of the
 *    snapshot;
 *  assignment_stale: IsTopologyAssignmentStale (:733-743; callers :621 and
 *    tas_elastic_workloads.go:47) for an internal TopologyAssignment
 *    {"levels","domains":[{"values","count"}]}: *stale = 1 when some
 *    domain's DomainID(values) is not a domain of the snapshot, *domain
 *    (kueue_tas_free; may be NULL) = that domain's values[0], else "";
 *  free_capacity_json: SerializeFreeCapacityPerDomain (:320-355; caller
 *    snapshot.go:113): {leaf DomainID: {"freeCapacity": {resource: quantity},
 *    "tasUsage": {...}}} with keys sorted, as json.Marshal writes it. */
int kueue_tas_host_has_level(kueue_tas_host* h, const char* topology_request_json, int32_t* out);
int kueue_tas_host_assignment_stale(kueue_tas_host* h, const char* assignment_json, int32_t* stale, char** domain);
int kueue_tas_host_free_capacity_json(kueue_tas_host* h, char** out_json);
/* resources.ResourceQuantityString (pkg/resources/requests.go:147-150): the
 * resource.Quantity text of value v of resource `name` (cpu in milli units,
 * memory / ephemeral-storage / hugepages-* BinarySI-canonical, else
 * DecimalSI), NUL-terminated into buf; *len = its length without the NUL;
 * KUEUE_TAS_EOVERFLOW when cap < *len + 1. */
int kueue_tas_resource_quantity_string(const char* name, int64_t value, char* buf, size_t cap, size_t* len);

/* ---- the device layer under a host snapshot ----------------------------------
 * For a binding that keeps its own batching but not its own request compiler:
 *  host_ctx: the device context holding the host snapshot (valid until the
 *    next call that rebuilds it; NULL on error);
 *  leaf_ids: JSON array of the leaves' DomainIDs by leaf index (decodes the
 *    (leaf, count) entries of kueue_tas_eval_batch);
 *  compile_workload: findTopologyAssignment's prelude (:804-897) for every
 *    PodSet group of one workload (podSets JSON array; groups and
 *    leader/workers as FindTopologyAssignmentsForFlavor :528-609 forms them):
 *    reqs[g] is group g's request for kueue_tas_eval_batch with its taint
 *    row at taint_table[g * P ..] (P = *taint_len / *n_groups profiles,
 *    num_taints for eval_batch in *num_taints, may be NULL), its affinity
 *    requirements rebased into affinity / affinity_values, and no assumed
 *    usage (the caller chains groups: addAssumedUsage :658-666);
 *    early_reasons_json (kueue_tas_free; may be NULL) = per group "" or the
 *    failure text of the prelude (the group is not evaluated then).  Sizes
 *    are always set; KUEUE_TAS_EOVERFLOW when a capacity is short.  A
 *    request naming a resource no column holds re-columns (and reloads) the
 *    device snapshot first. */
kueue_tas_ctx* kueue_tas_host_ctx(kueue_tas_host* h);
int kueue_tas_host_leaf_ids(kueue_tas_host* h, char** out_json);
int kueue_tas_host_compile_workload(kueue_tas_host* h, const char* podsets_json, int32_t simulate_empty,
                                    kueue_tas_eval_req* reqs, size_t reqs_cap, size_t* n_groups, int32_t* taint_table,
                                    size_t taint_cap, size_t* taint_len, int32_t* num_taints,
                                    kueue_tas_affinity_req* affinity, size_t affinity_cap, size_t* n_affinity,
                                    int32_t* affinity_values, size_t values_cap, size_t* n_values,
                                    char** early_reasons_json);

void kueue_tas_free(char* p);

/* Content hash of the sources the library was built from (first 16 hex
 * digits of sha256 over kueue_oss_amd/csrc's sources and this header, in the
 * Makefile's order); "unversioned" for builds outside that Makefile. */
const char* kueue_tas_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* KUEUE_TAS_H_ */
