#!/usr/bin/env python3
"""TAS placements/sec on MI355X (BASELINE.json metric) — C3: 131,072 nodes.

A step = one nominate batch (pkg/scheduler/scheduler.go:583-619): every rank
evaluates its shard of pending workloads (FindTopologyAssignmentsForWorkload,
pkg/cache/scheduler/clusterqueue_snapshot.go:191) against its replica of the
snapshot resident in HBM, starting from the workloads' TASPodSetRequests:
grouping and the findTopologyAssignment prelude run inside the step
(KUEUE_TAS_RUN_COMPILE), then request H2D, the kernel stages, result D2H and
the TopologyAssignment of every result (Values, Count; KUEUE_TAS_RUN_VALUES).
With N > 1 ranks the full assignments are then all-gathered over RCCL.
Weak scaling: per-rank batch fixed.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]

Rank 0 prints ONE JSON line.  After the timed region (untimed): the
precompiled-request rate, the admission loop (gather, Fits + AddUsage in
order on rank 0, delta broadcast, replicas apply), the whole timed batch
checked against the CPU oracle, the oracle's CPU baseline, the adversarial
C3J variant, and the widened rows.  See DESIGN.md §5.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batch", type=int, default=1024, help="pending workloads per rank per step")
    ap.add_argument("--cpu-sample", type=int, default=64, help="workloads timed on the single-thread CPU oracle")
    ap.add_argument("--parity-threads", type=int, default=16, help="oracle threads for the whole-batch check")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and the whole-batch oracle check")
    ap.add_argument("--no-extras", action="store_true", help="skip the C3J variant and the widened rows")
    return ap.parse_args()


def fill_algorithmic_bytes(N, n_fill, n_leader, R_used, label_cols, parents=0, n_alias=0):
    """Minimum HBM bytes of one fill launch: the SoA snapshot columns the
    batch requests (free + used int64 per requested column, the two presence
    words, taint profile, label ids) once per launch, plus the leaf counters
    written for every eval whose phase 1 runs (one per distinct phase-1 input:
    state int32, sliceState int32 unless the class is simple — `n_alias` of
    them: its sliceState is its state, the row aliases it; stateWithLeader,
    sliceStateWithLeader, leaderState for leader evals).  With the fused
    parent roll-up (`parents` leaf parents of uniform power-of-two fan-out)
    each phase-1 eval also writes the parents' state (+ sliceState) and a
    64-bit positive-children mask (+ the three leader fields)."""
    snap = N * (16 * R_used + 8 + 4 + 4 * label_cols)
    ss_rows = n_fill - n_alias
    writes = N * (4 * n_fill + 4 * ss_rows + 12 * n_leader) + parents * (12 * n_fill + 4 * ss_rows + 12 * n_leader)
    return snap + writes


def survey_8d_bytes(N, R_used, label_cols, W, SD, W_leader=0):
    """SURVEY.md §8(d) algorithmic bytes of fillInCounts + reduce for W
    phase-1 evaluations: B = N*(16*R + 2 + 4*K_sel) + W*SD*8 (+ W_leader*SD*12):
    free + used int64 per requested column, a 2-byte taint-profile id and the
    selector label ids per leaf once, then state + sliceState int32 for every
    domain of every evaluation (the leader fields for leader evaluations).
    W = the launch's phase-1 classes (evaluations with identical phase-1
    inputs share one fill: the per-unit figure times the units one launch
    processes)."""
    return N * (16 * R_used + 2 + 4 * label_cols) + W * SD * 8 + W_leader * SD * 12


def total_domains(doc):
    """Sum of the domains of every level (distinct level-value prefixes)."""
    levels = doc["levels"]
    return sum(len({tuple(n["labels"].get(k) for k in levels[:l + 1]) for n in doc["nodes"]}) for l in range(len(levels)))


def fused_parents(doc):
    """Number of leaf parents the fill rolls up itself (tas_device.hip
    kueue_tas_snapshot_load: uniform power-of-two fan-out <= 64, contiguous in
    leaf order, which the CSR layout gives), 0 when the snapshot does not qualify."""
    levels = doc["levels"]
    if len(levels) < 2:
        return 0
    from collections import Counter

    sizes = set(Counter(tuple(n["labels"].get(l) for l in levels[:-1]) for n in doc["nodes"]).values())
    if len(sizes) != 1:
        return 0
    F = sizes.pop()
    return len(doc["nodes"]) // F if F <= 64 and F & (F - 1) == 0 else 0


def load_traffic(path, config):
    """HBM bytes per fill launch from a committed PMC measurement of the same
    workload (tools/pmc.sh -> profiles/), None if absent."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("config") != config:
        return None, None
    return d.get("fill_bytes_per_launch"), {"file": "profiles/fill_traffic.json", "kernel": d.get("kernel"),
                                            "pmc": d.get("source"), "correction": d.get("correction"),
                                            "note": "committed PMC pass of the same command (tools/pmc.sh), "
                                                    "not measured in this run"}


def pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))]


def roofline_of(snap, doc, wls, steps, stage_sum):
    st = snap.last_stats()
    launches = max(st["fill_launches"], 1)
    per_launch_fill_ms = stage_sum["fill"] / (steps * launches)
    N = len(doc["nodes"])
    R_used = st["staged_cols"] or len({r for w in wls for p in w for r in p["requests"]} | {"pods"})
    label_cols = 1 if any(p.get("nodeSelector") for w in wls for p in w) else 0
    fill_bytes = fill_algorithmic_bytes(N, st["fill_evals"] / launches, min(st["leader_evals"], st["fill_evals"]) / launches,
                                        R_used, label_cols, fused_parents(doc), st.get("alias_fills", 0) / launches)
    W = st["fill_evals"] / launches
    bytes_8d = survey_8d_bytes(N, R_used, label_cols, W, total_domains(doc), min(st["leader_evals"], st["fill_evals"]) / launches)
    achieved = bytes_8d / (per_launch_fill_ms * 1e-3) / 1e9
    st["written_model_bytes"] = int(fill_bytes)  # the fill's own minimum traffic (aliased rows not written)
    return st, bytes_8d, per_launch_fill_ms, achieved, R_used


def _cpulist(path):
    try:
        with open(path) as f:
            txt = f.read().strip()
    except OSError:
        return []
    out = []
    for part in txt.split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def place_host(gpu, local_rank):
    """Pin this rank's main thread to one last-level-cache domain (CCD) on
    the GPU's NUMA node, a distinct one per local rank: the library's host
    pool then pins its workers to the other cores of that L3
    (tas_pool.h near_cpus), so the step's host passes stay within one L3 and
    the ranks of an 8-GPU node do not share cores.  Returns the CPU list (or
    None when the topology is not readable)."""
    try:
        allowed = os.sched_getaffinity(0)
        node = -1
        try:
            import torch

            pr = torch.cuda.get_device_properties(gpu)
            bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
            with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
                node = int(f.read().strip())
        except Exception:  # noqa: BLE001 - no PCI info: any node
            node = -1
        cpus = sorted(allowed if node < 0 else set(_cpulist(f"/sys/devices/system/node/node{node}/cpulist")) & allowed)
        l3s = []
        seen = set()
        for c in cpus:
            if c in seen:
                continue
            dom = [x for x in _cpulist(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") if x in allowed]
            seen.update(dom)
            if len(dom) >= 6:
                l3s.append(dom)
        if not l3s:
            return None
        dom = l3s[local_rank % len(l3s)]
        os.sched_setaffinity(0, dom)
        return dom
    except Exception:  # noqa: BLE001 - placement is an optimization only
        return None


def heartbeat(period=30.0):
    """A progress line on stderr every `period` s (long setup / oracle phases
    of the 1M-node config print nothing else for minutes)."""
    import threading

    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            print(f"[bench] alive {time.time() - t0:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main():
    a = parse()
    heartbeat()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = None
    gpu = local_rank
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # rehearsal knobs for a one-GPU box: every rank on device 0, gloo
        # collectives over host tensors (RCCL needs one GPU per rank)
        backend = os.environ.get("KTAS_BENCH_BACKEND", "nccl")
        if os.environ.get("KTAS_BENCH_SAME_DEVICE"):
            gpu = 0
        if backend == "nccl":
            torch.cuda.set_device(gpu)
            dist_mod.init_process_group("nccl", device_id=torch.device("cuda", gpu))
            device = f"cuda:{gpu}"
        else:
            dist_mod.init_process_group(backend)
            device = "cpu"
        dist = dist_mod

    import numpy as np
    import torch

    cpus_all = os.sched_getaffinity(0)
    placed = place_host(gpu, local_rank) if torch.cuda.is_available() else None
    from kueue_oss_amd import TASFlavorSnapshot, synth
    from kueue_oss_amd.sharding import admit_round, gather_assignments, shard_ids

    gen = synth.CONFIGS[a.config]
    t0 = time.time()
    snap_doc, all_wls = gen(n_workloads=a.batch * world) if a.config != "C1" else gen()
    ids = shard_ids(all_wls, world, rank)
    mine = [all_wls[i] for i in ids]
    gen_s = time.time() - t0

    t0 = time.time()
    snap = TASFlavorSnapshot(snap_doc, device=gpu if world > 1 else 0,
                             host_values=os.environ.get("KTAS_BENCH_HOST_VALUES", "0") == "1")
    snap.compile(all_wls)  # identical resource columns on every replica
    if world > 1:
        snap.set_shard(ids)
    load_s = time.time() - t0
    N = len(snap_doc["nodes"])
    FULL = TASFlavorSnapshot.RUN_COMPILE | TASFlavorSnapshot.RUN_VALUES

    def barrier():
        if dist is not None:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def step(flags=FULL, gather=True):
        snap.run_compiled(flags=flags)
        if dist is not None and gather:
            # RCCL all-gather of every rank's full assignments (quads) over xGMI.
            # The gathered block stays on the device on every rank: the step
            #  ends with the exchange; the admission that consumes it
            # is timed separately (`admission`, which copies it to rank 0's host)
            gather_assignments(snap.last_assignments(), world, dist, device, to_host=False)

    # the snapshot document and generated workloads are long-lived: keep them
    # out of the collector's scans during the timed loop
    gc.collect()
    gc.freeze()
    for _ in range(a.warmup):
        step()
    # the admission deltas of one whole batch (the timed region
    # includes delta application): admitted once untimed, then every timed
    # step applies them alternately negated and again after its evaluation,
    # so steps evaluate on S + D and S in turn (updateTASUsage on the
    # resident snapshot, kueue_tas_host_apply_deltas)
    snap.run_compiled(flags=FULL)
    if dist is not None:
        _, _, step_deltas = admit_round(snap, world, rank, dist, device)
    else:
        _, step_deltas = snap.admit(snap.last_assignments())
    neg_deltas = step_deltas.copy()
    neg_deltas["delta"] = -neg_deltas["delta"]
    plus = [True]  # the snapshot holds S + D

    def timed_step():
        step()
        snap.apply_deltas(neg_deltas if plus[0] else step_deltas)
        plus[0] = not plus[0]

    # timed region: only the fill's event bracket is recorded (the other stage
    # events are instrumentation); its per-launch time over exactly these
    # steps is the roofline's `avg_launch_ms`
    snap.set_stage_timing(False)
    snap.stage_accum(reset=True)
    barrier()
    per_step = [0.0] * a.steps
    clock = time.perf_counter
    t0 = clock()
    for i in range(a.steps):
        ts = clock()
        timed_step()
        per_step[i] = clock() - ts
    barrier()
    dt = time.perf_counter() - t0
    timed_stages, timed_runs, timed_fills = snap.stage_accum(reset=True)
    snap.set_stage_timing(True)
    if plus[0]:
        snap.apply_deltas(neg_deltas)  # back to S for everything below
    per_step = [x * 1e3 for x in per_step]
    # stage / host breakdown from the same step, in untimed repeats (their
    # ctypes getters stay out of the timed loop)
    stage_sum, dev_host_sum, detail_sum = {}, {}, {}
    host_sum = [0.0] * 4
    for _ in range(a.steps):
        step()
        for k, v in snap.last_stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
        host_sum = [x + y for x, y in zip(host_sum, snap.last_profile())]
        for k, v in snap.last_device_host_times().items():
            dev_host_sum[k] = dev_host_sum.get(k, 0.0) + v
        for k, v in snap.last_host_detail().items():
            detail_sum[k] = detail_sum.get(k, 0.0) + v
    barrier()
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    placements = len(all_wls) * a.steps  # every rank's shard, all steps
    value = placements / dt
    st, fill_bytes, per_launch_fill_ms, achieved, R_used = roofline_of(snap, snap_doc, mine, a.steps, stage_sum)
    # the roofline's duration: the fill launches of the timed steps themselves
    timed_fill_ms = timed_stages["fill"] / max(timed_fills, 1)
    achieved_timed = fill_bytes / (timed_fill_ms * 1e-3) / 1e9 if timed_fill_ms > 0 else achieved
    # the step's delta application alone (untimed repeats; pairs keep S)
    ta = time.perf_counter()
    for _ in range(10):
        snap.apply_deltas(step_deltas)
        snap.apply_deltas(neg_deltas)
    barrier()
    apply_ms = (time.perf_counter() - ta) / 20 * 1e3
    # the step's results on S (the timed steps alternate S + D and S)
    step()
    timed_results = snap.last_results() if rank == 0 and not a.no_cpu else None

    # ---- precompiled-request rate (round-1 definition of the step) ----
    pre_steps = max(10, a.steps // 2)
    barrier()
    t1 = time.perf_counter()
    for _ in range(pre_steps):
        step(flags=0, gather=False)
    barrier()
    pre_rate = len(mine) * pre_steps / (time.perf_counter() - t1)

    # ---- admission loop: evaluate, gather, rank 0 admits in order and
    # broadcasts its deltas, replicas apply; then the negated deltas (the
    # workloads finish) restore the snapshot for the next round ----
    rounds = 5
    adm_ms, admitted_n, deltas_n = [], 0, 0
    adm_parts = []
    adm_stats = (-1, -1, -1)
    for _ in range(rounds):
        barrier()
        ta = time.perf_counter()
        snap.run_compiled(flags=FULL)
        tb = time.perf_counter()
        if dist is not None:
            _, admitted, deltas = admit_round(snap, world, rank, dist, device)
        else:
            admitted, deltas = snap.admit(snap.last_assignments())
        barrier()
        adm_ms.append((time.perf_counter() - ta) * 1e3)
        adm_parts.append([(tb - ta) * 1e3, (time.perf_counter() - tb) * 1e3] + list(snap.last_admit_times()))
        if rank == 0:
            adm_stats = snap.last_admit_stats()
        if admitted is not None:
            admitted_n = int(admitted[:, 1].sum())
        deltas_n = len(deltas)
        neg = deltas.copy()
        neg["delta"] = -neg["delta"]
        snap.apply_deltas(neg)

    # ---- whole timed batch vs the CPU oracle; CPU baseline ----
    os.sched_setaffinity(0, cpus_all)  # the CPU legs run on the process's whole CPU set
    parity = cpu = None
    if rank == 0 and not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib

        thr = a.parity_threads
        want, psecs = oracle_lib.eval_workloads(snap_doc, mine, threads=thr)
        bad = [i for i in range(len(want)) if timed_results[i] != want[i]]
        parity = {"ok": not bad, "workloads": len(want), "mismatches": bad[:8], "oracle_threads": thr,
                  "oracle_seconds": round(psecs, 2)}
        if bad:
            print(f"PARITY MISMATCH on workloads {bad[:8]}", file=sys.stderr)
        sample = mine[: a.cpu_sample]
        _, secs = oracle_lib.eval_workloads(snap_doc, sample)
        model = ""
        try:
            with open("/proc/cpuinfo") as fh:
                model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
        except OSError:
            pass
        cpu = {"value": round(len(sample) / secs, 3), "unit": "placements/s", "cores": 1, "kind": "port",
               "sample": f"{len(sample)} {a.config} workloads x {N} nodes, oracle/tas_oracle.cpp single thread "
                         f"(C++ restatement of the Go path; Go toolchain absent)",
               "seconds": round(secs, 3),
               "threaded": {"value": round(len(want) / psecs, 3), "threads": thr,
                            "sample": f"the whole {len(want)}-workload batch", "seconds": round(psecs, 3)},
               "cpu_model": model, "gomaxprocs": "n/a (Go toolchain absent)"}

    extras = {}
    if placed:  # the API rows run where the step ran (the CPU legs had the whole CPU set)
        os.sched_setaffinity(0, placed)
    if rank == 0 and world == 1 and not a.no_extras:
        extras = widened_rows(a, snap, snap_doc, mine, synth)
        extras["c3j"] = c3j_variant(a, synth, TASFlavorSnapshot, FULL)
        if a.config == "C3":
            extras["admission_8192"] = admission_8192(snap, synth, FULL)

    stages = {k + "_ms": round(v / a.steps, 3) for k, v in stage_sum.items()}
    host = dict(zip(("staging_ms", "eval_calls_ms", "decode_ms", "total_ms"), (round(x / a.steps, 3) for x in host_sum)))
    host["eval_call_detail_ms"] = {k: round(v / a.steps, 3) for k, v in dev_host_sum.items()}
    host["staging_detail_ms"] = {k: round(v / a.steps, 3) for k, v in detail_sum.items()}
    traffic, traffic_src = load_traffic(os.path.join(ROOT, "profiles", "fill_traffic.json"), a.config)
    if rank == 0:
        line = {
            "metric": "TAS placements/sec at 128k nodes (1/2/4/8 GPU); % HBM roofline",
            "value": round(value, 1),
            "unit": "placements/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "step_ms": {"median": round(pct(per_step, 0.5), 3), "p10": round(pct(per_step, 0.1), 3),
                        "p90": round(pct(per_step, 0.9), 3), "max": round(max(per_step), 3),
                        "over_1ms": sum(1 for x in per_step if x > 1.0)},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded generator modelled on test/performance/scheduler/generator)",
            "config": {"workload": f"{a.config}: {N} nodes, {a.batch} pending workloads per GPU per step from "
                                   "TASPodSetRequests (grouping + request compile + evaluation + TopologyAssignment "
                                   "values in the step; 50% BestFit required/preferred, 50% LeastFreeCapacity "
                                   "unconstrained; taints + nodeSelector)",
                       "nodes": N, "batch_per_gpu": a.batch, "parallelism": f"dp{world} (replicated snapshot)"},
            "roofline": {"kernel": "fill_pair_kernel" if st.get("fill_paths", 0) & 8192 else "fill_leaves_staged_kernel",
                         "bound": "hbm", "achieved": round(achieved_timed, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved_timed / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src, "bytes_per_launch": int(fill_bytes),
                         "bytes_definition": "SURVEY.md §8(d): N*(16*R + 2 + 4*K_sel) + W*SD*8 (+ W_leader*SD*12), "
                                             "W = the launch's phase-1 classes",
                         "bytes_written_model": st.get("written_model_bytes"),
                         "avg_launch_ms": round(timed_fill_ms, 4),
                         "avg_launch_source": f"HIP events on the fill's stream around each of the {timed_fills} fill "
                                              f"launches of the {timed_runs} timed steps",
                         "avg_launch_ms_stage_profile": round(per_launch_fill_ms, 4),
                         "per_launch": f"{N} leaves x {st['fill_evals'] // max(st['fill_launches'], 1)} phase-1 evals "
                                       f"({st['evals'] // max(st['batches'], 1)} evals, deduplicated), {R_used} columns"},
            "precompiled_rate": {"value": round(pre_rate * world, 1), "unit": "placements/s",
                                 "note": "requests compiled once before timing, no TopologyAssignment values "
                                         "(round-1 step definition), no gather"},
            "deltas_in_step": {"records": int(len(step_deltas)), "apply_ms": round(apply_ms, 4),
                               "note": "every timed step applies one whole-batch "
                               "admission's deltas (alternately negated and again) after its evaluation"},
            "class_merge_reruns": snap.merge_reruns(),
            "admission": {"round_ms_median": round(pct(adm_ms, 0.5), 3), "rounds": rounds,
                          "admitted": admitted_n, "deltas": deltas_n,
                          "device_pass": dict(zip(["window_rounds", "in_order_candidates", "candidates"],
                                                  [int(x) for x in adm_stats])),
                          "parts_ms_median": dict(zip(["evaluate", "gather_admit_broadcast", "admit_host_prep",
                                                       "admit_device", "admit_delta_list"],
                                                      [round(pct([p[k] for p in adm_parts], 0.5), 3)
                                                       for k in range(5)])),
                          "round": "evaluate + all-gather assignments + rank-0 Fits/AddUsage in workload order "
                                   "(order-free candidates in parallel, the rest admit_window_kernel) + delta "
                                   "broadcast + replicas apply"},
            "stages": stages,
            "host": host,
            "work": st,
            "cpu_baseline": cpu,
            "parity_full_batch": parity,
            "extras": extras,
            "setup_s": {"generate": round(gen_s, 2), "snapshot_load_and_compile": round(load_s, 2)},
            "host_placement": {"l3_cpus": placed, "note": "rank's main thread bound to one L3 domain on the "
                               "GPU's NUMA node; the library pins its host pool to that L3's other cores"},
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    snap.close()


def widened_rows(a, snap, snap_doc, mine, synth):
    """§8f rows on the bench snapshot (after the timed region)."""
    import copy

    N = len(snap_doc["nodes"])
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        snap.last_v1beta2(materialize=False)
    enc_ms = (time.perf_counter() - t0) / reps * 1e3
    got = snap.find_topology_assignments_for_workloads(mine[:64])
    recs = [r for w, res in zip(mine[:64], got) for r in synth.usage_records(w, res)]
    t0 = time.perf_counter()
    for _ in range(reps):
        snap.fits(recs[:8])
    fits_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    snap.add_usage(recs[:8])
    snap.remove_usage(recs[:8])
    upd_ms = (time.perf_counter() - t0) / 2 * 1e3
    # batched preemption search (preemption.go:307-345): 16 admitted
    # workloads as candidates, one batch over their prefixes + fill-back
    cands = [synth.usage_records(w, res) for w, res in zip(mine[:64], got)]
    cands = [c for c in cands if c][:16]
    for c in cands:
        snap.add_usage(c)
    pre = [dict(p, count=p.get("count", 1) * 4) for p in mine[0]]
    enc = json.dumps(cands).encode()
    snap.preemption_search(pre, enc)
    t0 = time.perf_counter()
    pr = snap.preemption_search(pre, enc)
    pre_ms = (time.perf_counter() - t0) * 1e3
    for c in cands:
        snap.remove_usage(c)
    # batched partial-admission search (podset_reducer.go:37-86): the first
    # workload whose full counts x 8 do not fit, every PodSet down to 1 pod
    pa = None
    for w in mine[:64]:
        big = [dict(p, count=p.get("count", 1) * 8, minCount=1) for p in w]
        if any(r["reason"] for r in snap.find_topology_assignments_for_flavor(big)):
            snap.partial_admission_search(big)
            t0 = time.perf_counter()
            r = snap.partial_admission_search(big)
            pa = {"ms": round((time.perf_counter() - t0) * 1e3, 3), "found": r["found"], "probes": r["probes"],
                  "evaluations": r["evaluations"], "device_batches": r["batches"],
                  "full_counts": [p["count"] for p in big], "counts": r["counts"]}
            break
    evs = [{"namespace": "bench", "name": f"np{k}", "nodeName": snap_doc["nodes"][k * 977 % N]["name"],
            "phase": "Running", "requests": {"cpu": 1000, "memory": 1 << 30}} for k in range(64)]
    t0 = time.perf_counter()
    snap.update_pods(evs)
    snap.update_pods([dict(e, delete=True) for e in evs])
    pod_ms = (time.perf_counter() - t0) / 2 * 1e3
    upd = [copy.deepcopy(snap_doc["nodes"][k * 997 % N]) for k in range(64)]
    for nd in upd:
        nd["allocatable"]["cpu"] = nd["allocatable"].get("cpu", 0) - 1000
    t0 = time.perf_counter()
    rebuilt = snap.update_nodes(upd)
    node_ms = (time.perf_counter() - t0) * 1e3
    snap.update_nodes([copy.deepcopy(snap_doc["nodes"][k * 997 % N]) for k in range(64)])
    # nodes leaving (NotReady) and returning, in place (kueue_tas_snapshot_set_leaf_live)
    gone = [dict(copy.deepcopy(snap_doc["nodes"][k * 991 % N]), conditions=[{"type": "Ready", "status": "False"}])
            for k in range(64)]
    snap.update_nodes(gone[:1])  # first dead leaf: the device liveness map is created
    snap.update_nodes([copy.deepcopy(snap_doc["nodes"][0])])
    t0 = time.perf_counter()
    left_rebuilt = snap.update_nodes(gone)
    leave_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    back_rebuilt = snap.update_nodes([copy.deepcopy(snap_doc["nodes"][k * 991 % N]) for k in range(64)])
    return_ms = (time.perf_counter() - t0) * 1e3
    # node replacement (findReplacementAssignment) of one assigned node of a placed workload
    rep_ms, rep_ok = None, None
    for w, res in zip(mine[:64], got):
        a0 = res[0].get("assignment")
        if a0 and a0["domains"] and not w[0].get("podSetGroupName"):
            wl = {"unhealthyNodes": [a0["domains"][0]["values"][-1]],
                  "podSetAssignments": [{"name": res[0]["name"], "topologyAssignment": a0}]}
            snap.find_topology_assignments_for_workload(w, wl)
            t0 = time.perf_counter()
            rr = snap.find_topology_assignments_for_workload(w, wl)
            rep_ms = (time.perf_counter() - t0) * 1e3
            rep_ok = not rr[0]["reason"]
            break
    # single-workload latency through the C-ABI (JSON in, JSON out) on the resident snapshot
    lat = []
    for w in mine[:40]:
        t0 = time.perf_counter()
        snap.find_topology_assignments_for_flavor(w)
        lat.append((time.perf_counter() - t0) * 1e3)
    lat.sort()
    # nodes joining (new hosts under existing racks): spliced into the tree in place
    host = "kubernetes.io/hostname"
    joins = []
    for k in range(65):
        nd = copy.deepcopy(snap_doc["nodes"][k * 983 % N])
        nd["name"] = f"{nd['name']}-join{k}"
        nd["labels"][host] = f"{nd['labels'][host]}-join{k}"
        joins.append(nd)
    c0 = snap.snapshot_counters()
    t0 = time.perf_counter()
    add1_rebuilt = snap.update_nodes(joins[:1])
    add1_ms = (time.perf_counter() - t0) * 1e3
    add1_detail = snap.last_update_detail()
    t0 = time.perf_counter()
    add_rebuilt = snap.update_nodes(joins[1:])
    add_ms = (time.perf_counter() - t0) * 1e3
    add_detail = snap.last_update_detail()
    c1 = snap.snapshot_counters()
    return {"single_call_ms": {"median": round(lat[len(lat) // 2], 3), "p90": round(lat[int(len(lat) * 0.9)], 3),
                               "calls": len(lat), "path": "kueue_tas_host_find (JSON) on the C3 snapshot"},
            "node_leave_ms_per_64": round(leave_ms, 3), "node_return_ms_per_64": round(return_ms, 3),
            "node_leave_return_rebuilt": bool(left_rebuilt or back_rebuilt),
            "node_add_ms": round(add1_ms, 3), "node_add_ms_per_64": round(add_ms, 3),
            "node_add_rebuilt": bool(add1_rebuilt or add_rebuilt),
            "node_add_device": {"loads": c1[0] - c0[0], "splices": c1[1] - c0[1]},
            "node_add_detail_ms": {"first": add1_detail, "per_64": add_detail},
            "node_replacement_ms": None if rep_ms is None else round(rep_ms, 3), "node_replacement_ok": rep_ok,
            "pod_events_ms_per_64": round(pod_ms, 3),
            "node_updates_ms_per_64": round(node_ms, 3), "node_updates_rebuilt": rebuilt,
            "preemption_search_profile_ms": pr["profileMs"],
            "preemption_search_ms": round(pre_ms, 3), "preemption_candidates": len(cands),
            "preemption_first_fit": pr["firstFit"], "preemption_fill_back_evals": pr["fillBackEvals"],
            "partial_admission_search": pa,
            "v1beta2_encode_ms_per_batch": round(enc_ms, 3),
            "fits_ms_per_call": round(fits_ms, 3), "fits_records_per_call": min(8, len(recs)),
            "usage_update_ms_per_call": round(upd_ms, 3)}


def admission_8192(snap, synth, flags, n=8 * 1024, reps=4):
    """Rank 0's admission round at 8 GPUs (8 x 1,024 gathered candidates) on
    this snapshot: the C3 generator's first n workloads evaluated in device
    batches of 1,024, then Fits + AddUsage in workload order (kueue_tas_host_admit),
    each repetition's deltas negated afterwards.  Run last: it recompiles the
    snapshot's workload set."""
    import numpy as np

    import torch

    _, wls = synth.config_c3(n_workloads=n)
    snap.compile(wls)
    snap.set_shard(list(range(n)))
    snap.run_compiled(flags=flags)
    quads = snap.last_assignments().reshape(-1)
    # the gathered block as RCCL's all-gather leaves it on rank 0's device:
    # 8 rows [len, quads...], one per rank's 1,024 workloads
    heads = np.flatnonzero(quads[1::4] < 0) * 4
    cuts = [int(heads[k]) for k in range(1024, len(heads), 1024)]
    bounds = [0] + cuts + [quads.size]
    rows = [quads[bounds[k]:bounds[k + 1]] for k in range(len(bounds) - 1)]
    cap = max(r.size for r in rows) + 1
    blk = np.zeros((len(rows), cap), dtype=np.int32)
    for r, row in enumerate(rows):
        blk[r, 0] = row.size
        blk[r, 1:1 + row.size] = row
    block = torch.from_numpy(blk).to(torch.device("cuda", torch.cuda.current_device()))
    lens = [r.size for r in rows]
    torch.cuda.synchronize()

    def rounds(admit):
        times, parts = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            admitted, deltas = admit()
            times.append((time.perf_counter() - t0) * 1e3)
            parts.append(snap.last_admit_times())
            stats = snap.last_admit_stats()
            neg = deltas.copy()
            neg["delta"] = -neg["delta"]
            snap.apply_deltas(neg)
        return times, parts, stats, admitted, deltas

    times, parts, stats, admitted, deltas = rounds(lambda: snap.admit_block(block, lens))
    htimes, hparts, _, hadm, hdel = rounds(lambda: snap.admit(quads))
    same = bool((hadm == admitted).all() and len(hdel) == len(deltas) and (hdel == deltas).all())
    return {"candidates": n, "round_ms_median": round(float(np.median(times)), 3),
            "path": "kueue_tas_host_admit_block on the gathered device block (8 rows)",
            "parts_ms_median": dict(zip(["admit_table", "admit_device", "admit_out"],
                                        [round(float(np.median([p[k] for p in parts])), 3) for k in range(3)])),
            "host_path": {"round_ms_median": round(float(np.median(htimes)), 3),
                          "parts_ms_median": dict(zip(["admit_host_prep", "admit_device", "admit_delta_list"],
                                                      [round(float(np.median([p[k] for p in hparts])), 3)
                                                       for k in range(3)])),
                          "same_verdicts_and_deltas": same},
            "admitted": int(admitted[:, 1].sum()), "deltas": int(len(deltas)),
            "device_pass": dict(zip(["window_rounds", "in_order_candidates", "candidates"], [int(x) for x in stats]))}


def c3j_variant(a, synth, TASFlavorSnapshot, flags, steps=20, sample=32):
    """The adversarial C3 variant: ragged racks and one request signature per
    workload (config_c3j), same step definition; parity on a sample."""
    doc, wls = synth.config_c3j(n_workloads=a.batch)
    snap = TASFlavorSnapshot(doc)
    snap.compile(wls)
    for _ in range(3):
        snap.run_compiled(flags=flags)
    stage_sum = {}
    t0 = time.perf_counter()
    for _ in range(steps):
        snap.run_compiled(flags=flags)
        for k, v in snap.last_stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    dt = time.perf_counter() - t0
    st, fill_bytes, fill_ms, achieved, _ = roofline_of(snap, doc, wls, steps, stage_sum)
    res = snap.last_results()
    ok = None
    if not a.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib

        want, _ = oracle_lib.eval_workloads(doc, wls[:sample], threads=a.parity_threads)
        ok = res[:sample] == want
    snap.close()
    return {"nodes": len(doc["nodes"]), "workloads": len(wls), "value": round(len(wls) * steps / dt, 1),
            "ms_per_step": round(dt / steps * 1e3, 3), "phase1_classes": st["fill_evals"] // max(st["batches"], 1),
            "fill_frac": round(achieved / HBM_PEAK_GBS, 4), "fill_avg_launch_ms": round(fill_ms, 4),
            "stages_ms": {k: round(v / steps, 3) for k, v in stage_sum.items()},
            "parity_sample_ok": ok, "parity_sample": sample}


if __name__ == "__main__":
    main()
