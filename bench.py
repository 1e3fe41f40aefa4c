#!/usr/bin/env python3
"""TAS placements/sec on MI355X (BASELINE.json metric) — C3: 131,072 nodes.

A step = one nominate batch (pkg/scheduler/scheduler.go:583-619): every rank
evaluates its shard of pending workloads (FindTopologyAssignmentsForWorkload,
pkg/cache/scheduler/clusterqueue_snapshot.go:191) against its replica of the
snapshot resident in HBM, through the C-ABI host layer (request H2D, three
kernel stages, result D2H and decode), then the per-workload result records
are all-gathered over RCCL (N > 1).  Weak scaling: per-rank batch fixed.

    python bench.py [--gpus N] [--steps K] [--warmup W]

Rank 0 prints ONE JSON line.  See DESIGN.md §Measurement for the roofline
bytes and the CPU baseline (the C++ oracle, "port", timed on a bounded sample).
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
    ap.add_argument("--cpu-sample", type=int, default=64, help="workloads timed on the CPU oracle (rank 0)")
    ap.add_argument("--parity-sample", type=int, default=24)
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def fill_algorithmic_bytes(N, n_fill, n_leader, R_used, label_cols, parents=0):
    """Minimum HBM bytes of one fill launch: the SoA snapshot columns the
    batch requests (free + used int64 per requested column, the two presence
    words, taint profile, label ids) once per launch, plus the leaf counters
    written for every eval whose phase 1 runs (one per distinct phase-1 input:
    state + sliceState int32; stateWithLeader, sliceStateWithLeader,
    leaderState for leader evals).  With the fused parent roll-up (`parents`
    leaf parents of uniform power-of-two fan-out) each phase-1 eval also
    writes the parents' state + sliceState and a 64-bit positive-children
    mask (+ the three leader fields)."""
    snap = N * (16 * R_used + 8 + 4 + 4 * label_cols)
    writes = N * (8 * n_fill + 12 * n_leader) + parents * (16 * n_fill + 12 * n_leader)
    return snap + writes


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


def load_traffic(path, config, n_fill):
    """HBM bytes per fill launch from a committed PMC measurement of the same
    workload (tools/pmc.sh -> profiles/), scaled per launch; None if absent."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("config") != config:
        return None
    return d.get("fill_bytes_per_launch")


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist_mod.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = dist_mod

    from kueue_oss_amd import TASFlavorSnapshot, synth
    from kueue_oss_amd.sharding import gather_records, shard_workloads

    gen = synth.CONFIGS[a.config]
    t0 = time.time()
    snap_doc, all_wls = gen(n_workloads=a.batch * world) if a.config != "C1" else gen()
    mine = shard_workloads(all_wls, world, rank)
    gen_s = time.time() - t0

    t0 = time.time()
    snap = TASFlavorSnapshot(snap_doc, device=local_rank if world > 1 else 0)
    snap.compile(mine)
    load_s = time.time() - t0
    N = len(snap_doc["nodes"])

    # ---- parity (untimed, after the timed region so the CPU burn cannot
    # disturb it): product vs CPU oracle on a sample; CPU baseline timing ----
    def cpu_leg():
        parity = None
        cpu = None
        if rank == 0 and not a.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib

            sample = mine[: max(a.parity_sample, a.cpu_sample)]
            got = snap.find_topology_assignments_for_workloads(sample)
            want, secs = oracle_lib.eval_workloads(snap_doc, sample[: a.cpu_sample])
            parity = all(got[i] == want[i] for i in range(len(want)))
            cpu = {"value": round(len(want) / secs, 3), "unit": "placements/s", "cores": 1, "kind": "port",
                   "sample": f"{len(want)} {a.config} workloads x {N} nodes, oracle/tas_oracle.cpp single thread "
                             f"(C++ restatement of the Go path; Go toolchain absent)",
                   "seconds": round(secs, 3)}
            # mode (ii) of BASELINE.md: the batch's independent workloads over host threads
            thr = int(os.environ.get("KTAS_CPU_THREADS", "16"))
            tsample = mine[: 4 * thr]
            _, tsecs = oracle_lib.eval_workloads(snap_doc, tsample, threads=thr)
            model = ""
            try:
                with open("/proc/cpuinfo") as fh:
                    model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
            except OSError:
                pass
            cpu["threaded"] = {"value": round(len(tsample) / tsecs, 3), "threads": thr,
                               "sample": f"{len(tsample)} workloads", "seconds": round(tsecs, 3)}
            cpu["cpu_model"] = model
            cpu["gomaxprocs"] = "n/a (Go toolchain absent)"
            if not parity:
                bad = [i for i in range(len(want)) if got[i] != want[i]]
                print(f"PARITY MISMATCH on workloads {bad[:8]}", file=sys.stderr)
        return parity, cpu

    import torch

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize() if torch.cuda.is_available() else None

    rec = None
    gathered = None

    def step():
        nonlocal rec, gathered
        h = snap.run_compiled()
        if dist is not None:
            # RCCL all-gather of the per-workload result records over xGMI (shards differ in size: padded)
            gathered = gather_records(snap.last_records(len(mine)), world, dist, device=f"cuda:{local_rank}")
        return h

    # the snapshot document and generated workloads are long-lived: keep them
    # out of the collector's scans during the timed loop
    gc.collect()
    gc.freeze()
    for _ in range(a.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    stage_sum = {}
    host_sum = [0.0] * 4
    dev_host_sum = {}
    counts = None
    for _ in range(a.steps):
        step()
        _, counts = snap.last_timings()
        for k, v in snap.last_stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
        host_sum = [x + y for x, y in zip(host_sum, snap.last_profile())]
        for k, v in snap.last_device_host_times().items():
            dev_host_sum[k] = dev_host_sum.get(k, 0.0) + v
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    placements = len(all_wls) * a.steps  # every rank's shard, all steps
    value = placements / dt
    parity, cpu = cpu_leg()

    # ---- widened rows, after the timed region: v1beta2 encoding of the last
    # batch's assignments and the admission re-check + usage update ----
    extras = {}
    if rank == 0:
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
        enc = json.dumps(cands).encode()  # the caller's records, serialized outside the timed call
        snap.preemption_search(pre, enc)
        t0 = time.perf_counter()
        pr = snap.preemption_search(pre, enc)
        pre_ms = (time.perf_counter() - t0) * 1e3
        for c in cands:
            snap.remove_usage(c)
        # device-resident maintenance: 64 non-TAS pod events (add, then delete)
        # replace only the touched leaves instead of rebuilding the snapshot
        evs = [{"namespace": "bench", "name": f"np{k}", "nodeName": f"node-{k % 4}-{k % 16}-{k % 64}-{k % 32}",
                "phase": "Running", "requests": {"cpu": 1000, "memory": 1 << 30}} for k in range(64)]
        t0 = time.perf_counter()
        snap.update_pods(evs)
        snap.update_pods([dict(e, delete=True) for e in evs])
        pod_ms = (time.perf_counter() - t0) / 2 * 1e3
        # 64 in-place node updates (allocatable change), then restored
        import copy
        upd = [copy.deepcopy(snap_doc["nodes"][k * 997 % N]) for k in range(64)]
        for nd in upd:
            nd["allocatable"]["cpu"] = nd["allocatable"].get("cpu", 0) - 1000
        t0 = time.perf_counter()
        rebuilt = snap.update_nodes(upd)
        node_ms = (time.perf_counter() - t0) * 1e3
        snap.update_nodes([copy.deepcopy(snap_doc["nodes"][k * 997 % N]) for k in range(64)])
        extras = {"pod_events_ms_per_64": round(pod_ms, 3),
                  "node_updates_ms_per_64": round(node_ms, 3), "node_updates_rebuilt": rebuilt,
                  "preemption_search_profile_ms": pr["profileMs"],
                  "preemption_search_ms": round(pre_ms, 3), "preemption_candidates": len(cands),
                  "preemption_first_fit": pr["firstFit"], "preemption_fill_back_evals": pr["fillBackEvals"],
                  "v1beta2_encode_ms_per_batch": round(enc_ms, 3),
                  "fits_ms_per_call": round(fits_ms, 3), "fits_records_per_call": min(8, len(recs)),
                  "usage_update_ms_per_call": round(upd_ms, 3)}

    batches, evals, leader_evals = counts
    st = snap.last_stats()
    launches = max(st["fill_launches"], 1)
    per_launch_fill_ms = stage_sum["fill"] / (a.steps * launches)
    R_used = st["staged_cols"] or len({r for w in mine for p in w for r in p["requests"]} | {"pods"})
    label_cols = 1 if any(p.get("nodeSelector") for w in mine for p in w) else 0
    fill_bytes = fill_algorithmic_bytes(N, st["fill_evals"] / launches, min(leader_evals, st["fill_evals"]) / launches,
                                        R_used, label_cols, fused_parents(snap_doc))
    achieved = fill_bytes / (per_launch_fill_ms * 1e-3) / 1e9
    traffic = load_traffic(os.path.join(ROOT, "profiles", "fill_traffic.json"), a.config, st["fill_evals"])
    stages = {k + "_ms": round(v / a.steps, 3) for k, v in stage_sum.items()}
    host = dict(zip(("staging_ms", "eval_calls_ms", "decode_ms", "total_ms"), (round(x / a.steps, 3) for x in host_sum)))
    host["eval_call_detail_ms"] = {k: round(v / a.steps, 3) for k, v in dev_host_sum.items()}
    if rank == 0:
        line = {
            "metric": "TAS placements/sec at 128k nodes (1/2/4/8 GPU); % HBM roofline",
            "value": round(value, 1),
            "unit": "placements/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded generator modelled on test/performance/scheduler/generator)",
            "config": {"workload": f"{a.config}: {N} nodes, {a.batch} pending workloads per GPU per step "
                                   "(50% BestFit required/preferred, 50% LeastFreeCapacity unconstrained; "
                                   "taints + nodeSelector)",
                       "nodes": N, "batch_per_gpu": a.batch, "parallelism": f"dp{world} (replicated snapshot)"},
            "roofline": {"kernel": "fill_leaves_kernel", "bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "bytes_per_launch": int(fill_bytes),
                         "avg_launch_ms": round(per_launch_fill_ms, 4),
                         "per_launch": f"{N} leaves x {st['fill_evals'] // launches} phase-1 evals "
                                       f"({evals // max(batches, 1)} evals, deduplicated), {R_used} columns"},
            "stages": stages,
            "host": host,
            "work": st,
            "cpu_baseline": cpu,
            "parity_sample_ok": parity,
            "extras": extras,
            "setup_s": {"generate": round(gen_s, 2), "snapshot_load_and_compile": round(load_s, 2)},
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    snap.close()


if __name__ == "__main__":
    main()
