#!/bin/bash
# Round-end measurements after the GPU tests (their own call): the full C3
# bench (CPU baseline, whole-batch parity, C3J, widened rows), a kernel-trace
# profile of the bench (csv), the PMC passes, the per-eval select profile and
# the host-stage probe.  Each GPU step under its own limit, chained: stop at
# the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -5 gpurun_out/smoke.log; exit 1; }
timeout -k 10 420 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['stages'], d['roofline']['frac'], d['parity_full_batch']['ok'], d['extras']['c3j']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-extras > gpurun_out/prof_bench.json 2> gpurun_out/prof.log || { echo PROF_FAILED; exit 1; }
bash tools/pmc.sh || { echo PMC_FAILED; exit 1; }
timeout -k 10 200 python tools/probe_host.py > gpurun_out/probe_host.log 2>&1 || { echo HOST_PROBE_FAILED; exit 1; }
timeout -k 10 150 python tools/probe_join.py --reps 3 > gpurun_out/probe_join.log 2>&1 || { echo JOIN_PROBE_FAILED; exit 1; }
echo rc=0
