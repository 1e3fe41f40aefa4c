#!/bin/bash
# Perf pass without the test suite: C3 bench (no CPU leg), the per-eval
# select profile, and a kernel-trace profile of the bench.  Each GPU step
# under its own limit; stop at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --no-extras > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench_quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print(d['value'], d['step_ms'], d['stages'], d['roofline']['frac'], d['host'])"
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/probe_select.log 2>&1 || { echo PROBE_FAILED; exit 1; }
tail -12 gpurun_out/probe_select.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-extras > gpurun_out/prof_bench.json 2> gpurun_out/prof.log || { echo PROF_FAILED; tail -20 gpurun_out/prof.log; exit 1; }
f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -24
echo rc=0
