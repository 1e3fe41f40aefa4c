#!/bin/bash
# One iteration on the GPU box: the GPU tests named in $1 (a -k expression,
# optional), the C3 bench without the CPU legs, the host trace, then a
# kernel-trace profile of a short bench.  Each step under its own limit.
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread -k "$1" > gpurun_out/gpu_iter.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_iter.log; exit 1; }
  tail -2 gpurun_out/gpu_iter.log
fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench_iter.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_iter.json')); print(d['value'], d['ms_per_step'], d['step_ms'], d['stages'], d['host'], d['roofline']['frac'], d['extras']['c3j']['value'], d['extras']['c3j']['parity_sample_ok'])"
timeout -k 10 120 python tools/probe_trace.py C3 > gpurun_out/trace_iter.log 2>&1 && cat gpurun_out/trace_iter.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iter -o run -- python3 bench.py --no-cpu --no-extras --steps 20 --warmup 5 > gpurun_out/prof_iter_bench.json 2> gpurun_out/prof_iter.log || { echo PROF_FAILED; exit 1; }
f=$(find gpurun_out/prof_iter -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -16
echo rc=0
