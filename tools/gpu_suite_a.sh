#!/bin/bash
# GPU suite part A: every GPU test except the full-size ones, then smoke.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --ignore=tests/test_full_size.py > gpurun_out/gpu_suite_a.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_suite_a.log; exit 1; }
tail -2 gpurun_out/gpu_suite_a.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log

timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench_a.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_a.json')); print(d['value'], d['ms_per_step'], d['step_ms'], d['stages'], d['roofline']['frac'], d['extras']['c3j']['value'], d['extras']['c3j']['stages_ms'], d['class_merge_reruns'], d['deltas_in_step'])"
echo rc=0
