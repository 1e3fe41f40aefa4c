#!/bin/bash
# GPU tests, then quick C3 and C3J benches (no CPU leg): stage times.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu_bench.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-extras --config C3J --steps 20 --warmup 3 > gpurun_out/bench_c3j.json 2> gpurun_out/bench_c3j.err || { echo C3J_FAILED; tail -5 gpurun_out/bench_c3j.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c3j.json')); print('C3J', d['value'], d['step_ms'], d['stages'], d['roofline']['frac'])"
echo rc=0
