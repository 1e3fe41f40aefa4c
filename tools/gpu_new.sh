#!/bin/bash
# The GPU tests named in $1 (a -k expression), then the C3 bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$1" > gpurun_out/gpu_new.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_new.log; exit 1; }
tail -3 gpurun_out/gpu_new.log
timeout -k 10 420 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['stages'], d['host'], d['roofline']['frac'], d['parity_full_batch']['ok'], d['extras']['c3j']['value'], d['extras']['usage_update_ms_per_call'], d['extras']['partial_admission_search'])"
echo rc=0
