#!/bin/bash
# Quick GPU check: parity tests, then a bench without the CPU leg, then the
# per-eval select profile.  Each GPU step under its own limit; stop at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu --no-extras > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo BENCH_FAILED; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print(d['value'], d['step_ms'], d['stages'], d['roofline']['frac'])"
if [ "$1" = "probe" ]; then
  :
  timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/probe_select.log 2>&1 || { echo PROBE_FAILED; exit 1; }
  tail -12 gpurun_out/probe_select.log
fi
echo rc=0
