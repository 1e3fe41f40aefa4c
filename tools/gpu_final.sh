#!/bin/bash
# Round-end evidence in one call: GPU tests, the full C3 bench (CPU baseline,
# whole-batch parity, C3J, widened rows), a kernel-trace profile of the
# bench, the PMC passes, the per-eval select profile and the host-stage
# probe.  Each GPU step under its own limit, chained: stop at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$RUN_TESTS" ]; then  # the whole GPU suite takes ~10 min: usually a call of its own
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['stages'], d['roofline']['frac'], d['parity_full_batch'], d['extras']['c3j'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-extras > gpurun_out/prof_bench.json 2> gpurun_out/prof.log || { echo PROF_FAILED; exit 1; }
bash tools/pmc.sh || { echo PMC_FAILED; exit 1; }
timeout -k 10 150 python tools/probe_join.py --reps 3 > gpurun_out/probe_join.log 2>&1 || { echo JOIN_PROBE_FAILED; exit 1; }
timeout -k 10 200 python tools/probe_host.py > gpurun_out/probe_host.log 2>&1 || { echo HOST_PROBE_FAILED; exit 1; }
cat gpurun_out/probe_host.log
echo rc=0
