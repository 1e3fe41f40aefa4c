#!/bin/bash
# Tests -> quick C3 bench -> PMC passes.  Each GPU step under its own limit,
# chained: stop at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu_bench.sh || exit 1
python -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print(json.dumps(d['admission']))"
bash tools/pmc.sh || { echo PMC_FAILED; exit 1; }
echo rc=0
