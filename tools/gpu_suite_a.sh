#!/bin/bash
# GPU suite part A: every GPU test except the full-size ones, then smoke.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --ignore=tests/test_full_size.py > gpurun_out/gpu_suite_a.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_suite_a.log; exit 1; }
tail -2 gpurun_out/gpu_suite_a.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo rc=0
