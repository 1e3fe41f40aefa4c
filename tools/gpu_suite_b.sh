#!/bin/bash
# GPU suite part B: the full-size tests, then the full C3 bench (CPU legs,
# extras) three times (box noise).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_full_size.py -m gpu -x -v --timeout 880 --timeout-method thread > gpurun_out/gpu_suite_b.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_suite_b.log; exit 1; }
tail -2 gpurun_out/gpu_suite_b.log
echo rc=0
