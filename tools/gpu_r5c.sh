#!/bin/bash
# Category fill at 8 waves per SIMD (every block of the C3 grid resident):
# kernel trace, C3 wall + oracle check, pair-fill GPU test.  Each step limited.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_w8 -o run -- python3 tools/profile_batch.py > gpurun_out/prof_w8.log 2>&1 || { echo PROF_FAILED; exit 1; }
timeout -k 10 300 python tools/probe_c3j.py --config C3 --check 1024 > gpurun_out/c3_w8.log 2>&1 || { echo C3_FAILED; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pair_fill.py > gpurun_out/pair_fill_w8.log 2>&1 || { echo PAIR_FAILED; exit 1; }
echo rc=0
