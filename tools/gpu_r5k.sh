#!/bin/bash
# rollup_tail with int4 level-maximum reads: C3 stage times + oracle check,
# kernel trace, GPU parity tests.  Chained, each step limited.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/probe_c3j.py --config C3 --check 1024 > gpurun_out/c3_tail.log 2>&1 || { echo C3_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_tail -o run -- python3 tools/profile_batch.py > gpurun_out/kt_tail.log 2>&1 || { echo K1_FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_ragged_rollup.py tests/test_pair_fill.py > gpurun_out/gpu_parity_tail.log 2>&1 || { echo PARITY_FAILED; exit 1; }
echo rc=0
