#!/bin/bash
# lfc_emit per (chunk, slot): C3 per-eval ticks, kernel trace, stage times +
# whole-batch oracle check, GPU parity tests of the LFC paths.  Chained.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/probe_c3j.py --config C3 --check 1024 > gpurun_out/c3_emit.log 2>&1 || { echo C3_FAILED; exit 1; }
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/sel_emit.log 2>&1 || { echo S1_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_emit -o run -- python3 tools/profile_batch.py > gpurun_out/kt_emit.log 2>&1 || { echo K1_FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_full_size.py -k "not c5" > gpurun_out/gpu_parity_emit.log 2>&1 || { echo PARITY_FAILED; exit 1; }
echo rc=0
