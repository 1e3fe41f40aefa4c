#!/bin/bash
# LFC select latency (batched first-fit scan and work-item bin loads): C3
# stage times + oracle check, kernel trace, emulated-path GPU parity tests of
# the fast-LFC path.  Each step limited, chained.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/probe_c3j.py --config C3 --check 1024 > gpurun_out/c3_lfc.log 2>&1 || { echo C3_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lfc -o run -- python3 tools/profile_batch.py > gpurun_out/prof_lfc.log 2>&1 || { echo PROF_FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/gpu_parity_lfc.log 2>&1 || { echo PARITY_FAILED; exit 1; }
echo rc=0
