#!/bin/bash
# select_kernel at issue priority 3: per-eval ticks of the whole C3 batch,
# kernel trace, C3 stage times + oracle check.  Chained, each step limited.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/sel_prio.log 2>&1 || { echo S1_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_prio -o run -- python3 tools/profile_batch.py > gpurun_out/kt_prio.log 2>&1 || { echo K1_FAILED; exit 1; }
timeout -k 10 300 python tools/probe_c3j.py --config C3 --check 1024 > gpurun_out/c3_prio.log 2>&1 || { echo C3_FAILED; exit 1; }
echo rc=0
