#!/bin/bash
# Host-side experiments on the GPU box: pool variants, host thread counts,
# and the per-eval select profile of the C3 batch.
export TMPDIR=/tmp
mkdir -p gpurun_out
(cd tools/micro && g++ -O2 -std=c++17 -pthread pool_bench.cpp -o pool_bench) || exit 1
timeout -k 5 60 tools/micro/pool_bench > gpurun_out/pool_bench.log 2>&1; cat gpurun_out/pool_bench.log
nproc; python -c "import os; print(len(os.sched_getaffinity(0)), 'cpus in affinity')"; lscpu | grep -E "Model name|Thread|Core|Socket|NUMA node\(s\)" 
bash tools/exp_knobs.sh KUEUE_TAS_HOST_THREADS 3 4 6 8 || exit 1
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/probe_select.log 2>&1 || { echo PROBE_FAILED; tail gpurun_out/probe_select.log; exit 1; }
tail -14 gpurun_out/probe_select.log
BF_ONLY=1 timeout -k 10 200 python tools/probe_select.py > gpurun_out/probe_select_bf.log 2>&1 || { echo PROBE_FAILED; exit 1; }
tail -8 gpurun_out/probe_select_bf.log
echo rc=0
