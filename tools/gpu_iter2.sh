#!/bin/bash
# Host-side measurements on the GPU box: HIP event / sync costs, the pool job
# round trip, the host trace (with the records / class-merge cycle counters),
# then the bench (no CPU legs) and a kernel trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
(cd tools/micro && g++ -O2 -std=c++17 -pthread pool_bench.cpp -o pool_bench) || exit 1
timeout -k 5 60 tools/micro/pool_bench > gpurun_out/pool_bench.log 2>&1; cat gpurun_out/pool_bench.log
timeout -k 5 60 tools/micro/sync_cost > gpurun_out/sync_cost.log 2>&1 || { echo SYNC_FAILED; exit 1; }
cat gpurun_out/sync_cost.log
timeout -k 10 120 python tools/probe_trace.py C3 > gpurun_out/trace_iter.log 2>&1 || { echo TRACE_FAILED; tail gpurun_out/trace_iter.log; exit 1; }
tail -12 gpurun_out/trace_iter.log
bash tools/gpu_iter.sh "$1"
