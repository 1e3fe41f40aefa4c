#!/bin/bash
# One GPU session: parity tests -> bench (with CPU baseline) -> kernel-trace
# profile of the bench -> separate PMC passes (FETCH_SIZE, WRITE_SIZE).
# Every GPU step has its own time limit; the chain stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu > gpurun_out/prof_bench.json 2> gpurun_out/prof.log || { echo PROF_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc1 -o p -- python3 tools/profile_batch.py > gpurun_out/pmc1.log 2>&1 || { echo PMC1_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc2 -o p -- python3 tools/profile_batch.py > gpurun_out/pmc2.log 2>&1 || { echo PMC2_FAILED; exit 1; }
echo rc=0
