#!/bin/bash
# Round-start GPU check: parity tests, one bench, and the fill/select
# instruction-counter PMC pass (its own rocprofv3 run, no tracing domains).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc3 -o p -- python3 tools/profile_batch.py > gpurun_out/pmc3.log 2>&1 || { echo PMC3_FAILED; exit 1; }
echo rc=0
