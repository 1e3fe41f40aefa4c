#!/bin/bash
# Round-5 GPU cycle: parity tests named in $TESTS (default: the fill and
# parity suites), a bench without the CPU leg, a rocprofv3 kernel-trace of
# the same bench (per-kernel stats with VGPR/SGPR from the database).
# Each GPU step under its own limit; stop at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_pair_fill.py tests/test_gpu_parity.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu $TESTS > gpurun_out/r5_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5_tests.log; exit 1; }
tail -2 gpurun_out/r5_tests.log
timeout -k 10 300 python bench.py --no-cpu --no-extras > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r5_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5_bench.json')); print(d['value'], d['step_ms'], d['stages'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['work']['fill_paths'])"
rm -rf gpurun_out/r5_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_prof -o run -- python3 bench.py --no-cpu --no-extras --steps 20 > gpurun_out/r5_prof_bench.json 2> gpurun_out/r5_prof.log || { echo PROF_FAILED; tail -20 gpurun_out/r5_prof.log; exit 1; }
db=$(find gpurun_out/r5_prof -name '*.db' | head -1)
python tools/rocpd_stats.py "$db" gpurun_out/r5_kernel_stats.csv && cut -d, -f1-6,8-11 gpurun_out/r5_kernel_stats.csv | head -16
echo rc=0
