#!/bin/bash
# Round-5 validation: dense multi-run chunks under leaf categories (pair-fill
# GPU test, C3J and C3 A/B with oracle checks, C3 kernel traces both ways),
# admission sweeps with backoff.  Each step limited, chained.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pair_fill.py > gpurun_out/pair_fill.log 2>&1 || { echo PAIR_FAILED; exit 1; }
timeout -k 10 300 python tools/probe_c3j.py --check 1024 > gpurun_out/c3j_dense.log 2>&1 || { echo C3J_FAILED; exit 1; }
NO_DENSE=1 timeout -k 10 300 python tools/probe_c3j.py > gpurun_out/c3j_single.log 2>&1 || { echo C3J2_FAILED; exit 1; }
NO_CAT=1 timeout -k 10 300 python tools/probe_c3j.py > gpurun_out/c3j_nocat.log 2>&1 || { echo C3J3_FAILED; exit 1; }
timeout -k 10 300 python tools/probe_c3j.py --config C3 --check 1024 > gpurun_out/c3_dense.log 2>&1 || { echo C3_FAILED; exit 1; }
NO_DENSE=1 timeout -k 10 300 python tools/probe_c3j.py --config C3 > gpurun_out/c3_single.log 2>&1 || { echo C3S_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dense -o run -- python3 tools/profile_batch.py > gpurun_out/prof_dense.log 2>&1 || { echo PROF_FAILED; exit 1; }
NO_DENSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_single -o run -- python3 tools/profile_batch.py > gpurun_out/prof_single.log 2>&1 || { echo PROF2_FAILED; exit 1; }
timeout -k 10 300 python tools/probe_admit.py C3 1024 8192 > gpurun_out/probe_admit.log 2>&1 || { echo ADMIT_FAILED; exit 1; }
timeout -k 10 300 python tools/probe_admit.py C5 8192 > gpurun_out/probe_admit_c5.log 2>&1 || { echo ADMIT5_FAILED; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_admission.py > gpurun_out/admission_tests.log 2>&1 || { echo ADM_TESTS_FAILED; exit 1; }
echo rc=0
