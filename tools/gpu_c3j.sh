#!/bin/bash
# C3J (ragged racks, one phase-1 class per workload): kernel-trace stats and
# the SQ instruction/wait PMC passes of its batch.  Chained, each step limited.
export TMPDIR=/tmp CONFIG=C3J
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3j_prof -o run -- python3 tools/profile_batch.py > gpurun_out/c3j_prof.log 2>&1 || { echo PROF_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/c3j_pmc3 -o p -- python3 tools/profile_batch.py > gpurun_out/c3j_pmc3.log 2>&1 || { echo PMC_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/c3j_pmc4 -o p -- python3 tools/profile_batch.py > gpurun_out/c3j_pmc4.log 2>&1 || { echo PMC_FAILED; exit 1; }
echo rc=0
