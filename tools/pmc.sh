#!/bin/bash
# Separate rocprofv3 --pmc passes (never combined with tracing domains).
# usage: [CONFIG=C3J] bash tools/pmc.sh [tag]   (tag: suffix of the output directories)
export TMPDIR=/tmp
set -e
T="${1:-}"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc1$T -o p -- python tools/profile_batch.py > gpurun_out/pmc1$T.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc2$T -o p -- python tools/profile_batch.py > gpurun_out/pmc2$T.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc3$T -o p -- python tools/profile_batch.py > gpurun_out/pmc3$T.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc4$T -o p -- python tools/profile_batch.py > gpurun_out/pmc4$T.log 2>&1
echo pmc_done
