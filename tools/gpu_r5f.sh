#!/bin/bash
# Is the BestFit select's 20 us stall the pinned-host entry writes (select and
# lfc_emit store (leaf, count) pairs over PCIe)?  The same batch with the
# packed device-side entries (KUEUE_TAS_CFG_PACKED_ENTRIES): per-eval ticks
# and kernel traces, both ways.  Chained, each step limited.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/sel_mapped.log 2>&1 || { echo S1_FAILED; exit 1; }
PACKED=1 timeout -k 10 200 python tools/probe_select.py --prof > gpurun_out/sel_packed.log 2>&1 || { echo S2_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_mapped -o run -- python3 tools/profile_batch.py > gpurun_out/kt_mapped.log 2>&1 || { echo K1_FAILED; exit 1; }
PACKED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_packed -o run -- python3 tools/profile_batch.py > gpurun_out/kt_packed.log 2>&1 || { echo K2_FAILED; exit 1; }
echo rc=0
