#!/bin/bash
# Wave-time split of the fill kernels (one --pmc pass, C3 batch via tools/profile_batch.py).
export TMPDIR=/tmp
mkdir -p gpurun_out
set -e
rm -rf gpurun_out/pmcw
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmcw -o p -- python tools/profile_batch.py > gpurun_out/pmcw.log 2>&1
f=$(find gpurun_out/pmcw -name '*counter_collection.csv' | head -1)
python - "$f" <<'PY'
import csv,sys,collections
d=collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'fill_pair' in r['Kernel_Name']: d[r['Counter_Name']].append(float(r['Counter_Value']))
w=sum(d['SQ_WAVE_CYCLES'])/len(d['SQ_WAVE_CYCLES'])
print({k: round(sum(v)/len(v)/w,3) for k,v in d.items()})
PY
