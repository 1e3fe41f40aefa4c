#!/bin/bash
# A/B of the fill variants on one box: instruction mix (one --pmc pass each)
# and kernel-only durations (kernel trace), category fill vs per-leaf.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -e
for v in cat nocat; do
  if [ $v = nocat ]; then export NO_CAT=1; else unset NO_CAT; fi
  rm -rf gpurun_out/ab_pmc_$v gpurun_out/ab_kt_$v
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/ab_pmc_$v -o p -- python tools/profile_batch.py > gpurun_out/ab_pmc_$v.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_kt_$v -o p -- python tools/profile_batch.py > gpurun_out/ab_kt_$v.log 2>&1
  echo "== $v"
  f=$(find gpurun_out/ab_kt_$v -name '*kernel_stats.csv' | head -1); grep fill_pair "$f" | cut -d, -f1-5
  f=$(find gpurun_out/ab_pmc_$v -name '*counter_collection.csv' | head -1)
  python - "$f" <<'PY'
import csv,sys,collections
d=collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'fill_pair' in r['Kernel_Name']: d[r['Counter_Name']].append(float(r['Counter_Value']))
w=sum(d['SQ_WAVES'])/len(d['SQ_WAVES'])
print({k: round(sum(v)/len(v)/(w if k.startswith('SQ_INSTS') else 1),1) for k,v in d.items()}, 'waves', w)
PY
done
