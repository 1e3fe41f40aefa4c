#!/bin/bash
# Runs GPU steps in order, each under its own time limit:
#   tools/gpu_steps.sh SECONDS 'cmd1' SECONDS 'cmd2' ...
# An ordinary failure (exit 1-2, e.g. a failed assertion) is reported and the
# next step runs; a fault, abort, segfault or time limit (124, 134, 137, 139,
# or any status >= 128) ends the call: nothing more touches the GPU.
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  secs=$1
  cmd=$2
  shift 2
  echo "[step] $cmd"
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "[step] rc=$rc"
  if [ $rc -ge 124 ]; then
    echo "[step] stopping after rc=$rc"
    exit $rc
  fi
done
