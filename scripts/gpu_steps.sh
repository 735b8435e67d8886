#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/<dir>/<name>.log.
# A step that fails normally (exit 1-2: a failed test, a bad argument) does not stop the
# rest; a time limit (124 / 137), an abort (134), a segfault (139) or any signal exit
# (> 128) ends the run at once: nothing more touches the GPU after a fault.
#
#   bash scripts/gpu_steps.sh <dir> <name>:<seconds>:'<command>' ...
set -u
dir="gpurun_out/$1"
shift
mkdir -p "$dir"
worst=0
for spec in "$@"; do
  name="${spec%%:*}"
  rest="${spec#*:}"
  secs="${rest%%:*}"
  cmd="${rest#*:}"
  echo "== $name ($secs s): $cmd" | tee -a "$dir/steps.txt"
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$dir/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc in $(( $(date +%s) - t0 )) s" | tee -a "$dir/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -gt $worst ]; then worst=$rc; fi
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then
    echo "== stopping: $name ended by a signal or its time limit" | tee -a "$dir/steps.txt"
    exit $rc
  fi
done
exit $worst
