#!/bin/bash
# The mean-shift rule on the 100k canary, one box: its spread (one-step sigma vs the
# horizon-scaled band sigma) and its threshold (sigmas): recall at 1.5 / 2 sigma level shifts
# and false positives with nothing injected.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/shift_thr
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name FAILED"; tail -5 $OUT/$name.err; exit 1; }
  echo "$name done"
}
for sp in one-step horizon; do
  for t in ${THRS:-1.0 1.25 1.5}; do
    a="--pairwise-shift $t --pairwise-shift-spread $sp"
    for s in 1.5 2; do run ${sp}_t${t}_shift$s $a --anomaly-kind shift --anomaly-size $s; done
    run ${sp}_t${t}_none $a --anomaly-frac 0
  done
done
