#!/bin/bash
# The mean-shift rule's spread, A/B on one box: one-step sigma (default) vs the horizon-scaled
# band sigma (ML_PAIRWISE_SHIFT_ONE_STEP=0), on the 100k canary (level shifts of 1.5 / 2 / 3
# sigma, x1.2 scale, nothing injected) and the product path's false positives (--config node).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/shift_ab
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name FAILED"; tail -5 $OUT/$name.err; exit 1; }
  echo "$name done"
}
for mode in 1 0; do
  export ML_PAIRWISE_SHIFT_ONE_STEP=$mode
  for s in 1.5 2 3; do run os${mode}_shift$s --anomaly-kind shift --anomaly-size $s; done
  run os${mode}_scale1.2 --anomaly-kind scale --anomaly-size 1.2
  run os${mode}_none --anomaly-frac 0
  run os${mode}_node --config node
done
