#!/bin/bash
# LSTM-AE detection vs regression size (level term included), the default configs' timing and
# the false positives with nothing injected: JSON lines to gpurun_out/lsweep/.  Extra bench.py
# arguments (e.g. thresholds) pass through.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lsweep
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 200 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  echo "$name done"
}
for c in lstm multivariate; do
  run ${c}_default --config $c "$@"
  run ${c}_clean --config $c --steps 5 --warmup 2 --anomaly-frac 0 "$@"
  for s in 3 6; do run ${c}_shift$s --config $c --steps 5 --warmup 2 --anomaly-kind shift --anomaly-size $s "$@"; done
done
