#!/bin/bash
# LSTM-AE detection vs regression size (level term included), plus the default configs' timing:
# JSON lines to gpurun_out/lsweep/.  Extra bench.py arguments (e.g. thresholds) pass through.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lsweep
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 200 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  echo "$name done"
}
run lstm_default --config lstm "$@"
run mv_default --config multivariate "$@"
for s in 3 6; do run lstm_shift$s --config lstm --steps 5 --warmup 2 --anomaly-kind shift --anomaly-size $s "$@"; done
for s in 3 6; do run mv_shift$s --config multivariate --steps 5 --warmup 2 --anomaly-kind shift --anomaly-size $s "$@"; done
run mv_clean --config multivariate --anomaly-frac 0 "$@"
run mv_thr5 --config multivariate --lstm-threshold 5 "$@"
run mv_thr5_shift3 --config multivariate --lstm-threshold 5 --steps 5 --warmup 2 --anomaly-kind shift --anomaly-size 3 "$@"
