#!/bin/bash
# Detection quality vs regression size on the 100k-series canary (HW + pairwise) and the
# LSTM-AE configs: one bench.py run per size, JSON lines to gpurun_out/sweep/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 150 python bench.py --steps 5 --warmup 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  echo "$name done"
}
for s in 1.5 2 3 4 6; do run canary_shift$s --anomaly-kind shift --anomaly-size $s; done
for s in 1.2 1.5 2; do run canary_scale$s --anomaly-kind scale --anomaly-size $s; done
for s in 3 6 10; do run lstm_shift$s --config lstm --anomaly-kind shift --anomaly-size $s; done
for s in 3 6 10; do run mv_shift$s --config multivariate --anomaly-kind shift --anomaly-size $s; done
