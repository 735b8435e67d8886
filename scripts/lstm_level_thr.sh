#!/bin/bash
# The LSTM-AE level term's threshold (bench --lstm-level-threshold; default 5.5), one box:
# recall of +3 sigma level shifts and false positives with nothing injected, configs 3 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lstm_thr
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python bench.py --steps 5 --warmup 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name FAILED"; tail -5 $OUT/$name.err; exit 1; }
  echo "$name done"
}
for cfgname in lstm multivariate; do
  for t in ${THRS:-5.5 4.5 4.0}; do
    run ${cfgname}_t${t}_shift3 --config $cfgname --lstm-level-threshold $t --anomaly-kind shift --anomaly-size 3
    run ${cfgname}_t${t}_none --config $cfgname --lstm-level-threshold $t --anomaly-frac 0
  done
done
