#!/bin/bash
# Multi-metric rollout jobs and the node tick on the GPU: joint-model tests, node benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/node_r4
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/node_r4/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "gpurun_out/node_r4/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests burst_auto arrival"}
for s in $STEPS; do
  case $s in
    tests) run joint_tests 600 python -u -m pytest tests/test_rollout_joint.py tests/test_rollout.py tests/test_lstm_monitor.py tests/test_node.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    burst) run burst 900 python bench.py --config node --steps 8 --warmup 1 ;;
    lstmcfg) run lstm_cfg 600 python bench.py --config lstm --steps 20 --warmup 5 ;;
    burst_auto) run burst_auto 600 python bench.py --config node --steps 8 --warmup 1 --algorithm auto ;;
    arrival) run arrival 900 python bench.py --config node --arrival-per-tick ${J:-2000} --steps ${T:-60} ;;
    nodelstm) run node_lstm 900 python bench.py --config node-lstm --steps ${T:-30} ;;
    nodemv) run node_mv 900 python bench.py --config node-lstm --lstm-features 2 --steps ${T:-30} ;;
    cold) run cold 900 python bench.py --config node --cold --steps 8 --warmup 1 ;;
    prof) run prof 900 python scripts/prof_node.py --out gpurun_out/node_r4/prof --ticks 20 --warmup 12 --arrival-per-tick ${J:-2000} ;;
    profauto) run prof_auto 900 python scripts/prof_node.py --out gpurun_out/node_r4/prof_auto --ticks 8 --algorithm auto ;;
    profarrauto) run prof_arr_auto 900 python scripts/prof_node.py --out gpurun_out/node_r4/prof_arr_auto --ticks 10 --warmup 12 --arrival-per-tick ${J:-2000} --algorithm auto ;;
    arrival_auto) run arrival_auto 900 python bench.py --config node --arrival-per-tick ${J:-2000} --steps ${T:-60} --algorithm auto ;;
  esac
done
