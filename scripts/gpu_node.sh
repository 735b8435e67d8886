#!/bin/bash
# Node-path GPU runs: rollout / node GPU tests, the steady-arrival bench, the 20k-job burst bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/node_r4
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/node_r4/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "gpurun_out/node_r4/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests arrival burst"}
for s in $STEPS; do
  case $s in
    tests) run tests 600 python -u -m pytest tests/test_rollout.py tests/test_node.py tests/test_job_plan.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    arrival) run arrival 900 python bench.py --config node --arrival-per-tick ${J:-2000} --steps ${T:-60} ;;
    burst) run burst 600 python bench.py --config node --steps 8 --warmup 1 ;;
    prof) run prof 900 python scripts/prof_node.py --out gpurun_out/node_r4/prof --ticks 8 ;;
  esac
done
