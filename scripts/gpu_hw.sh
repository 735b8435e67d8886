#!/bin/bash
# Holt-Winters fit GPU runs: the variant-5 parity / pruning tests, the prune / spec / waves A/B,
# optional PMC passes.  Outputs under gpurun_out/hw_r4/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hw_r4
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/hw_r4/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "gpurun_out/hw_r4/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests ab"}
for s in $STEPS; do
  case $s in
    tests) run tests 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "hw or holt or smoothing or es_ or des or decompose" ;;
    ab) run ab 600 python scripts/hw_prune_ab.py --iters ${ITERS:-8} ${AB_ARGS:-} ;;
    abmix) run abmix 600 python scripts/hw_prune_ab.py --iters ${ITERS:-8} --mix ${AB_ARGS:-} ;;
    kern) run kern 600 python scripts/bench_kernels.py --only es,decompose --variants "" --rounds 3 ;;
    k4) run k4_tests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "decompose"
        run k4_bench 300 python scripts/bench_kernels.py --only decompose --variants "" --rounds 5 ;;
    lstmsweep) SKIP_TRAIN=1 N=${LSTM_N:-24576,49152,73728,98304,100000,122880} run lstm_sweep 300 python scripts/bench_lstm_kernels.py ;;
    canary) run canary 600 python bench.py --steps 20 --warmup 5 ;;
  esac
done
