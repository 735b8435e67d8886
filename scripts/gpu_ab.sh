#!/bin/bash
# Same-box A/B of an alternative kernel library (FOREMAST_HIP_LIB): kernel timings of both,
# then the parity tests on the alternative.  Outputs under gpurun_out/ab/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
ALT=${ALT:-foremast_amd/ops/_lib/ab/libforemast_hip.so}
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/ab/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 8 "gpurun_out/ab/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"es hw tests"}
for s in $STEPS; do
  case $s in
    es) run es_base 300 python scripts/bench_kernels.py --only es --variants "" --rounds 3
        FOREMAST_HIP_LIB=$ALT run es_alt 300 python scripts/bench_kernels.py --only es --variants "" --rounds 3 ;;
    hw) run hw_base 300 python scripts/bench_kernels.py --only hw --variants 5 --rounds 3
        FOREMAST_HIP_LIB=$ALT run hw_alt 300 python scripts/bench_kernels.py --only hw --variants 5 --rounds 3 ;;
    tests) FOREMAST_HIP_LIB=$ALT run tests_alt 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "hw or holt or smoothing or es_ or des" ;;
    lstm) SKIP_TRAIN=1 N=98304,100000 run lstm_base 300 python scripts/bench_lstm_kernels.py
          SKIP_TRAIN=1 N=98304,100000 FOREMAST_HIP_LIB=$ALT run lstm_alt 300 python scripts/bench_lstm_kernels.py
          SKIP_TRAIN=1 N=98304,100000 run lstm_base2 300 python scripts/bench_lstm_kernels.py ;;
    lstmtests) FOREMAST_HIP_LIB=$ALT run lstmtests_alt 600 python -u -m pytest tests/test_lstm.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    canary) FOREMAST_HIP_LIB=$ALT run canary_alt 600 python bench.py --steps 20 --warmup 5 ;;
  esac
done
