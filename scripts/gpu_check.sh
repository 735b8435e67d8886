#!/bin/bash
# GPU round script: each GPU step under its own time limit; a test FAILURE (rc 1)
# does not stop later steps, but a fault / abort / timeout (any other rc) does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests smoke bench prof"}
for s in $STEPS; do
  case $s in
    tests) run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    kgpu) run kernel_tests 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    bench0) run bench_frac0 600 python bench.py --steps 20 --warmup 5 --anomaly-frac 0 ;;
    benchshift) run bench_shift 600 python bench.py --steps 20 --warmup 5 --anomaly-kind shift3sigma ;;
    hw10k) run bench_hw10k 600 python bench.py --config hw10k --steps 20 --warmup 5 ;;
    hw10k100) run bench_hw10k100 600 python bench.py --config hw10k --steps 100 --warmup 10 ;;
    b12k) run bench_12k5 600 python bench.py --series 12500 --steps 100 --warmup 10 ;;
    graph) run bench_graph 600 python bench.py --steps 20 --warmup 5 --graph ;;
    kbench) run kbench 600 python scripts/bench_kernels.py ;;
    lstm) run bench_lstm 600 python bench.py --config lstm --steps 20 --warmup 5 ;;
    mv) run bench_mv 600 python bench.py --config multivariate --steps 20 --warmup 5 ;;
    lstmauto) run bench_lstm_autograd 600 python bench.py --config lstm --steps 20 --warmup 5 --lstm-autograd ;;
    lstmk) run lstm_kbench 300 python scripts/bench_lstm_kernels.py ;;
    lstmtests) run lstm_tests 600 python -m pytest tests/test_lstm.py -m gpu -x -q ;;
    proflstm)
      export TMPDIR=/tmp
      run proflstm 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/proflstm" -o run -- python3 "$PWD/bench.py" --config lstm --steps 5 --warmup 2 ;;
    prof)
      export TMPDIR=/tmp
      run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python3 "$PWD/bench.py" --steps 5 --warmup 2 ;;
  esac
done
