#!/bin/bash
# variant 6 (hw_seq.hip): GPU tests, kernel timings at the short seasons against the 60 s
# step and variant 3, and the canary bench at the 1200 s step.  Every GPU step has its own
# time limit; a fault / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/seq
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/seq/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 12 "gpurun_out/seq/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
STEPS=${STEPS:-"tests k72 k1440 k24 k144 canary72"}
for s in $STEPS; do
  case $s in
    tests) step tests 300 python -u -m pytest tests/test_hw_seq.py -x -v --timeout 120 --timeout-method thread ;;
    k72) step k72 300 python -u scripts/bench_hw_gaps.py --season 72 --cases dense,miss1e-3,gap20,v3dense,v3miss1e-3 ;;
    k1440) step k1440 300 python -u scripts/bench_hw_gaps.py --season 1440 --cases dense ;;
    k24) step k24 300 python -u scripts/bench_hw_gaps.py --season 24 --cases dense,v3dense ;;
    k144) step k144 300 python -u scripts/bench_hw_gaps.py --season 144 --cases dense,miss1e-3,v3dense ;;
    k48) step k48 300 python -u scripts/bench_hw_gaps.py --season 48 --cases dense,v3dense ;;
    k96) step k96 300 python -u scripts/bench_hw_gaps.py --season 96 --cases dense,v3dense ;;
    canary72) step canary72 300 python -u bench.py --season 72 --ring 504 --steps 20 --warmup 5 ;;
    canary72m) step canary72m 300 python -u bench.py --season 72 --ring 504 --steps 20 --warmup 5 --miss-rate 1e-3 ;;
    prof72)
      export TMPDIR=/tmp
      step prof72 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/seq/prof72" -o run -- python3 "$PWD/bench.py" --season 72 --ring 504 --steps 5 --warmup 2 ;;
  esac
done
