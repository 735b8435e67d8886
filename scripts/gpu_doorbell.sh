#!/bin/bash
# Doorbell graph ticks: the equality test, then same-box A/Bs at the 12.5k share, config 2
# (hw10k) and the 100k headline.  Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/doorbell
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '^{' $OUT/$name.log | cut -c1-120; tail -n 2 $OUT/$name.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step test 300 python -u -m pytest tests/test_rccl_gpu.py -x -q --timeout 200 --timeout-method thread -k "doorbell or double_buffered"
for r in 1 2; do
  step b12k_bell_$r 300 python bench.py --series 12500 --steps 100 --warmup 10 --doorbell
  step b12k_plain_$r 300 python bench.py --series 12500 --steps 100 --warmup 10 --no-doorbell
  step hw10k_bell_$r 300 python bench.py --config hw10k --steps 100 --warmup 10 --doorbell
  step hw10k_plain_$r 300 python bench.py --config hw10k --steps 100 --warmup 10 --no-doorbell
done
step b100k_bell 300 python bench.py --steps 20 --warmup 5 --doorbell
step b100k_plain 300 python bench.py --steps 20 --warmup 5 --no-doorbell
