#!/bin/bash
# PMC counter profile of the HW kernel (kernel-trace + counters only; no sys/runtime trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY"; do
  tag=$(echo $C | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$PWD/gpurun_out/pmc/$tag" -o run -- python3 "$PWD/scripts/bench_kernels.py" --series 20000 --rounds 1 --only hw --variants 2 > "gpurun_out/pmc/$tag.log" 2>&1
  rc=$?; echo "$tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/pmc/$tag.log"; fi
  if [ $rc -gt 1 ] && [ $rc -ne 2 ]; then exit $rc; fi
done
