#!/bin/bash
# PMC counter profiles (kernel-trace + counters only; never combined with
# sys/runtime traces).  TARGET selects the workload:
#   hw    — Holt-Winters scan kernel (default variant) on 20k x 10080
#   lstm  — LSTM training (per phase) + scoring kernels
#   dec   — seasonal decomposition
#   es    — ES / DES sequential fit (and the time-parallel scan variants)
#   rank  — rank tests, small-window sort path and the pairwise sweep (100k x 55 + 55)
#   seq   — Holt-Winters variant 6 (hw_seq.hip) at a short season (SEASON, default 72)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TARGET=${TARGET:-hw}
OUT="$PWD/gpurun_out/pmc_$TARGET"
mkdir -p "$OUT"
export TMPDIR=/tmp
case $TARGET in
  hw)   CMD=("$PWD/scripts/bench_kernels.py" --series 20000 --rounds 1 --only hw --variants=${VARIANTS:-3,4}) ;;
  dec)  CMD=("$PWD/scripts/bench_kernels.py" --series 20000 --rounds 1 --only decompose --variants=3) ;;
  es)   CMD=("$PWD/scripts/bench_kernels.py" --series 20000 --rounds 1 --only es --variants=) ;;
  lstm) CMD=("$PWD/scripts/bench_lstm_kernels.py") ;;
  rank) CMD=("$PWD/scripts/bench_rank.py") ;;
  gaps) CMD=("$PWD/scripts/bench_hw_gaps.py" --series 20000 --rounds 1 --cases ${CASES:-dense,dgall,miss1e-3}) ;;
  seq)  CMD=("$PWD/scripts/bench_hw_gaps.py" --series 100000 --rounds 1 --season ${SEASON:-72} --cases dense) ;;
esac
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
      "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
      "SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY")
# (FETCH_SIZE / WRITE_SIZE need many replay passes: > 5 min for these workloads — not collected)
for C in "${SETS[@]}"; do
  tag=$(echo $C | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/$tag" -o run -- python3 "${CMD[@]}" > "$OUT/$tag.log" 2>&1
  rc=$?; echo "$tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$tag.log"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
