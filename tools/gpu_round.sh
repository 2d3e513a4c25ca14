#!/bin/bash
# One GPU-box session: gpu tests, the default bench, a rocprofv3 kernel-trace summary of the
# bench, and three PMC passes (FETCH_SIZE; WRITE_SIZE; MFMA busy + bf16/f16/f32 MFMA ops + cycles).
#   bash tools/gpu_round.sh TAG [tests|notests] [bench|nobench]
# Every GPU step runs under its own time limit; a fault / abort / timeout ends the script.
TAG=${1:-run}
MODE=${2:-tests}
BENCH=${3:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

fatal() {  # exit statuses that mean the GPU step crashed or hung
  case $1 in 124|134|137|139) return 0 ;; esac
  [ "$1" -ge 128 ] && return 0
  return 1
}

step() {  # step NAME SECONDS cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"
  tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name"; exit $rc; fi
  return 0
}

if [ "$MODE" = tests ]; then
  step pytest_gpu 1200 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
fi
if [ "$BENCH" = bench ]; then
  step bench 400 python -u bench.py
fi
step rocprof_stats 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_mfma 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE -d "$OUT/pmc_mfma" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
python3 tools/pmc_summary.py "$OUT/pmc.json" gemm_nt_h3_ $(find "$OUT"/pmc_fetch "$OUT"/pmc_write "$OUT"/pmc_mfma -name '*counter_collection.csv') > "$OUT/pmc_summary.txt" 2>&1
echo "== done"
