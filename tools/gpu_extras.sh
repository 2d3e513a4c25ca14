#!/bin/bash
# Extra measurements for one GPU session (after tools/gpu_round.sh TAG): stream A/B, the fused
# loss at the bandwidth-regime size and at C2, the CPU baselines C1 / C2. Each step has its own
# time limit; a crash or hang ends the script.
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # run NAME SECONDS cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -4 "$OUT/$name.log"
  case $rc in 0|1) ;; *) echo "FATAL in $name"; exit $rc ;; esac
}
run ab_streams 300 python -u tools/ab_streams.py --rounds 4 --steps 10
run loss_b64 120 python -u tools/bench_loss.py --B 64
run loss_c2 120 python -u tools/bench_loss.py --B 8
run cpu_baseline 400 python -u tools/cpu_baseline.py --configs c1
echo "== extras done"
