#!/bin/bash
# Helpers for one GPU-box session:  source tools/gpu_lib.sh TAG; step NAME SECONDS cmd...
# Each step runs under its own time limit with its log in gpurun_out/TAG/NAME.log; a crash, abort
# or timeout (exit >= 124) ends the session (exit with that code); test failures (1) do not.
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"
  tail -4 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "FATAL in $name"; exit $rc; fi
  return 0
}
