#!/bin/bash
# Same-box A/B of environment knobs on the C2 bench: alternating bench.py runs, one JSON line each.
#   bash tools/ab_env.sh OUTDIR "VAR=a VAR=b ..." [rounds]
# Each GPU step runs under its own time limit; a failing run ends the script.
OUT=$1; VARIANTS=$2; ROUNDS=${3:-2}
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARIANTS; do
    env "$v" timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/b_${v}_$r.log" 2>&1 || exit $?
    python - "$v" "$OUT/b_${v}_$r.log" >> "$OUT/summary.txt" <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1], round(d["value"], 2), round(d["ms_per_step"], 3))
PY
  done
done
cat "$OUT/summary.txt"
