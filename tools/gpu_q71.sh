#!/bin/bash
OUT=gpurun_out/q73; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "== $n"; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== $n exit $rc"; tail -8 $OUT/$n.log; case $rc in 0|1) ;; *) exit $rc;; esac; }
step ab 600 python -u tools/ab_tune.py --shared --variants "base;16=0;22=0;base;13=1" --rounds 8 --steps 10
