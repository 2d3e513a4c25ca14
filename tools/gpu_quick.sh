#!/bin/bash
# Short GPU session: selected gpu tests (pytest -k expression) + extras.
#   bash tools/gpu_quick.sh TAG "pytest -k expr" [extras...]
TAG=${1:-quick}; KEXPR=${2:-loss}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run NAME SECONDS cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -4 "$OUT/$name.log"
  case $rc in 0|1) ;; *) echo "FATAL in $name"; exit $rc ;; esac
}
run pytest_sel 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$KEXPR"
shift 2
for x in "$@"; do
  case $x in
    ab) run ab_streams 300 python -u tools/ab_streams.py --rounds 4 --steps 10 ;;
    loss) run loss_b64 120 python -u tools/bench_loss.py --B 64; run loss_c2 120 python -u tools/bench_loss.py --B 8 ;;
    lossmodes) run lossmodes_b64 120 python -u tools/bench_loss.py --B 64 --modes 0,1,2,1:2,1:4,2:2,2:4; run lossmodes_c2 120 python -u tools/bench_loss.py --B 8 --modes 0,1,2,1:2,2:2 ;;
    bench) run bench 300 python -u bench.py --no-cpu-baseline ;;
    bench29b) run bench_k29_1 300 python -u bench.py --no-cpu-baseline --steps 20 --tune 29=1 && run bench_k29_3 300 python -u bench.py --no-cpu-baseline --steps 20 --tune 29=3 && run bench_k29_1b 300 python -u bench.py --no-cpu-baseline --steps 20 --tune 29=1 ;;
    prof29) run prof29 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof29" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --tune 29=1 ;;
    directw3) run direct_wgrad3 300 python -u tools/bench_kernels.py --key 29 --variants 0,2 --ops wgrad --rounds 3 --layers enc3.conv0,dec2.conv0,enc1.conv1 ;;
    dstall) run dstall 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d "$OUT/dstall" -o run --output-format csv -- python3 tools/bench_kernels.py --key 29 --variants 2 --ops fwd,dgrad,wgrad --rounds 1 --layers enc1.conv1,enc2.conv1 && run dstall2 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/dstall2" -o run --output-format csv -- python3 tools/bench_kernels.py --key 29 --variants 2 --ops fwd,dgrad,wgrad --rounds 1 --layers enc1.conv1,enc2.conv1 ;;
    wgt) run wgrad_t 300 python -u tools/bench_kernels.py --key 31 --variants 0,1 --ops wgrad --rounds 3 --layers dec2.conv0,enc3.conv1,dec3.conv0,enc4.conv0,enc4.conv1,dec4.conv0,bottleneck ;;
    benchwt) for v in 0 1 0 1; do run bench_wt$v 300 python -u bench.py --no-cpu-baseline --steps 20 --tune 31=$v || exit 1; done ;;
    wgtpmc) run wgtpmc 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d "$OUT/wgtpmc" -o run --output-format csv -- python3 tools/bench_kernels.py --key 31 --variants 0,1 --ops wgrad --rounds 1 --layers enc3.conv1,enc4.conv1,bottleneck ;;
    wgthbm) run wgthbm1 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d "$OUT/wgthbm1" -o run --output-format csv -- python3 tools/bench_kernels.py --key 31 --variants 0,1 --ops wgrad --rounds 1 --layers enc3.conv1,enc4.conv1,dec4.conv0 && run wgthbm2 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/wgthbm2" -o run --output-format csv -- python3 tools/bench_kernels.py --key 31 --variants 0,1 --ops wgrad --rounds 1 --layers enc3.conv1,enc4.conv1,dec4.conv0 && run wgtkt 120 rocprofv3 --kernel-trace --stats -d "$OUT/wgtkt" -o run --output-format csv -- python3 tools/bench_kernels.py --key 31 --variants 0,1 --ops wgrad --rounds 1 --layers enc3.conv1,enc4.conv1,dec4.conv0 ;;
    pol) for v in 1 3 4 5 1; do run bench_p$v 300 python -u bench.py --no-cpu-baseline --steps 20 --tune 29=$v || exit 1; done ;;
    bench29) run bench_k29_0 300 python -u bench.py --no-cpu-baseline --steps 20 && run bench_k29_1 300 python -u bench.py --no-cpu-baseline --steps 20 --tune 29=1 ;;
    direct) run direct_kernels 300 python -u tools/bench_kernels.py --key 29 --variants 0,2 --ops fwd,dgrad --rounds 3 --layers enc1.conv1,dec1.conv0,enc2.conv0,enc2.conv1,dec2.conv0,enc3.conv0,enc3.conv1 ;;
    directw) run direct_wgrad 300 python -u tools/bench_kernels.py --key 29 --variants 0,2 --ops wgrad --rounds 3 --layers enc1.conv1,dec1.conv0,enc2.conv0,enc2.conv1,dec2.conv0 ;;
    directprof) run directprof 200 rocprofv3 --kernel-trace --stats -d "$OUT/directprof" -o run --output-format csv -- python3 tools/bench_kernels.py --key 29 --variants 0,2 --ops fwd,dgrad --rounds 1 --layers enc1.conv1,dec1.conv0,enc2.conv1 ;;
    gemm) run bench_gemm 300 python -u tools/bench_gemm.py --variants 6,11,12 --rounds 3 --check ;;
    lossprof) run lossprof 200 rocprofv3 --kernel-trace --stats -d "$OUT/lossprof" -o run --output-format csv -- python3 tools/bench_loss.py --B 64 --reps 20 ;;
    lossprof8) run lossprof8 200 rocprofv3 --kernel-trace --stats -d "$OUT/lossprof8" -o run --output-format csv -- python3 tools/bench_loss.py --B 8 --reps 20 ;;
  esac
done
echo "== quick done"
