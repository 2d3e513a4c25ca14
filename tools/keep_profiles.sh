#!/bin/bash
# Copy one GPU session's judged artefacts from gpurun_out/TAG into profiles/TAG_*.
TAG=$1
D=gpurun_out/$TAG
[ -f $D/pytest_gpu.log ] && cp $D/pytest_gpu.log profiles/${TAG}_pytest_gpu.log
[ -f $D/bench.log ] && grep '^{' $D/bench.log | tail -1 > profiles/${TAG}_bench.json
[ -f $D/prof/run_kernel_stats.csv ] && cp $D/prof/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
[ -f $D/pmc.json ] && cp $D/pmc.json profiles/${TAG}_pmc.json
[ -f $D/pmc_summary.txt ] && cp $D/pmc_summary.txt profiles/${TAG}_pmc_summary.txt
ls profiles/${TAG}_* 2>/dev/null
