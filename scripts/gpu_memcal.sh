#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the kernels' own access patterns
# (scripts/ubench_mem.hip), one counter per pass, plus the kernel times.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/memcal
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 $R/scripts/ubench_mem > $O/times.txt 2>&1 || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -f csv -d $O/pmc_$C -o run -- $R/scripts/ubench_mem > $O/pmc_$C.log 2>&1 || exit $?
done
