#!/bin/bash
# HBM traffic counters for the crypto kernels, one counter per pass
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE
# cannot share a pass).  Kernel-trace only beside --pmc.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC:-}; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -f csv -d $R/gpurun_out/pmc_$C -o run -- python3 $R/bench.py --no-cpu-baseline --no-verify --steps 2 --warmup 1 ${BENCH_ARGS:-} > $R/gpurun_out/pmc_$C.log 2>&1 || exit $?
done
