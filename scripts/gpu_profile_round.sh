#!/bin/bash
# Round profile set: kernel-trace stats + FETCH/WRITE traffic passes for
# BASELINE configs 2, 3 and 4 (each GPU step under its own time limit).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for c in 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_c$c -o run -- python3 $R/bench.py --config $c --no-cpu-baseline --no-verify --steps 5 --warmup 1 > $R/gpurun_out/prof_c$c.log 2>&1 || exit $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -f csv -d $R/gpurun_out/pmc_c${c}_$C -o run -- python3 $R/bench.py --config $c --no-cpu-baseline --no-verify --steps 2 --warmup 1 > $R/gpurun_out/pmc_c${c}_$C.log 2>&1 || exit $?
  done
done
