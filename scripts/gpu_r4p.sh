#!/bin/bash
# Kernel-trace stats of the default bench (config 2, synchronous pair).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4p
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/stats_c2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
cd $R
timeout -k 10 240 python3 scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
