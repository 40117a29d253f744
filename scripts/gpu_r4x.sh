#!/bin/bash
# Kernel + memory-copy trace of the host-window mode (srtp_*_batch).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4x
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $O/tr -o run -- python3 $R/bench.py --host-arrays --no-cpu-baseline --steps 6 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
