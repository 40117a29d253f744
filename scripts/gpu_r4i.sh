#!/bin/bash
# SRTCP-GCM unprotect traffic: write requests by size and L2 write-backs
# per dispatch, config 3 over SRTCP and over RTP.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4i
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
BA="--no-cpu-baseline --no-verify --steps 2 --warmup 1"
C="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_NORMAL_WRITEBACK_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum"
p() { local t=$1; shift; timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace -f csv -d $O/${t}_wr -o run -- python3 $R/bench.py $BA "$@" > $O/${t}_wr.log 2>&1 || exit $?; }
p c3rtcp --config 3 --rtcp
p c3 --config 3
p c2rtcp --config 2 --rtcp
