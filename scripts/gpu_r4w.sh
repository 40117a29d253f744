#!/bin/bash
# Final build, the driver's step counts (20 / 5): configs 2, 3, 4, 2 SRTCP.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4w
mkdir -p $O
cd $R
b() { local name=$1; shift; timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 "$@" > $O/$name.json 2> $O/$name.err; }
b c2 && b c3 --config 3 --no-cpu-baseline && b c4 --config 4 --no-cpu-baseline && b c2_rtcp --rtcp --no-cpu-baseline || exit $?
