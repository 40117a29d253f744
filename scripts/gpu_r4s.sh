#!/bin/bash
# Sync vs async pair for config 2 at the driver's step counts (20 / 5),
# interleaved, twice each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s
mkdir -p $O
cd $R
for k in ${KS:-1 2}; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/sync_$k.json 2> $O/sync_$k.err || exit $?
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --async > $O/async_$k.json 2> $O/async_$k.err || exit $?
done
