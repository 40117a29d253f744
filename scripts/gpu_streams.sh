#!/bin/bash
# Per-stream planner: its parity tests, then config-2 bench lines with one
# session over K SSRCs against the one-SSRC headline (same box).
set -o pipefail
mkdir -p gpurun_out/streams
O=gpurun_out/streams
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_streams.py > $O/tests.log 2>&1 || exit $?
B="--no-cpu-baseline --steps 10 --warmup 2"
for r in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/c2_k1_$r.json 2> $O/c2_k1_$r.err || exit $?
  timeout -k 10 200 python bench.py $B --ssrcs 2 > $O/c2_k2_$r.json 2> $O/c2_k2_$r.err || exit $?
done
timeout -k 10 200 python bench.py $B --ssrcs 2 --fresh-streams > $O/c2_k2_fresh.json 2> $O/c2_k2_fresh.err || exit $?
timeout -k 10 200 python bench.py $B --ssrcs 8 > $O/c2_k8.json 2> $O/c2_k8.err || exit $?
timeout -k 10 200 python bench.py $B --tune splan=1 > $O/c2_k1_forced.json 2> $O/c2_k1_forced.err || exit $?
timeout -k 10 200 python bench.py $B --config 3 --ssrcs 2 > $O/c3_k2.json 2> $O/c3_k2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --ssrcs 2 > $O/prof.log 2>&1 || exit $?
