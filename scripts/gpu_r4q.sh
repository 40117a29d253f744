#!/bin/bash
# Fresh multi-SSRC planner hint: tests + bench; kernel-trace of the default
# bench (config 2, synchronous pair); rx_index timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4q
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_streams.py tests/test_gpu_async.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --ssrcs 2 --fresh-streams --no-cpu-baseline > $O/c2_ssrc2_fresh.json 2> $O/c2_ssrc2_fresh.err || exit $?
timeout -k 10 200 python3 bench.py --ssrcs 2 --no-cpu-baseline > $O/c2_ssrc2.json 2> $O/c2_ssrc2.err || exit $?
timeout -k 10 240 python3 scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/stats_c2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
