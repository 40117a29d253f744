#!/bin/bash
# GPU tests, then config-4 bench and a kernel trace of it (timeline gaps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config 4 ${BENCH_ARGS:-} > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/tl4 -o run -- python3 $R/bench.py --config 4 --no-cpu-baseline --no-verify --steps 3 --warmup 1 > $R/gpurun_out/tl4.log 2>&1
