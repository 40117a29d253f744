#!/bin/bash
# Profiler guard words stored by the kernels: async/profiler tests, then
# config 2 (and with fresh streams: rejected plans) lines.
set -o pipefail
O=gpurun_out/r4n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_async.py tests/test_gpu_fastpath.py tests/test_gpu_streams.py > $O/pytest.log 2>&1 || exit $?
b() { local n=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b c2
b c2_fresh --ssrcs 2 --fresh-streams
b c4 --config 4
b c2b
