#!/bin/bash
# Small-kernel completion by a pinned word: launch ubench, per-call tests
# and bench (CM80, GCM128).
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp
#timeout -k 10 120 ./scripts/ubench_launch.bin > $O/ubench_launch.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_percall.py tests/test_gpu_parity.py tests/test_gpu_host_safety.py tests/test_gpu_faults.py tests/test_gpu_fastpath.py tests/test_gpu_srtcp.py > $O/pytest.log 2>&1 || exit $?
b() { local n=$1; shift; timeout -k 10 300 python bench.py --percall --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b cm80
b gcm128 --percall-suite 4
