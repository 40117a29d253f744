#!/bin/bash
# Per-call: runner slots, GCM in the small kernel. Tests, then A/B.
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_percall.py tests/test_gpu_parity.py tests/test_gpu_host_safety.py tests/test_gpu_faults.py tests/test_gpu_srtcp.py tests/test_gpu_shard.py tests/test_gpu_fastpath.py > $O/pytest.log 2>&1 || exit $?
b() { local n=$1; shift; timeout -k 10 300 python bench.py --percall --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
timeout -k 10 300 python scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
b gcm128 --percall-suite 4
b r1 --tune pcrunners=1
b r2 --tune pcrunners=2
b r3 --tune pcrunners=3
b r4 --tune pcrunners=4
b r2spin10k --tune pcrunners=2 --tune pcspin=10000
