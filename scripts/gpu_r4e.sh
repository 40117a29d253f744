#!/bin/bash
# Per-call fused launches: the per-call tests, the parity/fault tests that
# run per-packet calls, then the per-call bench with and without fusion.
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_percall.py tests/test_gpu_parity.py tests/test_gpu_faults.py tests/test_gpu_host_safety.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --percall --no-cpu-baseline > $O/percall_fuse.json 2> $O/percall_fuse.err || exit $?
timeout -k 10 300 python bench.py --percall --no-cpu-baseline --tune nofuse=1 > $O/percall_nofuse.json 2> $O/percall_nofuse.err || exit $?
