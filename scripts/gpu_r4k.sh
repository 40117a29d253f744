#!/bin/bash
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_shard.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
