#!/bin/bash
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_shard.py > $O/pytest.log 2>&1 || exit $?
