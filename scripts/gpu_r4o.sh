#!/bin/bash
# New bench defaults (sync pair for one session) + the bench GPU tests.
set -o pipefail
O=gpurun_out/r4o3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_async.py > $O/pytest.log 2>&1 || exit $?
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b c2
b c3 --config 3 --no-cpu-baseline
b c4 --config 4 --no-cpu-baseline
b c2_forge001 --forge 0.001 --no-cpu-baseline
b c2_async --async --no-cpu-baseline
b c5_2rank --gpus 2 --same-device --no-cpu-baseline
