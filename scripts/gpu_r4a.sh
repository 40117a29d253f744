#!/bin/bash
# round 4 GPU pass: the named GPU tests ($TESTS), then one headline bench
# line; the bench runs after failed tests (exit 1) but after nothing worse
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  ${1:-tests/test_gpu_faults.py tests/test_gpu_async.py tests/test_gpu_shard.py tests/test_gpu_udp.py tests/test_gpu_libre.py tests/test_gpu_rtcp.py} > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
[ -n "$NOBENCH" ] || timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit $?
exit $rc
