#!/bin/bash
# round 4, first GPU pass: the changed GPU tests, the co-issue
# microbenchmark, one headline bench line
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 120 ./scripts/ubench_coissue.bin > $O/coissue.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_faults.py tests/test_gpu_async.py tests/test_gpu_shard.py \
  tests/test_gpu_udp.py tests/test_gpu_libre.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit $?
