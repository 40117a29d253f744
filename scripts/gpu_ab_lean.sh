#!/bin/bash
# A/B: lean device-planned CTR kernels vs the general ones (config 2),
# after the parity tests of the paths they serve.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_shard.py tests/test_gpu_fastpath.py > gpurun_out/ab_tests.log 2>&1 || exit $?
for r in 1 2; do
for v in lean nolean; do
  t=""; [ $v = nolean ] && t="--tune nolean=1"
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 $t > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || exit $?
done
done
