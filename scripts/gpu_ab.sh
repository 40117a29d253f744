#!/bin/bash
# A/B of the in-tree library against re_amd/lib/variants/*.so
# (scripts/build_variants.sh), configs in $CONFIGS (default 2), after the
# parity tests ($TESTS, default the fast-path and full-size suites).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_fullsize.py tests/test_gpu_fastpath.py} > gpurun_out/ab_tests.log 2>&1 || exit $?
for r in 1 2; do
 for c in ${CONFIGS:-2}; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/ab_base_c${c}_$r.json 2> gpurun_out/ab_base_c${c}_$r.err || exit $?
  for so in re_amd/lib/variants/*.so; do
   [ -e "$so" ] || continue
   n=$(basename $so .so)
   RE_SRTP_LIB=$PWD/$so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/ab_${n}_c${c}_$r.json 2> gpurun_out/ab_${n}_c${c}_$r.err || exit $?
  done
 done
done
