#!/bin/bash
# Interleaved A/B of library variants (scripts/build_variants.sh) on one box:
#   VARIANTS="base prio" ROUNDS=2 ARGS="--no-cpu-baseline" TAG=ab scripts/ab_variants.sh
# -> gpurun_out/$TAG/<variant>_<round>.json; every run under its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
cd $R
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    RE_SRTP_LIB=$R/re_amd/lib/variants/$v.so timeout -k 10 ${BENCH_TIMEOUT:-150} \
      python bench.py ${ARGS:---no-cpu-baseline} > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
  done
done
echo done > $O/done
