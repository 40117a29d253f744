#!/bin/bash
# Time every library variant in re_amd/lib/variants (scripts/build_variants.sh)
# with bench.py; one JSON line per variant in gpurun_out/var_NAME.json.
set -o pipefail
mkdir -p gpurun_out
for so in re_amd/lib/variants/*.so; do
  name=$(basename $so .so)
  RE_SRTP_LIB=$PWD/$so timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var_$name.json 2> gpurun_out/var_$name.err || exit $?
  echo "$name done"
done
