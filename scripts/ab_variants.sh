set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for so in re_amd/lib/variants/*.so; do
  name=$(basename $so .so)
  RE_SRTP_LIB=$PWD/$so timeout -k 10 200 python bench.py --no-cpu-baseline --no-verify --steps 10 > gpurun_out/var_${name}_$rep.json 2> gpurun_out/var_$name.err || exit $?
done
done
