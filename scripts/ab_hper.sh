set -o pipefail
O=gpurun_out/ab_hper; mkdir -p $O
for v in hper4 hper8 hper2 hper4 hper8 hper2; do
  RE_SRTP_LIB=re_amd/lib/variants/$v.so timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --steps 20 > $O/$v.$RANDOM.json 2>$O/$v.err || exit $?
done
