set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/lpab
mkdir -p $O
cd $R
for v in d lp2 lp8 d2 lp2b lp8b; do
  case $v in d|d2) L=;; lp2|lp2b) L=$R/re_amd/lib/libre_srtp_amd_lp2.so;; lp8|lp8b) L=$R/re_amd/lib/libre_srtp_amd_lp8.so;; esac
  RE_SRTP_LIB=$L timeout -k 10 300 python3 bench.py --config 3 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit $?
done
echo done > $O/done
