#!/bin/bash
# Host-window API (srtp_*_batch): window checks and staging copies in the
# pool's parts.  Full GPU suite, then config-2 --host-arrays A/B vs
# re_amd/lib/v_base (HEAD), interleaved, 20/5 steps; config 4 host arrays.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4y
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 240 python3 bench.py --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/par_$k.json 2> $O/par_$k.err || exit $?
  RE_SRTP_LIB=$R/re_amd/lib/v_base/libre_srtp_amd.so timeout -k 10 240 python3 bench.py --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/base_$k.json 2> $O/base_$k.err || exit $?
done
timeout -k 10 240 python3 bench.py --config 4 --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_par.json 2> $O/c4_par.err || exit $?
RE_SRTP_LIB=$R/re_amd/lib/v_base/libre_srtp_amd.so timeout -k 10 240 python3 bench.py --config 4 --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_base.json 2> $O/c4_base.err || exit $?
