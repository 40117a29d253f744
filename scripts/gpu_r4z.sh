#!/bin/bash
# Host-window API A/B, second form: window checks in parts and the
# multi-session staging copies in parts; the single-stream copy serial.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4z
mkdir -p $O
cd $R
B=$R/re_amd/lib/v_base/libre_srtp_amd.so
for k in 1 2; do
  timeout -k 10 240 python3 bench.py --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/par_$k.json 2> $O/par_$k.err || exit $?
  RE_SRTP_LIB=$B timeout -k 10 240 python3 bench.py --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/base_$k.json 2> $O/base_$k.err || exit $?
  timeout -k 10 240 python3 bench.py --config 4 --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_par_$k.json 2> $O/c4_par_$k.err || exit $?
  RE_SRTP_LIB=$B timeout -k 10 240 python3 bench.py --config 4 --host-arrays --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_base_$k.json 2> $O/c4_base_$k.err || exit $?
done
