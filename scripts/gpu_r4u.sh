#!/bin/bash
# Multi-session plan: state uploads on the workspace's side stream.
# Multi-session GPU tests, then config-4 A/B vs re_amd/lib/v_base (HEAD),
# interleaved, 20/5 steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4u
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fastpath.py tests/test_gpu_mfold.py tests/test_gpu_async.py tests/test_gpu_keying.py > $O/pytest.log 2>&1 || exit $?
for k in 1 2 3; do
  timeout -k 10 200 python3 bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > $O/side_$k.json 2> $O/side_$k.err || exit $?
  RE_SRTP_LIB=$R/re_amd/lib/v_base/libre_srtp_amd.so timeout -k 10 200 python3 bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline > $O/base_$k.json 2> $O/base_$k.err || exit $?
done
