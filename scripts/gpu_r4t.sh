#!/bin/bash
# k_plan_scan folded into k_plan_desc: planner tests, then config-2 A/B
# (fused default vs re_amd/lib/v_noscan with the separate scan), 20/5 steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4t
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fastpath.py tests/test_gpu_parity.py tests/test_gpu_devfold.py tests/test_gpu_async.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1 || exit $?
for k in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/fused_$k.json 2> $O/fused_$k.err || exit $?
  RE_SRTP_LIB=$R/re_amd/lib/v_noscan/libre_srtp_amd.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/scan_$k.json 2> $O/scan_$k.err || exit $?
done
