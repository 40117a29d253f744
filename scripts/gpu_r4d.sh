#!/bin/bash
# round 4: per-packet path + device rx index -- tests, per-call bench A/B,
# rx index timing, rocprof of the per-call kernels
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_percall.py tests/test_gpu_faults.py tests/test_gpu_shard.py > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --percall --no-cpu-baseline > $O/percall.json 2> $O/percall.err || exit $?
RE_SRTP_NOSMALL=1 timeout -k 10 400 python bench.py --percall --no-cpu-baseline > $O/percall_nosmall.json 2> $O/percall_nosmall.err || exit $?
timeout -k 10 300 python scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
timeout -k 10 300 python bench.py --rtcp-report --steps 5 > $O/rtcp_report.json 2> $O/rtcp_report.err || exit $?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- $R/re_amd/lib/percall 3000 1 > $R/$O/prof_percall.json 2> $R/$O/prof.err || exit $?
exit $rc
