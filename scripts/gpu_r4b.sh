#!/bin/bash
# round 4: the per-packet path (small fused kernel) -- parity tests, then
# the per-call bench with and without it (same box A/B)
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  ${1:-tests/test_gpu_parity.py tests/test_gpu_percall.py tests/test_gpu_faults.py} > $O/tests.log 2>&1
rc=$?
[ $rc -le 1 ] || cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- $R/re_amd/lib/percall 3000 1 > $R/$O/prof_percall.json 2> $R/$O/prof.err || exit $?
exit $rc
timeout -k 10 400 python bench.py --percall --no-cpu-baseline > $O/percall.json 2> $O/percall.err || exit $?
RE_SRTP_NOSMALL=1 timeout -k 10 400 python bench.py --percall --no-cpu-baseline > $O/percall_nosmall.json 2> $O/percall_nosmall.err || exit $?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- $R/re_amd/lib/percall 3000 1 > $R/$O/prof_percall.json 2> $R/$O/prof.err || exit $?
exit $rc
