#!/bin/bash
# per-call path: kernel durations of one thread's srtp_encrypt/decrypt
# calls (rocprofv3 kernel trace), small path and general path
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/small -o run -- $R/re_amd/lib/percall 3000 1 > $R/$O/small.json 2> $R/$O/small.err || exit $?
RE_SRTP_NOSMALL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/general -o run -- $R/re_amd/lib/percall 3000 1 > $R/$O/general.json 2> $R/$O/general.err || exit $?
