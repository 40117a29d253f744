#!/bin/bash
# CTR per-lane steady stores together (CTRF_SB_ST) A/B: parity, traffic
# and time for configs 2 and 4.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_fastpath.py > $O/pytest.log 2>&1 || exit $?
V=$R/re_amd/lib/variants/sbst0.so
b() { local n=$1 lib=$2; shift 2; RE_SRTP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b c4_new "" --config 4
b c4_old $V --config 4
b c2_new "" --config 2
b c2_old $V --config 2
b c4_new2 "" --config 4
b c4_old2 $V --config 4
cd /tmp
BA="--no-cpu-baseline --no-verify --steps 2 --warmup 1"
p() { local t=$1 c=$2 lib=$3; shift 3; RE_SRTP_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -f csv -d $O/${t}_$c -o run -- python3 $R/bench.py $BA "$@" > $O/${t}_$c.log 2>&1 || exit $?; }
for c in WRITE_SIZE FETCH_SIZE; do
  p c4new $c "" --config 4
  p c4old $c $V --config 4
done
