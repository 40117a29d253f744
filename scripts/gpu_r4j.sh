#!/bin/bash
# GCM chunk stores kept together: parity (GCM tests + full-size digests),
# then traffic passes and bench lines for config 3 over RTP and SRTCP.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_fastpath.py tests/test_gpu_srtcp.py > $O/pytest.log 2>&1 || exit $?
cd /tmp
BA="--no-cpu-baseline --no-verify --steps 2 --warmup 1"
p() { local t=$1 c=$2; shift 2; timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -f csv -d $O/${t}_$c -o run -- python3 $R/bench.py $BA "$@" > $O/${t}_$c.log 2>&1 || exit $?; }
for c in WRITE_SIZE FETCH_SIZE; do
  p c3rtcp $c --config 3 --rtcp
  p c3 $c --config 3
done
cd $R
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit $?
timeout -k 10 300 python bench.py --config 3 --rtcp --no-cpu-baseline > $O/c3_rtcp.json 2> $O/c3_rtcp.err || exit $?
