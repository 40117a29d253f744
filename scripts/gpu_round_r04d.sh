#!/bin/bash
# Round-4 final measurement set (after every change of the round): the
# full GPU suite and smoke, the BASELINE configs and SRTCP, the API modes,
# forged packets, several SSRCs, the per-packet API per suite family, the
# UDP helper, the 2-rank same-device rehearsal, the fold costs and the
# RTCP report path.  Every GPU step under its own time limit; the first
# failure ends the script.
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b c2
b c3 --config 3 --no-cpu-baseline
b c4 --config 4 --no-cpu-baseline
b c2_rtcp --rtcp --no-cpu-baseline
b c3_rtcp --config 3 --rtcp --no-cpu-baseline
b c2_host --host-arrays --no-cpu-baseline
b c2_sync --sync --no-cpu-baseline
b c2_e2e --e2e --no-cpu-baseline
b c2_forge001 --forge 0.001 --no-cpu-baseline
b c4_forge001 --config 4 --forge 0.001 --no-cpu-baseline
b c2_ssrc2 --ssrcs 2 --no-cpu-baseline
b c2_ssrc2_fresh --ssrcs 2 --fresh-streams --no-cpu-baseline
b c2_percall --percall --no-cpu-baseline
b c3_percall_gcm128 --percall --percall-suite 4 --no-cpu-baseline
b c3_percall_gcm256 --percall --percall-suite 5 --no-cpu-baseline
b c2_udp --udp --udp-seconds 4
b c5_2rank_same_device --gpus 2 --same-device --no-cpu-baseline
timeout -k 10 300 python scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
b rtcp_report --rtcp-report --steps 10
