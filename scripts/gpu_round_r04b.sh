#!/bin/bash
# Round-4 end measurement set, part B: host-array API, synchronous pairs,
# end to end, forged packets, several SSRCs, the per-packet API, the UDP
# helper, a 2-rank same-device rehearsal, rx_index timing, the RTCP report
# path, and the MP_HPER A/B of the multi-stream planner (config 4).
# Every GPU step under its own time limit; the first failure ends it.
set -o pipefail
O=gpurun_out/r04
mkdir -p $O $O/ab_hper
export TMPDIR=/tmp
b() { local n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; }
b c2_host --host-arrays --no-cpu-baseline
b c2_sync --sync --no-cpu-baseline
b c2_e2e --e2e --no-cpu-baseline
b c2_forge1 --forge 1 --no-cpu-baseline
b c2_forge001 --forge 0.001 --no-cpu-baseline
b c4_forge1 --config 4 --forge 1 --no-cpu-baseline
b c4_forge001 --config 4 --forge 0.001 --no-cpu-baseline
b c2_ssrc2 --ssrcs 2 --no-cpu-baseline
b c2_ssrc2_fresh --ssrcs 2 --fresh-streams --no-cpu-baseline
b c2_percall --percall --no-cpu-baseline
b c3_percall_gcm128 --percall --percall-suite 4 --no-cpu-baseline
b c2_udp --udp --udp-seconds 4
b c5_2rank_same_device --gpus 2 --same-device --no-cpu-baseline
timeout -k 10 300 python scripts/rx_index_timing.py > $O/rx_index.json 2> $O/rx_index.err || exit $?
b rtcp_report --rtcp-report --steps 10
for v in hper4 hper8 hper2 hper4 hper8 hper2; do
  RE_SRTP_LIB=re_amd/lib/variants/$v.so timeout -k 10 200 python bench.py --config 4 --no-cpu-baseline --steps 20 > $O/ab_hper/$v.$RANDOM.json 2> $O/ab_hper/$v.err || exit $?
done
