#!/bin/bash
# Build kernel variants of the library for A/B timing on the GPU box:
#   scripts/build_variants.sh NAME "-DKNOB=V ..." [NAME "-D..."]...
# -> re_amd/lib/variants/NAME.so (load with RE_SRTP_LIB=...; bench.py as usual)
set -e
cd "$(dirname "$0")/../re_amd"
make -s -j8 >/dev/null
mkdir -p lib/variants /tmp/variants
HIPCC=/opt/rocm/bin/hipcc
FL="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-parameter -I../include -Icsrc"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  $HIPCC $FL $defs -c csrc/hip/ctr10.hip -o /tmp/variants/ctr10_$name.o &
  $HIPCC $FL $defs -c csrc/hip/ctr10a.hip -o /tmp/variants/ctr10a_$name.o &
  $HIPCC $FL $defs -c csrc/hip/gcm.hip -o /tmp/variants/gcm_$name.o &
  $HIPCC $FL $defs -c csrc/hip/plan_multi.hip -o /tmp/variants/plan_multi_$name.o &
  $HIPCC $FL $defs -c csrc/hip/fused.hip -o /tmp/variants/fused_$name.o &
  wait
  objs="build/srtp.o build/batch_host.o build/batch_dev.o build/batch_async.o build/percall.o build/rxfold.o build/pool.o build/udp.o build/keying.o build/mem.o build/mbuf.o build/srtp_kernels.o build/ctr14.o build/ctr14a.o build/plan_streams.o build/dtls_prf.o build/rtcp_walk.o build/rtcp_encode.o build/small.o"
  # NOMAP=1: every symbol exported (diagnostic variants' dump functions)
  map="-Wl,--version-script=build/exports.map"; [ -n "$NOMAP" ] && map=
  $HIPCC -shared -fPIC --offload-arch=gfx950 -o lib/variants/$name.so $objs $map \
    /tmp/variants/ctr10_$name.o /tmp/variants/ctr10a_$name.o /tmp/variants/gcm_$name.o /tmp/variants/plan_multi_$name.o \
    /tmp/variants/fused_$name.o -lpthread
  echo "built lib/variants/$name.so ($defs)"
done
