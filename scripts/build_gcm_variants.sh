#!/bin/bash
# Like build_variants.sh, but only gcm.hip differs between variants.
set -e
cd "$(dirname "$0")/../re_amd"
make -s -j8 >/dev/null
mkdir -p lib/variants /tmp/variants
HIPCC=/opt/rocm/bin/hipcc
FL="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-parameter -I../include -Icsrc"
pids=()
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  name=${args[i]}; defs=${args[i+1]}
  $HIPCC $FL $defs -c csrc/hip/gcm.hip -o /tmp/variants/gcm_$name.o &
done
wait
for ((i = 0; i < ${#args[@]}; i += 2)); do
  name=${args[i]}
  objs="build/srtp.o build/mem.o build/mbuf.o build/srtp_kernels.o build/ctr10.o build/ctr14.o build/plan_multi.o"
  $HIPCC -shared -fPIC --offload-arch=gfx950 -o lib/variants/$name.so $objs /tmp/variants/gcm_$name.o -lpthread
  echo "built lib/variants/$name.so (${args[i+1]})"
done
