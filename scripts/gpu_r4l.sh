#!/bin/bash
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_same_device.py > $O/rccl.log 2>&1
echo "rc=$?" >> $O/rccl.log
