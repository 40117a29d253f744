"""Can RCCL run two ranks on one GPU?  (torch.distributed.run
--nproc-per-node 2; both ranks on cuda:0): one all_reduce and one
all_gather of CUDA tensors, printed by rank 0."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), float(rank + 1), device="cuda")
dist.all_reduce(x)
outs = [torch.empty(3, device="cuda") for _ in range(2)]
dist.all_gather(outs, torch.full((3,), float(rank), device="cuda"))
torch.cuda.synchronize()
if rank == 0:
    print("all_reduce", x.tolist(), "all_gather", [o.tolist() for o in outs],
          "backend", dist.get_backend(), flush=True)
dist.barrier()
dist.destroy_process_group()
