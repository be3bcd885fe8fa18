"""Can two ranks share one GPU under RCCL? (a rehearsal transport for the
multi-rank path on a one-GPU box). Each rank: init nccl on cuda:0, one
all_reduce and one all_to_all_single; prints the result or the error.
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/rccl_shared_gpu_probe.py"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
        x = torch.full((4,), rank + 1.0, device="cuda:0")
        dist.all_reduce(x)
        y = torch.arange(world * 2, dtype=torch.float32, device="cuda:0") + 100 * rank
        z = torch.empty_like(y)
        dist.all_to_all_single(z, y)
        torch.cuda.synchronize()
        print(f"rank {rank}: all_reduce {x.tolist()} all_to_all {z.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: FAILED {type(e).__name__}: {e}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
