"""Probe: can RCCL (torch 'nccl' backend) run two ranks on one GPU of this pool's boxes?

Run under torch.distributed.run with --nproc-per-node 2. Every rank uses cuda:0. Prints
one line per rank with the all_to_all_single result, or the exception text.
"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", device_id=dev)
        x = torch.arange(world * 4, dtype=torch.uint8, device=dev) + 16 * rank
        y = torch.empty_like(x)
        dist.all_to_all_single(y, x)
        torch.cuda.synchronize()
        print(f"rank {rank}: ok {y.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # the point of the probe is the error text
        print(f"rank {rank}: {type(e).__name__}: {e}", flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
