"""Probe: can two ranks share one GPU under RCCL (torch nccl backend)?"""
import os
import sys
import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    t = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    out = torch.empty(8, device="cuda")
    dist.all_to_all_single(out, torch.arange(8, dtype=torch.float32, device="cuda") + 100 * rank)
    torch.cuda.synchronize()
    print(rank, t.tolist(), out.tolist(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
