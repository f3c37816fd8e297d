"""RCCL transport smoke on one box: two ranks over the "nccl" backend (RCCL),
exercising the collectives the sharded step uses (all_reduce, all_gather
_into_tensor, all_to_all_single, barrier) on device tensors.  With one GPU both
ranks share it, which RCCL may refuse; the outcome is printed either way."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ngpu)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.full((4,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    g = torch.empty((ws * 3,), device=dev)
    dist.all_gather_into_tensor(g, torch.arange(3, device=dev, dtype=torch.float32) + 10 * rank)
    a = torch.arange(ws * 2, device=dev, dtype=torch.float32) + 100 * rank
    b = torch.empty_like(a)
    w = dist.all_to_all_single(b, a, async_op=True)
    w.wait()
    dist.barrier()
    torch.cuda.synchronize()
    exp_sum = ws * (ws + 1) / 2
    ok = bool((x == exp_sum).all()) and g.view(ws, 3)[:, 0].tolist() == [10.0 * r for r in range(ws)] and \
        b.view(ws, 2)[:, 0].tolist() == [100.0 * r + 2 * rank for r in range(ws)]
    print(f"rank {rank}/{ws} on {dev} (of {ngpu}): all_reduce {x[0].item()} all_gather {g.tolist()} "
          f"all_to_all {b.tolist()} -> {'OK' if ok else 'MISMATCH'}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
