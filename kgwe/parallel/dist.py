"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

Reads the rank environment that the platform injects into training pods
(``kgwe.parallel.rccl_env``) or that torchrun sets: RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR, MASTER_PORT.  On ROCm the ``"nccl"`` backend string
IS RCCL; on CPU hosts (tests) gloo is used so the same code path runs with
world_size > 1 and no GPU.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int
    local_rank: int
    world_size: int
    device: torch.device
    backend: str

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def _free_port() -> int:
    import socket  # noqa: PLC0415

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init(backend: str | None = None, timeout_s: int = 600, force_group: bool = False) -> DistInfo:
    """force_group: create a (possibly 1-rank) process group even when
    WORLD_SIZE == 1 — FSDP2 needs a device mesh at any world size."""
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    gpu = torch.cuda.is_available()
    if backend is None:
        backend = "nccl" if gpu else "gloo"
    if gpu:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    if (world > 1 or force_group) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            if world > 1:
                raise RuntimeError("MASTER_PORT must be set for world_size > 1")
            os.environ["MASTER_PORT"] = str(_free_port())
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistInfo(rank, local_rank, world, device, backend)


def barrier(info: DistInfo) -> None:
    if info.world_size > 1 and dist.is_initialized():
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def all_reduce_max(x: float, info: DistInfo) -> float:
    if info.world_size == 1 or not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_mean(x: float, info: DistInfo) -> float:
    if info.world_size == 1 or not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item()) / info.world_size


def all_gather_floats(x: list[float], info: DistInfo) -> list[list[float]]:
    if info.world_size == 1 or not dist.is_initialized():
        return [x]
    t = torch.tensor(x, dtype=torch.float64, device=info.device)
    out = [torch.empty_like(t) for _ in range(info.world_size)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
