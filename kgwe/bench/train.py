"""FSDP Llama training harness (the workload the scheduler places).

One process per GPU (torchrun / the pod env the platform injects), FSDP2 over
RCCL, bf16 compute, fp32 master weights, fused HIP AdamW, synthetic tokens,
random-init weights.  Used by ``bench.py`` (timed steps + gfx_activity
sampling) and by ``__graft_entry__.smoke``.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from ..models import llama
from ..ops import FusedAdamW
from ..parallel import dist as kdist
from ..parallel.fsdp import shard_model
from ..utils.amdsmi_util import UtilSampler


@dataclass
class TrainConfig:
    model: str = "llama3-8b"
    seq_len: int = 4096
    micro_batch: int = 2
    lr: float = 3e-4
    activation_checkpointing: bool = False
    fsdp: bool = True
    seed: int = 1234


class Trainer:
    def __init__(self, tc: TrainConfig, info: kdist.DistInfo):
        self.tc = tc
        self.info = info
        self.cfg = llama.PRESETS[tc.model]
        dev = info.device
        torch.manual_seed(tc.seed)
        self.model = llama.build(self.cfg, device=dev, dtype=torch.float32)
        self.model.activation_checkpointing = tc.activation_checkpointing
        if tc.fsdp:
            if not torch.distributed.is_initialized():
                raise RuntimeError("FSDP needs a process group: kdist.init(force_group=True)")
            shard_model(self.model)
        self.opt = FusedAdamW(self.model.parameters(), lr=tc.lr)
        g = torch.Generator(device=dev).manual_seed(tc.seed + info.rank)
        self.tokens = torch.randint(0, self.cfg.vocab_size, (tc.micro_batch, tc.seq_len + 1),
                                    device=dev, generator=g)
        self.last_loss: torch.Tensor | None = None

    def step(self) -> torch.Tensor:
        inp = self.tokens[:, :-1]
        lab = self.tokens[:, 1:]
        loss = self.model(inp, lab)
        loss.backward()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.last_loss = loss.detach()
        return self.last_loss

    @property
    def tokens_per_step(self) -> int:
        return self.tc.micro_batch * self.tc.seq_len

    def sync(self):
        if self.info.device.type == "cuda":
            torch.cuda.synchronize(self.info.device)


@dataclass
class RunResult:
    seconds: float
    steps: int
    tokens_per_s_local: float
    util_mean: float | None
    util_samples: int
    loss: float
    peak_mem_gb: float


def timed_run(tr: Trainer, steps: int, warmup: int, sample_util: bool = True) -> RunResult:
    info = tr.info
    for _ in range(warmup):
        tr.step()
    tr.sync()
    kdist.barrier(info)
    tr.sync()
    sampler = UtilSampler(info.local_rank if info.device.type == "cuda" else 0)
    if sample_util and info.device.type == "cuda":
        sampler.start()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    tr.sync()
    kdist.barrier(info)
    tr.sync()
    dt = time.perf_counter() - t0
    sampler.stop()
    loss = float(tr.last_loss.float().item()) if tr.last_loss is not None else float("nan")
    peak = (torch.cuda.max_memory_allocated(info.device) / 2**30
            if info.device.type == "cuda" else 0.0)
    return RunResult(dt, steps, tr.tokens_per_step * steps / dt, sampler.mean,
                     len(sampler.samples), loss, peak)
