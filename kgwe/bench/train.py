"""Data-parallel Llama training harness (the workload the scheduler places).

One process per GPU (torchrun / the pod env the platform injects), sharded
data parallelism over RCCL (kgwe.parallel.zero, or FSDP2), bf16 compute, fp32
master weights, fused HIP AdamW, synthetic tokens, random-init weights.  Used by ``bench.py`` (timed steps + gfx_activity
sampling) and by ``__graft_entry__.smoke``.
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass

import torch

from ..models import llama
from ..ops import FusedAdamW
from ..parallel import dist as kdist
from ..parallel.fsdp import shard_model
from ..parallel.zero import ShardedDataParallel
from ..utils import gemm_tuning
from ..utils.amdsmi_util import UtilSampler


@dataclass
class TrainConfig:
    model: str = "llama3-8b"
    seq_len: int = 4096
    micro_batch: int = 4
    lr: float = 3e-4
    activation_checkpointing: bool = False
    # "zero": replicated bf16 weights + sharded fp32 optimizer state with
    #         bucketed RCCL reduce-scatter/all-gather (kgwe.parallel.zero);
    # "fsdp": PyTorch FSDP2 (ZeRO-3 style per-block all-gathers);
    # "none": single process, no process group.
    parallel: str = "zero"
    data: str = "random"  # "random": fresh uniform tokens each step; "fixed": one batch
    seed: int = 1234


_T0 = time.perf_counter()


def log(info, msg: str) -> None:
    if info.rank == 0 and os.environ.get("KGWE_QUIET") != "1":
        print(f"[kgwe {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


class Trainer:
    def __init__(self, tc: TrainConfig, info: kdist.DistInfo):
        self.tc = tc
        self.info = info
        self.cfg = llama.PRESETS[tc.model]
        dev = info.device
        torch.manual_seed(tc.seed)
        log(info, f"building {tc.model} ({self.cfg.num_params() / 1e9:.2f}B params) on {dev}")
        self.model = llama.build(self.cfg, device=dev, dtype=torch.float32)
        self.model.activation_checkpointing = tc.activation_checkpointing
        self.opt = None
        self.dp = None
        self.tuned_gemms = dev.type == "cuda" and gemm_tuning.enable()
        if self.tuned_gemms:
            log(info, f"GEMM solutions pinned from {gemm_tuning.RESULTS.name}")
        if tc.parallel == "fsdp":
            if not torch.distributed.is_initialized():
                raise RuntimeError("FSDP needs a process group: kdist.init(force_group=True)")
            shard_model(self.model)
            self.opt = FusedAdamW(self.model.parameters(), lr=tc.lr)
            log(info, f"FSDP2 sharded over {info.world_size} rank(s)")
        elif tc.parallel in ("zero", "none"):
            if tc.parallel == "none" and info.world_size > 1:
                raise RuntimeError("parallel='none' with WORLD_SIZE > 1")
            self.dp = ShardedDataParallel(self.model, lr=tc.lr)
            log(info, f"sharded DP over {info.world_size} rank(s): {len(self.dp.buckets)} buckets, "
                      f"replicated bf16 weights, fp32 optimizer shard "
                      f"{sum(b.shard for b in self.dp.buckets) * 12 / 2**30:.1f} GiB/rank")
        else:
            raise ValueError(f"unknown parallel mode {tc.parallel!r}")
        self._gen = torch.Generator(device=dev).manual_seed(tc.seed + info.rank)
        self.tokens = torch.empty((tc.micro_batch, tc.seq_len + 1), dtype=torch.long, device=dev)
        self.tokens.random_(0, self.cfg.vocab_size, generator=self._gen)
        self.last_loss: torch.Tensor | None = None

    @property
    def parallelism(self) -> str:
        w = self.info.world_size
        return {"fsdp": f"fsdp{w}", "zero": f"zero2-dp{w}", "none": "single"}[self.tc.parallel]

    def next_batch(self) -> None:
        """A fresh uniform-random batch every step (generated on device, ~10 us),
        so the loss stays near ln(vocab) instead of memorising one batch."""
        if self.tc.data == "random":
            self.tokens.random_(0, self.cfg.vocab_size, generator=self._gen)

    def step(self) -> torch.Tensor:
        self.next_batch()
        inp = self.tokens[:, :-1]
        lab = self.tokens[:, 1:]
        loss = self.model(inp, lab)
        loss.backward()
        if self.dp is not None:
            self.dp.step()
        else:
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
    for i in range(warmup):
        t = time.perf_counter()
        tr.step()
        tr.sync()
        log(info, f"warmup step {i}: {time.perf_counter() - t:.3f}s")
    kdist.barrier(info)
    tr.sync()
    sampler = UtilSampler(info.local_rank if info.device.type == "cuda" else 0)
    if sample_util and info.device.type == "cuda":
        sampler.start()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    tr.sync()
    log(info, f"timed {steps} steps: {time.perf_counter() - t0:.3f}s")
    kdist.barrier(info)
    tr.sync()
    dt = time.perf_counter() - t0
    sampler.stop()
    loss = float(tr.last_loss.float().item()) if tr.last_loss is not None else float("nan")
    peak = (torch.cuda.max_memory_allocated(info.device) / 2**30
            if info.device.type == "cuda" else 0.0)
    return RunResult(dt, steps, tr.tokens_per_step * steps / dt, sampler.mean,
                     len(sampler.samples), loss, peak)
