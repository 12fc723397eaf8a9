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
from ..parallel.checkpoint import Checkpointer
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
    ckpt_dir: str | None = None  # sharded checkpoints (kgwe.parallel.checkpoint); resume if present
    ckpt_every: int = 0          # steps between checkpoints (0: only at the end of run())
    # gradient reduce-scatter dtype of the sharded-DP path at world > 1: fp32
    # (exact sums) or bf16 (half the xGMI bytes per step)
    reduce_dtype: torch.dtype = torch.bfloat16  # gradient reduce-scatter at world > 1 (see kgwe.parallel.zero)


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
            self.dp = ShardedDataParallel(self.model, lr=tc.lr, reduce_dtype=tc.reduce_dtype)
            log(info, f"sharded DP over {info.world_size} rank(s): {len(self.dp.buckets)} buckets, "
                      f"replicated bf16 weights, fp32 optimizer shard "
                      f"{sum(b.shard for b in self.dp.buckets) * 12 / 2**30:.1f} GiB/rank")
        else:
            raise ValueError(f"unknown parallel mode {tc.parallel!r}")
        self._gen = torch.Generator(device=dev).manual_seed(tc.seed + info.rank)
        self.tokens = torch.empty((tc.micro_batch, tc.seq_len + 1), dtype=torch.long, device=dev)
        self.tokens.random_(0, self.cfg.vocab_size, generator=self._gen)
        self.last_loss: torch.Tensor | None = None
        self.global_step = 0
        self.ckpt = None
        if tc.ckpt_dir:
            if self.dp is None:
                raise ValueError("checkpointing needs the sharded-DP trainer (parallel='zero')")
            self.ckpt = Checkpointer(tc.ckpt_dir)
            got = self.ckpt.load(self.dp)
            if got is not None:  # resumed (e.g. rescheduled after a node / GPU failure)
                self.global_step = got["step"]
                gs = got["extra"].get("gen_state")
                if gs is not None and gs.numel():
                    self._gen.set_state(gs)
                log(info, f"resumed from {tc.ckpt_dir} at step {self.global_step}")

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
        self.global_step += 1
        if self.ckpt is not None and self.tc.ckpt_every and self.global_step % self.tc.ckpt_every == 0:
            self.checkpoint()
        return self.last_loss

    def checkpoint(self, blocking: bool = False) -> None:
        gen = self._gen.get_state()
        self.ckpt.save(self.dp, self.global_step, {"gen_state": gen.cpu()}, blocking=blocking)

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


def train(tr: Trainer, total_steps: int) -> float:
    """Run until ``total_steps`` (counting steps done before a resume), then
    write a final checkpoint.  Returns the last loss."""
    while tr.global_step < total_steps:
        loss = tr.step()
        if tr.global_step % 10 == 0:
            log(tr.info, f"step {tr.global_step}: loss {loss.float().item():.4f}")
    if tr.ckpt is not None:
        tr.checkpoint(blocking=True)
    return float(tr.last_loss.float().item()) if tr.last_loss is not None else float("nan")


def main(argv=None) -> int:
    """Training entrypoint for a placed job (``kgwe launch -- torchrun ...
    -m kgwe.bench.train``): resumes from --ckpt-dir when a checkpoint exists."""
    import argparse

    ap = argparse.ArgumentParser(prog="kgwe-train")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-every", type=int, default=0)
    a = ap.parse_args(argv)
    info = kdist.init(force_group=True)
    tr = Trainer(TrainConfig(model=a.model, seq_len=a.seq_len, micro_batch=a.micro_batch, lr=a.lr,
                             ckpt_dir=a.ckpt_dir, ckpt_every=a.ckpt_every), info)
    loss = train(tr, a.steps)
    log(info, f"done at step {tr.global_step}: loss {loss:.4f}")
    kdist.shutdown()
    return 0


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


if __name__ == "__main__":
    raise SystemExit(main())
