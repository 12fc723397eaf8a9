"""Sharded data parallelism sized for 288 GB of HBM3E per GPU.

An 8B model's bf16 weights are 16 GB — 6 % of one MI355X — so there is no
reason to re-gather them layer by layer every forward (ZeRO-3 / FSDP).  This
module keeps the **bf16 weights replicated** and shards only what is large:
the fp32 master weights and both Adam moments (12 B/param) and the reduced
gradient (ZeRO-2):

* parameters live in a few large flat bf16 **buckets** (~100 M elements,
  backward order); every ``nn.Parameter`` is a view into one, so the model
  code is unchanged;
* backward: with the default bf16 reduce, each linear layer's
  weight-gradient GEMM writes straight into its slice of the bucket's
  gradient buffer (``_grad_sink``: no gradient tensor, no copy); the few
  other parameters (norms, embedding) and the fp32-reduce option go through
  a post-accumulate-grad hook that copies the gradient in and frees it.  When
  a bucket is complete its **reduce-scatter** is issued asynchronously over
  RCCL, so the collectives of early buckets overlap the rest of backward.
  bf16 reduction halves the bytes on the xGMI ring; it perturbs the update no
  more than the bf16 rounding of the local gradients already does (bounded
  against fp32 reduction for worlds 4 and 8 in tests/test_parallel_cpu.py);
* update, per bucket, as soon as the bucket's gradients are reduced — still
  inside backward, on a side HIP stream: a multi-tensor HIP AdamW launch over
  this rank's shard (fp32 master, m, v; grads averaged through
  ``grad_scale``) writes the rounded bf16 result straight into this rank's
  slice of the bucket, then an in-place **all-gather** re-replicates the
  weights.  The HBM-bound optimizer and the collectives thus run beside the
  MFMA-bound backward GEMMs; the next forward waits for a bucket only in the
  pre-hook of the first module that reads it.

Per step and per GPU that is one reduce-scatter of the gradients and one
all-gather of the bf16 weights — FSDP's volume with reshard_after_forward off
— in ~2 x (params / bucket) large collectives, the shape ring collectives
over point-to-point xGMI links want.

With one rank there is no communication at all: AdamW (still per bucket,
from the backward hooks) reads autograd's bf16 gradients in place and
writes the bf16 weights the next forward reads — no
cast, copy or all-gather-copy kernels (the FSDP2 path spends ~90 ms/step on
those at 1 GPU for Llama-3-8B, profiles/r01_pack).

Reference: distribution strategies are metadata only in the reference
(src/scheduler/types.go:157-166, ``FSDP``/``DeepSpeed`` = ZeRO); this is the
training-side implementation the platform places.
"""
from __future__ import annotations

import contextlib
import functools
import os

import torch
import torch.distributed as dist

from ..ops import functional as K
from ..ops.adamw import AdamPlan


class _Done:
    """Handle of a collective that has already completed."""

    def wait(self) -> None:
        pass


class _Bucket:
    __slots__ = ("params", "offsets", "numel", "padded", "shard", "flat", "master", "m", "v",
                 "gfull", "gshard", "pending", "seen", "rs_work", "ag_work", "ready", "updated",
                 "tparams", "flat_t")


class ShardedDataParallel:
    """overlap_step=True (default): each bucket's optimizer update is issued
    from the backward hook that completes the bucket, on a side HIP stream —
    world 1: AdamW straight from autograd's bf16 gradients; world N:
    reduce-scatter (compute-stream order) -> AdamW on the shard -> in-place
    all-gather, chained on the side / RCCL streams — so the HBM-bound AdamW
    and the collectives run under the rest of backward's MFMA-bound GEMMs,
    and only the last bucket's update is exposed.  A bucket's weights are free
    to change once its gradients are complete: every backward op that reads
    a weight (dX = dY W) runs in the same autograd node that produces that
    weight's gradient, before the accumulate-grad hook fires.  This assumes
    each parameter receives ONE gradient per backward (no weight tying).
    The next forward waits per bucket in a module pre-hook.

    transposed_weights=True (GPU): every linear weight W [N, K] also keeps a
    bf16 copy of W^T [K, N] (``p._kgwe_wt``), refreshed on the side stream
    right after the bucket's update (world 1) or all-gather (world N).  The
    input-gradient GEMM dX = dY W then runs as dY (W^T)^T — hipBLASLt's "nt"
    layout, ~1.5 PF/s on MI355X against ~1.35 for the "nn" layout W needs
    (tools/gemm_layouts.py) — at the price of 2 B/param of HBM (15 GB for an
    8B model, of 288 GB) and one 2x16 GB transpose pass per step, overlapped
    with backward."""

    def __init__(self, model: torch.nn.Module, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, bucket_elems: int = 100 * 2**20,
                 reduce_dtype: torch.dtype = torch.bfloat16, group=None, overlap_step: bool = True,
                 transposed_weights: bool = True, background_grid: int | None = None):
        self.model = model
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.reduce_dtype = reduce_dtype
        self.overlap = overlap_step
        # Workgroup cap of the AdamW launches that run BESIDE backward (every
        # bucket but the last to complete).  A full-grid HBM-bound update
        # co-resides on every CU and roughly doubles the GEMM next to it
        # (tools/gemm_instep.py), but a capped grid only stretches the damage
        # over more GEMMs: 699 ms/step uncapped, 701 / 723 / 777 / 882 at
        # 1024 / 256 / 128 / 64 workgroups (profiles/r02_step/SUMMARY.md).
        # Kept as a knob; 0 = no cap (default).
        if background_grid is None:
            background_grid = int(os.environ.get("KGWE_ADAMW_BG_GRID", "0"))
        self.background_grid = max(0, background_grid)
        self._step = 0
        self._armed = False  # this iteration's step counter already advanced
        # events every writer of master / m / v / flat must wait for before the
        # next update (e.g. a checkpoint's device -> host copy still reading them)
        self._fences: list = []
        self._plan = AdamPlan()
        params = [p for p in model.parameters() if p.requires_grad]
        if not params:
            raise ValueError("ShardedDataParallel: model has no trainable parameters")
        self.device = params[0].device
        # Side stream of the optimizer update, at the DEFAULT priority like
        # every other stream of the process: work on streams of different
        # priorities has hung on MI355X hosts (a high-priority update stream
        # measured ~5 ms/step faster, 701 vs 707 ms; not worth a hang).
        self._side = (torch.cuda.Stream(self.device)
                      if self.device.type == "cuda" and (self.overlap or self.world > 1) else None)
        self.buckets: list[_Bucket] = []
        bucket_elems = int(os.environ.get("KGWE_BUCKET_MELEMS", "0")) * 2**20 or bucket_elems
        cur: list[torch.nn.Parameter] = []
        n = 0
        for p in reversed(params):  # backward (gradient-ready) order
            if cur and n + p.numel() > bucket_elems:
                self.buckets.append(self._make_bucket(cur))
                cur, n = [], 0
            cur.append(p)
            n += p.numel()
        self.buckets.append(self._make_bucket(cur))
        self._setup_transposed(model, transposed_weights and self.device.type == "cuda")
        self._bucket_of = {id(p): b for b in self.buckets for p in b.params}
        self._slot = {id(p): (b, o) for b in self.buckets for p, o in zip(b.params, b.offsets)}
        self._hooks = []
        # Ranks whose tensors live on a GPU but whose backend is gloo (the
        # one-GPU rehearsal of the multi-rank path): collectives go through
        # host memory.
        self._host_staged = (self.world > 1 and self.device.type == "cuda"
                             and dist.get_backend(group) == "gloo")
        if self.world > 1 or self.overlap:
            for b in self.buckets:
                for p in b.params:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._grad_ready))
            for mod in model.modules():
                own = [self._bucket_of[id(p)] for p in mod.parameters(recurse=False)
                       if id(p) in self._bucket_of]
                if own:
                    uniq = list({id(b): b for b in own}.values())
                    self._hooks.append(mod.register_forward_pre_hook(
                        lambda _m, _a, bs=uniq: self._wait_params(bs)))

        # bf16 reduce: a linear weight's dW GEMM writes straight into the
        # bucket (kgwe.ops.functional._Linear), so its gradient is never copied.
        self._sinks = []
        if self.world > 1 and self.device.type == "cuda" and reduce_dtype == torch.bfloat16:
            embed = {id(m.weight) for m in model.modules() if isinstance(m, torch.nn.Embedding)}
            for b in self.buckets:
                for p in b.params:
                    if p.dim() == 2 and p.dtype == torch.bfloat16 and id(p) not in embed:
                        p._kgwe_grad_sink = functools.partial(self._grad_sink, p)
                        self._sinks.append(p)

    # ------------------------------------------------------------ layout
    def _make_bucket(self, params) -> _Bucket:
        b = _Bucket()
        b.params = params
        b.offsets = []
        off = 0
        for p in params:
            b.offsets.append(off)
            off += p.numel()
        b.numel = off
        align = self.world * 64  # shard edges 128 B (bf16) / 256 B (fp32) aligned
        b.padded = -(-off // align) * align
        b.shard = b.padded // self.world
        src = torch.zeros(b.padded, dtype=torch.float32, device=self.device)
        for p, o in zip(params, b.offsets):
            src[o:o + p.numel()].copy_(p.detach().reshape(-1))
        b.flat = src.to(torch.bfloat16)
        lo = self.rank * b.shard
        b.master = src[lo:lo + b.shard].clone()
        del src
        b.m = torch.zeros_like(b.master)
        b.v = torch.zeros_like(b.master)
        with torch.no_grad():
            for p, o in zip(params, b.offsets):
                p.data = b.flat[o:o + p.numel()].view(p.shape)
        if self.world > 1:
            b.gfull = torch.zeros(b.padded, dtype=self.reduce_dtype, device=self.device)
            b.gshard = torch.empty(b.shard, dtype=self.reduce_dtype, device=self.device)
        else:
            b.gfull = b.gshard = None
        b.pending = len(params)
        b.seen = set()
        b.rs_work = None
        b.ag_work = None
        b.ready = None
        b.updated = False
        return b

    def _setup_transposed(self, model, enabled: bool) -> None:
        embed = {id(m.weight) for m in model.modules() if isinstance(m, torch.nn.Embedding)}
        for b in self.buckets:
            b.tparams = []
            b.flat_t = None
            if not enabled:
                continue
            b.tparams = [p for p in b.params if p.dim() == 2 and id(p) not in embed
                         and p.shape[0] % 8 == 0 and p.shape[1] % 8 == 0]
            n = sum(p.numel() for p in b.tparams)
            if n == 0:
                continue
            b.flat_t = torch.empty(n, dtype=torch.bfloat16, device=self.device)
            off = 0
            for p in b.tparams:
                p._kgwe_wt = b.flat_t[off:off + p.numel()].view(p.shape[1], p.shape[0])
                off += p.numel()
            self._refresh_transposed(b)

    def _refresh_transposed(self, b: _Bucket) -> None:
        """W^T copies of bucket b's linear weights, on the current stream."""
        for p in b.tparams:
            K.transpose(p.detach(), out=p._kgwe_wt)

    # ------------------------------------------------------------ backward
    @torch.no_grad()
    def _grad_sink(self, p: torch.nn.Parameter, dy2: torch.Tensor, x2: torch.Tensor) -> bool:
        """Called by the linear layer's backward instead of returning dW: the
        weight-gradient GEMM writes this parameter's slice of the
        reduce-scatter bucket itself (no gradient tensor, no copy)."""
        b, o = self._slot[id(p)]
        K.weight_grad(dy2, x2, out=b.gfull[o:o + p.numel()].view(p.shape))
        self._param_done(p, b)
        return True

    @torch.no_grad()
    def _grad_ready(self, p: torch.nn.Parameter) -> None:
        b, o = self._slot[id(p)]
        if self.world > 1:
            if p.grad is None:
                # autograd ran the accumulate node without a gradient: the
                # linear layer's backward gave it to the sink instead, which
                # has already marked the parameter done
                return
            b.gfull[o:o + p.numel()].view(p.shape).copy_(p.grad)
            p.grad = None
        self._param_done(p, b)

    def _param_done(self, p: torch.nn.Parameter, b: _Bucket) -> None:
        if id(p) not in b.seen:
            b.seen.add(id(p))
            b.pending -= 1
            if b.pending == 0:
                self._bucket_complete(b)

    def _bucket_complete(self, b: _Bucket) -> None:
        if not self._armed:
            self._step += 1
            self._armed = True
        if self.world > 1:
            self._reduce_scatter(b)
        if self.overlap:
            # buckets complete in list order; the last one has no backward left to hide behind
            self._update(b, background=b is not self.buckets[-1])

    def _reduce_scatter(self, b: _Bucket) -> None:
        if self._host_staged:
            # gloo is given host tensors only: device -> host with a synchronous
            # copy (which also orders it after the gradients), reduce, and back
            h = b.gfull.cpu()
            out = torch.empty(b.shard, dtype=h.dtype)
            dist.reduce_scatter_tensor(out, h, op=dist.ReduceOp.SUM, group=self.group)
            b.gshard.copy_(out)
            b.rs_work = _Done()
            return
        b.rs_work = dist.reduce_scatter_tensor(b.gshard, b.gfull, op=dist.ReduceOp.SUM,
                                               group=self.group, async_op=True)

    def _all_gather(self, b: _Bucket, s0: int):
        if self._host_staged:
            torch.cuda.current_stream(self.device).synchronize()  # the shard's update has finished
            mine = b.flat[s0:s0 + b.shard].cpu()
            full = torch.empty(b.padded, dtype=mine.dtype)
            dist.all_gather_into_tensor(full, mine, group=self.group)
            b.flat.copy_(full)
            return _Done()
        return dist.all_gather_into_tensor(b.flat, b.flat[s0:s0 + b.shard], group=self.group, async_op=True)

    @torch.no_grad()
    def _update(self, b: _Bucket, background: bool = False) -> None:
        """AdamW on this rank's part of bucket ``b`` (+ all-gather for world
        > 1), on the side stream when there is one; ``background``: capped
        grid (backward still running beside it)."""
        b1, b2 = self.betas
        grid = self.background_grid if background else 0
        side = self._side
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(self.device))
            ctx = torch.cuda.stream(side)
        else:
            ctx = contextlib.nullcontext()
        with ctx:
            for ev in self._fences:
                torch.cuda.current_stream(self.device).wait_event(ev)
            if self.world > 1:
                b.rs_work.wait()
                b.rs_work = None
                s0 = self.rank * b.shard
                self._plan.launch([(b.master, b.gshard, b.m, b.v, b.flat[s0:s0 + b.shard])],
                                  self.lr, b1, b2, self.eps, self.wd, self._step,
                                  grad_scale=1.0 / self.world, max_grid=grid)
                b.ag_work = self._all_gather(b, s0)
                if b.tparams and side is not None:
                    b.ag_work.wait()  # the side stream waits for the gathered weights
                    b.ag_work = None
                    self._refresh_transposed(b)
                    b.ready = torch.cuda.Event()
                    b.ready.record(side)
            else:
                entries = []
                for p, o in zip(b.params, b.offsets):
                    g = p.grad
                    if g is None:
                        continue
                    g = g if g.is_contiguous() else g.contiguous()
                    if side is not None:
                        g.record_stream(side)  # freed by autograd's stream, read here
                    n = p.numel()
                    entries.append((b.master[o:o + n], g.view(-1), b.m[o:o + n], b.v[o:o + n],
                                    b.flat[o:o + n]))
                    p.grad = None
                self._plan.launch(entries, self.lr, b1, b2, self.eps, self.wd, self._step,
                                  max_grid=grid)
                self._refresh_transposed(b)
                if side is not None:
                    b.ready = torch.cuda.Event()
                    b.ready.record(side)
        b.updated = True

    def _wait_params(self, buckets) -> None:
        for b in buckets:
            if b.ag_work is not None:
                b.ag_work.wait()
                b.ag_work = None
            if b.ready is not None:
                torch.cuda.current_stream(self.device).wait_event(b.ready)
                b.ready = None

    def wait_params(self) -> None:
        """Make the current stream wait until every bucket's weights are
        updated and gathered — call before reading parameters outside a
        forward (eval, checkpoint)."""
        self._wait_params(self.buckets)

    # ------------------------------------------------------------ step
    @torch.no_grad()
    def step(self) -> None:
        """Finish the optimizer step: update the buckets no backward hook
        completed (overlap off, or parameters that got no gradient)."""
        if not self._armed:
            self._step += 1
        # Gather order: the next forward reads buckets in reverse (they are in
        # backward order) and collectives on one RCCL stream complete in issue
        # order, so the embedding / first layers' bucket goes first.
        for b in reversed(self.buckets):
            if b.updated:
                continue
            if self.world > 1 and b.rs_work is None:  # some parameter got no gradient
                for p, o in zip(b.params, b.offsets):
                    if id(p) not in b.seen:
                        b.gfull[o:o + p.numel()].zero_()
                self._reduce_scatter(b)
            self._update(b)
        for b in self.buckets:
            b.pending = len(b.params)
            b.seen.clear()
            b.updated = False
        self._armed = False
        self._fences.clear()  # every bucket's writer has waited on them

    def fence_writes(self, event) -> None:
        """The next optimizer update (every bucket, any stream) waits for
        ``event`` before writing master / m / v / weights."""
        if event is not None:
            self._fences.append(event)

    def close(self) -> None:
        """Drain in-flight collectives, remove the hooks and drop the flat
        buffers (e.g. before building another trainer in the same process)."""
        for b in self.buckets:
            for w in (b.rs_work, b.ag_work):
                if w is not None:
                    w.wait()
            b.rs_work = b.ag_work = None
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        for h in self._hooks:
            h.remove()
        self._hooks.clear()

        for b in self.buckets:
            for p in b.params:
                p.grad = None
                if hasattr(p, "_kgwe_wt"):
                    del p._kgwe_wt
                if hasattr(p, "_kgwe_grad_sink"):
                    del p._kgwe_grad_sink
            b.flat = b.master = b.m = b.v = b.gfull = b.gshard = b.flat_t = None
        self.buckets = []
        self._bucket_of.clear()
        self._slot.clear()

    def zero_grad(self) -> None:
        for b in self.buckets:
            for p in b.params:
                p.grad = None

    # ------------------------------------------------------------ checkpoint
    def shard_state(self) -> dict:
        """This rank's optimizer shard (fp32 master, m, v per bucket) + step."""
        return {"step": self._step, "world": self.world, "rank": self.rank,
                "buckets": [{"master": b.master, "m": b.m, "v": b.v} for b in self.buckets]}

    @torch.no_grad()
    def load_shard_state(self, state: dict) -> None:
        if state["world"] != self.world or len(state["buckets"]) != len(self.buckets):
            raise ValueError("checkpoint was written with a different world size / bucket layout")
        self._step = int(state["step"])
        for b, s in zip(self.buckets, state["buckets"]):
            b.master.copy_(s["master"])
            b.m.copy_(s["m"])
            b.v.copy_(s["v"])
            s0 = self.rank * b.shard
            b.flat[s0:s0 + b.shard].copy_(b.master)
            if self.world > 1:
                b.ag_work = dist.all_gather_into_tensor(b.flat, b.flat[s0:s0 + b.shard],
                                                        group=self.group, async_op=True)
        self.wait_params()
        for b in self.buckets:
            self._refresh_transposed(b)
