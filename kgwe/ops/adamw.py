"""Single-launch multi-tensor AdamW over fp32 (FSDP-sharded) parameters.

Works on plain tensors and on FSDP2 DTensor parameters (updates the local
shard in place).  On a GPU the ``kgwe_adamw_step`` HIP kernel does the whole
update in one launch; the pointer/chunk tables are rebuilt only when the
gradient storage moves.  On CPU the fp32 reference is used.
"""
from __future__ import annotations

import numpy as np
import torch

from . import reference as ref
from ._lib import check, lib, stream

_TENSOR_DT = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"),
                       ("shadow", "<u8"), ("n", "<i8")])
_CHUNK_DT = np.dtype([("tensor", "<i4"), ("pad", "<i4"), ("start", "<i8")])


def _local(t: torch.Tensor) -> torch.Tensor:
    return t.to_local() if hasattr(t, "to_local") else t


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._step = 0
        self._tables: dict = {}

    def _group_tensors(self, group):
        ps, gs, ms, vs = [], [], [], []
        for p in group["params"]:
            if p.grad is None:
                continue
            st = self.state[p]
            lp = _local(p).detach() if hasattr(p, "to_local") else p.data
            if "exp_avg" not in st:
                st["exp_avg"] = torch.zeros_like(lp, dtype=torch.float32)
                st["exp_avg_sq"] = torch.zeros_like(lp, dtype=torch.float32)
            g = _local(p.grad)
            if lp.numel() == 0:
                continue
            ps.append(lp)
            gs.append(g if g.dtype == torch.float32 else g.float())
            ms.append(st["exp_avg"])
            vs.append(st["exp_avg_sq"])
        return ps, gs, ms, vs

    def _device_tables(self, gi, ps, gs, ms, vs):
        key = tuple(t.data_ptr() for t in gs) + tuple(t.data_ptr() for t in ps)
        cached = self._tables.get(gi)
        if cached is not None and cached[0] == key:
            return cached[1], cached[2], cached[3]
        L = lib()
        chunk = L.kgwe_adamw_chunk_elems()
        tens = np.zeros(len(ps), dtype=_TENSOR_DT)
        chunks = []
        for i, (p, g, m, v) in enumerate(zip(ps, gs, ms, vs)):
            # Kernel contract: fp32, contiguous, equal element counts.
            if not (p.dtype == g.dtype == m.dtype == v.dtype == torch.float32
                    and p.is_contiguous() and g.is_contiguous()
                    and p.numel() == g.numel() == m.numel() == v.numel()):
                raise ValueError(f"FusedAdamW: tensor {i} violates the kernel contract "
                                 f"(p {p.dtype}/{p.shape}, g {g.dtype}/{g.shape})")
            tens[i] = (p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), 0, p.numel())
            for s in range(0, p.numel(), chunk):
                chunks.append((i, 0, s))
        ch = np.array(chunks, dtype=_CHUNK_DT)
        dev = ps[0].device
        # Pinned staging + async H2D on the compute stream: no host sync.  The
        # staging buffers stay referenced by the cache entry until the next
        # rebuild of this group, after which the stream has long consumed them.
        t_host = torch.from_numpy(tens.view(np.uint8).copy())
        c_host = torch.from_numpy(ch.view(np.uint8).copy())
        if dev.type == "cuda":
            t_host, c_host = t_host.pin_memory(), c_host.pin_memory()
        t_dev = t_host.to(dev, non_blocking=True)
        c_dev = c_host.to(dev, non_blocking=True)
        self._tables[gi] = (key, t_dev, c_dev, len(chunks), t_host, c_host)
        return t_dev, c_dev, len(chunks)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._step += 1
        for gi, group in enumerate(self.param_groups):
            ps, gs, ms, vs = self._group_tensors(group)
            if not ps:
                continue
            b1, b2 = group["betas"]
            if ps[0].is_cuda:
                t_dev, c_dev, n = self._device_tables(gi, ps, gs, ms, vs)
                check(lib().kgwe_adamw_step(t_dev.data_ptr(), c_dev.data_ptr(), n,
                                            group["lr"], b1, b2, group["eps"],
                                            group["weight_decay"], self._step, 1.0,
                                            stream(ps[0])), "adamw_step")
            else:
                for p, g, m, v in zip(ps, gs, ms, vs):
                    ref.adamw_(p, g, m, v, group["lr"], b1, b2, group["eps"],
                               group["weight_decay"], self._step)
        return loss
