"""Single-launch multi-tensor AdamW with fp32 master weights.

* fp32 parameters (incl. FSDP2 DTensor shards): updated in place.
* bf16 parameters: the optimizer keeps an fp32 master copy (plus fp32 m, v)
  and the kernel writes the rounded result straight back into the bf16
  parameter — the weight the next forward reads — and reads the bf16 gradient
  autograd produced without an up-cast pass.  This is the single-GPU /
  replicated-weights mixed-precision path (288 GB of HBM holds bf16 weights,
  fp32 master and both moments of an 8B model with room for activations).

On a GPU the ``kgwe_adamw_step`` HIP kernel updates 16 tensors per launch
with their pointers passed by value (no device tables).  On CPU the fp32
reference is used.
"""
from __future__ import annotations

import numpy as np
import torch

from . import reference as ref
from ._lib import check, lib, stream

_TENSOR_DT = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"),
                       ("shadow", "<u8"), ("n", "<i8"), ("g_bf16", "<i4"), ("pad", "<i4")])


def _local(t: torch.Tensor) -> torch.Tensor:
    return t.to_local() if hasattr(t, "to_local") else t


class AdamPlan:
    """Launcher for the multi-tensor AdamW kernel.

    ``entries`` = [(p fp32, g fp32|bf16, m fp32, v fp32, shadow bf16|None)], all
    contiguous with equal element counts (checked on the host: the kernel
    trusts the records).  The pointer records go to the kernel by value (16
    per launch), so a launch costs one small numpy record array on the host
    and nothing on the device — cheap enough to issue per gradient bucket."""

    _size_checked = False

    @staticmethod
    def _check(i, p, g, m, v, sh):
        ok = (p.dtype == m.dtype == v.dtype == torch.float32
              and g.dtype in (torch.float32, torch.bfloat16)
              and all(t.is_contiguous() for t in (p, g, m, v))
              and p.numel() == g.numel() == m.numel() == v.numel() > 0
              and all(t.device == p.device for t in (g, m, v))
              and (sh is None or (sh.dtype == torch.bfloat16 and sh.is_contiguous()
                                  and sh.numel() == p.numel() and sh.device == p.device)))
        if not ok:
            raise ValueError(f"AdamW: entry {i} violates the kernel contract "
                             f"(p {p.dtype}/{tuple(p.shape)}, g {g.dtype}/{tuple(g.shape)}, "
                             f"shadow {None if sh is None else (sh.dtype, tuple(sh.shape))})")

    @classmethod
    def records(cls, entries) -> np.ndarray:
        L = lib()
        if not AdamPlan._size_checked:
            assert L.kgwe_adamw_tensor_bytes() == _TENSOR_DT.itemsize
            AdamPlan._size_checked = True
        tens = np.zeros(len(entries), dtype=_TENSOR_DT)
        for i, (p, g, m, v, sh) in enumerate(entries):
            cls._check(i, p, g, m, v, sh)
            tens[i] = (p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                       0 if sh is None else sh.data_ptr(), p.numel(),
                       int(g.dtype == torch.bfloat16), 0)
        return tens

    def launch(self, entries, lr, b1, b2, eps, wd, step, grad_scale=1.0, max_grid=0):
        """max_grid > 0 caps the workgroups per launch (a background update
        beside other kernels; see kgwe_adamw_step)."""
        if not entries:
            return
        p0 = entries[0][0]
        if p0.is_cuda:
            tens = self.records(entries)
            check(lib().kgwe_adamw_step(tens.ctypes.data, len(entries), lr, b1, b2, eps, wd,
                                        step, grad_scale, int(max_grid), stream(p0)), "adamw_step")
            return
        for p, g, m, v, sh in entries:
            gg = g.float() * grad_scale if grad_scale != 1.0 else g.float()
            ref.adamw_(p, gg, m, v, lr, b1, b2, eps, wd, step)
            if sh is not None:
                sh.copy_(p)


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._step = 0
        self._plans: dict[int, AdamPlan] = {}

    def _entries(self, group):
        out = []
        for p in group["params"]:
            if p.grad is None:
                continue
            st = self.state[p]
            lp = _local(p).detach() if hasattr(p, "to_local") else p.data
            if lp.numel() == 0:
                continue
            g = _local(p.grad)
            if lp.dtype == torch.bfloat16:
                if "master" not in st:
                    st["master"] = lp.float()
                master, shadow = st["master"], lp
            elif lp.dtype == torch.float32:
                master, shadow = lp, None
                if g.dtype not in (torch.float32, torch.bfloat16):
                    g = g.float()
            else:
                raise ValueError(f"FusedAdamW: unsupported parameter dtype {lp.dtype}")
            if "exp_avg" not in st:
                st["exp_avg"] = torch.zeros_like(master)
                st["exp_avg_sq"] = torch.zeros_like(master)
            out.append((master, g.contiguous(), st["exp_avg"], st["exp_avg_sq"], shadow))
        return out

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._step += 1
        for gi, group in enumerate(self.param_groups):
            entries = self._entries(group)
            b1, b2 = group["betas"]
            self._plans.setdefault(gi, AdamPlan()).launch(
                entries, group["lr"], b1, b2, group["eps"], group["weight_decay"], self._step)
        return loss
