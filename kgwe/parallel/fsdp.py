"""FSDP2 wrapping for the Llama workload, sized for 288 GB HBM3E per GPU.

* fp32 master parameters, sharded across ranks (Zero-3): at 8 ranks an 8B
  model's params + grads + Adam states are 16 GB per GPU; even 1 rank fits
  (128 GB), so the harness runs unchanged from 1 to 8 GPUs (weak scaling:
  per-GPU micro-batch fixed).
* bf16 compute (MixedPrecisionPolicy.param_dtype) with fp32 gradient
  reduce-scatter — one bucket per transformer block, i.e. ~218 MB bf16
  all-gathers / ~436 MB fp32 reduce-scatters for Llama-3-8B: large, few
  collectives, which is what per-link-bound ring collectives over 7 xGMI
  links want.  FSDP2 overlaps the next block's all-gather and the previous
  block's reduce-scatter with compute on separate streams.
"""
from __future__ import annotations

import torch
from torch.distributed.fsdp import MixedPrecisionPolicy, fully_shard

from ..models.llama import Llama


def shard_model(model: Llama, reshard_after_forward: bool = False,
                param_dtype=torch.bfloat16, reduce_dtype=torch.float32) -> Llama:
    """reshard_after_forward=False (ZeRO-2-style gathered weights between
    forward and backward) is the MI355X default: the whole bf16 copy of an 8B
    model is 16 GB, ~6 % of one GPU's 288 GB, and keeping it resident removes
    the backward re-all-gather — a third of FSDP's collective traffic and of
    its copy-in/copy-out kernels."""
    mp = MixedPrecisionPolicy(param_dtype=param_dtype, reduce_dtype=reduce_dtype)
    for layer in model.layers:
        fully_shard(layer, mp_policy=mp, reshard_after_forward=reshard_after_forward)
    # The root unit holds embeddings, final norm and the LM head; its params
    # stay gathered through backward (no re-gather for the LM head grad).
    fully_shard(model, mp_policy=mp, reshard_after_forward=False)
    return model
