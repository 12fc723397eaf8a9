"""ctypes binding of ``libkgwe_ops.so`` (hand-written gfx950 HIP kernels).

The library exports a plain C ABI; every launcher takes device pointers and
the caller's ``hipStream_t`` so launches land on PyTorch's current stream
(and are therefore captured by ``torch.cuda.graph``).

Loading policy: on a machine with a GPU the library MUST load — a missing or
stale build raises instead of silently falling back to eager PyTorch.  On a
CPU-only host the ops dispatch to the fp32 PyTorch references in
``kgwe.ops.reference`` (used by the CPU test-suite and the control plane).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

# KGWE_OPS_LIB: load another build of the kernels (same-box A/B runs only).
_LIB_PATH = (Path(os.environ["KGWE_OPS_LIB"]) if os.environ.get("KGWE_OPS_LIB")
             else Path(__file__).resolve().parent.parent / "_lib" / "libkgwe_ops.so")
_lib = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_float = ctypes.c_float

_SIGS = {
    "kgwe_rmsnorm_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_int, c_int, c_float, c_void_p]),
    "kgwe_rmsnorm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "kgwe_rmsnorm_bwd_grid": (c_int, [c_int]),
    "kgwe_swiglu_fwd": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int, c_void_p]),
    "kgwe_swiglu_bwd": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                c_int64, c_int64, c_int, c_void_p]),
    "kgwe_swiglu_bwd_t": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                  c_int64, c_void_p, c_int64, c_int, c_void_p]),
    "kgwe_rope_qkv_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_int64, c_int, c_int, c_int, c_int, c_void_p]),
    "kgwe_rope_qkv_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_int64, c_int, c_int, c_int, c_int, c_void_p]),
    "kgwe_cross_entropy_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                       c_int64, c_void_p]),
    "kgwe_cross_entropy_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int64, c_int64, c_int64, c_void_p]),
    "kgwe_adamw_step": (c_int, [c_void_p, c_int, c_float, c_float, c_float, c_float,
                                c_float, c_int, c_float, c_int, c_void_p]),
    "kgwe_transpose_bf16": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
    "kgwe_adamw_chunk_elems": (c_int, []),
    "kgwe_decode_rope_append": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "kgwe_decode_attn": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                 c_int, c_int, c_int, c_int, c_int, c_float, c_void_p]),
    "kgwe_decode_attn_rope": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p]),
    "kgwe_decode_attn_workspace": (c_int64, [c_int, c_int, c_int, c_int]),
    "kgwe_decode_attn_splits": (c_int, [c_int, c_int, c_int]),
    "kgwe_decode_gemv": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                 c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "kgwe_decode_argmax_finish": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "kgwe_decode_argmax_slots": (c_int, [c_int, c_int, c_int]),
    "kgwe_decode_skinny": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "kgwe_decode_skinny_workspace": (c_int64, [c_int, c_int, c_int, c_int]),
    "kgwe_decode_skinny_blocks": (c_int, [c_int]),
    "kgwe_decode_skinny_slices": (c_int, [c_int, c_int, c_int]),
    "kgwe_decode_skinny_max_m": (c_int, []),
    "kgwe_adamw_tensor_bytes": (c_int, []),
    "kgwe_wgrad_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                c_int, c_int, c_int, c_int, c_void_p]),
    "kgwe_wgrad_splits": (c_int, [c_int, c_int, c_int]),
    "kgwe_wgrad_workspace": (c_int64, [c_int, c_int, c_int]),
}
_OPTIONAL_SIGS = {
    "kgwe_flash_attn_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_int, c_int, c_int, c_int, c_int, c_float, c_int,
                                    c_void_p]),
    "kgwe_flash_attn_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int, c_int, c_int, c_int, c_int, c_float,
                                    c_int, c_void_p]),
    "kgwe_flash_attn_bwd_workspace": (c_int64, [c_int, c_int, c_int, c_int, c_int]),
}


class KernelLibraryMissing(RuntimeError):
    pass


def gpu_available() -> bool:
    return torch.cuda.is_available()


def lib():
    """Return the loaded library, raising if it is missing on a GPU host."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        raise KernelLibraryMissing(
            f"{_LIB_PATH} not built; run `python -m kgwe._build` (hipcc, gfx950)")
    L = ctypes.CDLL(str(_LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in _OPTIONAL_SIGS.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
    _lib = L
    return L


def has_symbol(name: str) -> bool:
    try:
        return getattr(lib(), name, None) is not None
    except KernelLibraryMissing:
        return False


def stream(t: torch.Tensor | None = None) -> int:
    dev = t.device if t is not None else None
    return torch.cuda.current_stream(dev).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def use_hip(*tensors: torch.Tensor) -> bool:
    """True when the tensors live on a GPU: then the HIP kernels are mandatory."""
    return any(t is not None and t.is_cuda for t in tensors)
