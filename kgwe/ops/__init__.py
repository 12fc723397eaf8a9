"""gfx950 HIP kernels for the training hot path + their fp32 references."""
from .functional import cross_entropy, rmsnorm, rope_qkv, swiglu  # noqa: F401
from .attn import attention  # noqa: F401
from .adamw import FusedAdamW  # noqa: F401
