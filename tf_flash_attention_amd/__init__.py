"""MI355X-native (gfx950) fused flash attention — drop-in for nothingstopsme/tf_flash_attention.

See ``flash_attention.py`` for the public API (mirrors the reference's
``flash_attention/flash_attention.py``) and ``include/fa_api.h`` for the C ABI.
"""
from . import flash_attention
from .flash_attention import (full_1d, causal_1d, local_1d, full_2d, causal_2d, local_2d,  # noqa: F401
                              InvalidArgumentError, InternalError)

__all__ = ["flash_attention", "full_1d", "causal_1d", "local_1d", "full_2d", "causal_2d", "local_2d",
           "InvalidArgumentError", "InternalError"]
