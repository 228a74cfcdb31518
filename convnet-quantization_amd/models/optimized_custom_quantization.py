"""OptimizedCustomQuantization — placeholder for
/root/reference/models/optimized_custom_quantization.py:7-137.

The reference builds torchvision's ResNet-50 with IMAGENET1K_V1 weights in its
constructor (:13) — a network download — fuses some Conv-BN(-ReLU) groups and
quantize_dynamic's only the final fc (:41-45).  torchvision is not installed
and there is no network here, so this class cannot be constructed the same
way.  The int8 ResNet-style bottleneck path at 3x224x224 with per-channel
weights (BASELINE config 5) is the next row of SURVEY.md §8(f); until it lands
this raises a clear error instead of silently falling back.
"""
from __future__ import annotations


class OptimizedCustomQuantization:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            "OptimizedCustomQuantization needs torchvision ResNet-50 IMAGENET1K_V1 weights "
            "(network download) and the int8 bottleneck kernels of SURVEY.md §8(f) row 2, "
            "which are not part of this round's MI355X path")
