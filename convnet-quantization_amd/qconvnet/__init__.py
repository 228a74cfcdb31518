"""qconvnet — MI355X-native int8 ConvNet inference path (host runtime).

Layers of this package:
  _lib    ctypes binding of libqconvnet.so (C ABI: include/qconvnet.h)
  ops     tensor-level wrappers (device pointers + current HIP stream)
  quant   host-side qparam / BN-fold / weight-quantization arithmetic
  qmodel  QuantizedConvNet: calibration, packing, the kernel sequence, graphs
  dist    one-process-per-GPU sharded inference with an RCCL logits all-gather
"""
from . import quant  # noqa: F401  (pure numpy, always importable)

__all__ = ["quant"]
