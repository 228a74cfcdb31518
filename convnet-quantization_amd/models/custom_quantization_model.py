"""CustomQuantizationModel — drop-in for
/root/reference/models/custom_quantization_model.py:145-261 (BASELINE config 2),
and CustomQuantizedResNet50 (:104-148, config 5) below.

Reference behaviour: engine select (fbgemm, else qnnpack, else RuntimeError,
:155-161); load_state_dict (:163-167); quantize() = eval -> cpu ->
fuse_modules [conv_i, bn_i] x6 + [fc1, bn7] (:180-190) ->
CustomQuantizedSimpleConvNet, where every conv and fc1 is wrapped
QuantStub -> op -> DeQuantStub (:34-58), ReLU / max-pool run in fp32 outside the
wrapper (:237-252) and fc2 stays fp32 (:219).  As shipped, the stubs are never
converted, so the reference model is still fp32.

Here the stubs are live: quantize() calibrates every stub (MinMax observers,
per-tensor affine activations, symmetric s8 weights) and builds the per-layer
QDQ int8 model on the MI355X (``QuantizedConvNet`` in "qdq" mode) — each
conv's epilogue requantizes to its own output qparams and then performs the
dequantize -> ReLU -> [pool] -> quantize(next stub) hand-off in registers, with
torch.ao's fp32 op order, so the integer chain is bit-exact with torch.ao
(fbgemm) and only the fp32 fc2 GEMM differs by summation order.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from models.baseline_model import SimpleConvNet, load_checkpoint_state
from qconvnet import data
from qconvnet.qmodel import QuantizedConvNet, build_qspec, calibrate, fold_state_dict


class CustomQuantizationModel(nn.Module):
    """An nn.Module like the reference's (:145): ``model`` (the fp32
    SimpleConvNet) is its submodule, so state_dict() / parameters() / train()
    / eval() behave as there; ``quantized_model`` is the MI355X executor."""

    def __init__(self, device="cuda"):
        super().__init__()
        self.model = SimpleConvNet()
        self.quantized_model = None
        self.is_custom_quantized = True
        self.device = device
        # the reference selects a CPU quantization engine and raises if none
        # exists; the MI355X path needs the HIP library instead
        from qconvnet import _lib
        try:
            _lib.load()
        except _lib.QcnError as e:
            raise RuntimeError("No supported quantization engine found: " + str(e)) from e

    def load_state_dict(self, state_dict):
        self.model.load_state_dict(load_checkpoint_state(state_dict))

    def quantize(self, calibration_data_loader=None, per_channel=False, calibration_device="cpu",
                 max_batches=None):
        self.model.eval()
        folded = fold_state_dict(self.model.state_dict())
        batches = data.calibration_batches(calibration_data_loader, max_batches)
        ranges = calibrate(folded, batches, calibration_device)
        spec = build_qspec(folded, ranges, "qdq", per_channel)
        self.quantized_model = QuantizedConvNet(spec, self.device)
        return self.quantized_model

    def forward(self, x):
        if self.quantized_model is not None:
            return self.quantized_model(x)
        return self.model(x)

    def to(self, device):
        if self.quantized_model is not None:
            self.quantized_model.to(device)   # compute stays on the GPU; host I/O
        else:
            self.model.to(device)
        return self

    def cpu(self):
        return self.to("cpu")


class CustomQuantizedResNet50(nn.Module):
    """Drop-in for CustomQuantizedResNet50
    (/root/reference/models/custom_quantization_model.py:104-148): wraps a
    torchvision-layout ResNet (models.resnet.resnet50 or a torchvision model) —
    stem conv + maxpool, the CustomQuantizedBottleneck blocks (:60-102) with
    their float-domain residual add, avgpool and fc — as the static int8
    MI355X executor ``qconvnet.resnet.QuantizedResNet`` (BN folded, per-channel
    s8 weights, MinMax-calibrated u8 activations).  ``calibration_batches``:
    an iterable of fp32 [N,3,H,W] tensors (or (x, y) pairs); default 32
    synthetic ImageNet-normalised 224x224 images.  ``conv1_scale`` is accepted
    for signature compatibility; the reference never uses it.

    mode="static" (default): the static int8 executor above.  mode="reference":
    the reference's own block semantics (:60-143) with its per-layer stubs
    live — every conv QuantStub -> int8 conv -> DeQuantStub, BN / ReLU /
    max-pool / residual add / avg-pool in fp32 between them, nothing folded —
    as ``qconvnet.resnet_qdq.QuantizedResNetQDQ``."""

    def __init__(self, model, conv1_scale=1.0, calibration_batches=None, device="cuda",
                 per_channel=True, mode="static"):
        from qconvnet.resnet import quantize_resnet
        from qconvnet.resnet_qdq import quantize_resnet_reference
        from models.resnet import synthetic_images
        if mode not in ("static", "reference"):
            raise ValueError(f"unknown mode {mode!r}")
        super().__init__()
        if calibration_batches is None:
            calibration_batches = [torch.from_numpy(synthetic_images(32, 1))]
        batches = [b[0] if isinstance(b, (tuple, list)) else b for b in calibration_batches]
        self.conv1_scale = conv1_scale
        self.mode = mode
        build = quantize_resnet if mode == "static" else quantize_resnet_reference
        self.quantized_model = build(model.eval(), batches, device, per_channel)

    def forward(self, x):
        return self.quantized_model(x)

    def train(self, mode=True):
        if mode:
            raise RuntimeError("CustomQuantizedResNet50 is inference-only")
        return super().train(False)

    def to(self, device):
        self.quantized_model.to(device)
        return self

    def cpu(self):
        self.quantized_model.cpu()
        return self


def test_custom_quantization():
    model = CustomQuantizationModel()
    x = torch.randn(1, 3, 32, 32)
    y = model(x)
    print(f"Input shape: {tuple(x.shape)}\nOutput shape: {tuple(y.shape)}")
    return model


if __name__ == "__main__":
    test_custom_quantization()
