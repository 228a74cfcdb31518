"""OptimizedCustomQuantization — drop-in for
/root/reference/models/optimized_custom_quantization.py:7-137.

Reference behaviour: the constructor builds a ResNet-50 (torchvision,
IMAGENET1K_V1 weights, :13) and selects a CPU quantization engine (:17-22);
``quantize(model)`` moves it to the CPU, fuses Conv-BN(-ReLU) groups —
stem conv1+bn1+relu, every bottleneck's conv2+bn2+relu, conv3+bn3 and its
downsample conv+BN, the bottleneck's conv1 deliberately left unfused (:52-76)
— then ``quantize_dynamic`` with ``default_dynamic_qconfig`` everywhere
(:108-127).  torch has no dynamic mapping for Conv2d, so the result is the
fused fp32 body plus a dynamic-int8 ``fc``; it is tagged
``quantized`` / ``is_custom_quantized`` (:46-48).  A torchvision Bottleneck
uses ONE ``relu`` module three times, and fusing [conv2, bn2, relu] turns that
shared module into Identity: in the reference's quantized model a bottleneck
is conv1 -> bn1 (no ReLU) -> conv2+bn2+ReLU -> conv3+bn3 -> + identity (no
ReLU).  This class computes exactly that (tests/test_gpu_models.py checks it
against the reference's fusion run by torch on the CPU).

MI355X version: the same fused fp32 body on the GPU (torch / MIOpen: fp32
convolutions are outside this path's int8 scope), and the fc as the HIP
dynamic int8 Linear (device-side ChooseQuantizationParams with reduce_range,
u8 x s8 MFMA, y = fmaf(acc, s_x * s_w, b)) — bit-exact with FBGEMM's
``quantized::linear_dynamic`` for the same fp32 features.  There is no
network here: the constructor builds the restated ResNet-50
(``models.resnet``) with random weights unless a torchvision-layout
``state_dict`` is given.
"""
from __future__ import annotations

import io

import numpy as np
import torch
import torch.nn.functional as F

from models.resnet import resnet50
from qconvnet import ops
from qconvnet import quant as Q
from qconvnet.qmodel import cuda_device
from qconvnet.resnet import _fold, _np


class DynamicFcResNet:
    """Fused fp32 ResNet body on the GPU + dynamic int8 fc (HIP)."""

    def __init__(self, model, device="cuda", reduce_range=True):
        self.device = cuda_device(device)
        self.reduce_range = reduce_range
        self.quantized = True
        self.is_custom_quantized = True
        self.host_io = False
        g = {k: _np(v) for k, v in model.state_dict().items()}
        t = self._t
        w, b = _fold(g, "conv1", "bn1")                       # stem conv1+bn1(+relu)
        self.stem = (t(w), t(b))
        self.blocks = []
        for li in range(1, 5):
            for bi in range(len(getattr(model, f"layer{li}"))):
                p = f"layer{li}.{bi}."
                s = 2 if (bi == 0 and li > 1) else 1
                blk = {"c1": t(g[p + "conv1.weight"]),        # conv1 unfused (:61-63)
                       "bn1": tuple(t(g[p + "bn1." + k]) for k in ("running_mean", "running_var",
                                                                 "weight", "bias")),
                       "c2": tuple(map(t, _fold(g, p + "conv2", p + "bn2"))),
                       "c3": tuple(map(t, _fold(g, p + "conv3", p + "bn3"))), "stride": s}
                if p + "downsample.0.weight" in g:
                    blk["ds"] = tuple(map(t, _fold(g, p + "downsample.0", p + "downsample.1")))
                self.blocks.append(blk)
        fw, fb = g["fc.weight"], g["fc.bias"]
        s_w = Q.qparams_symmetric(fw.min(), fw.max())          # default_weight_observer
        wq = Q.quantize_weight(fw, s_w)
        self.fc = (t(wq), t(np.atleast_1d(s_w)), t(wq.astype(np.int64).sum(1).astype(np.int32)), t(fb))

    def _t(self, a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def features(self, x):
        """fp32 body: stem, bottlenecks, global average pool -> [N, 2048]
        (the bottleneck's shared ReLU is Identity after the reference's fusion)."""
        w, b = self.stem
        x = F.max_pool2d(F.relu(F.conv2d(x, w, b, stride=2, padding=3)), 3, 2, 1)
        for blk in self.blocks:
            bn = blk["bn1"]
            y = F.batch_norm(F.conv2d(x, blk["c1"]), bn[0], bn[1], bn[2], bn[3], False, 0.0, 1e-5)
            y = F.relu(F.conv2d(y, *blk["c2"], stride=blk["stride"], padding=1))
            y = F.conv2d(y, *blk["c3"])
            idn = F.conv2d(x, *blk["ds"], stride=blk["stride"]) if "ds" in blk else x
            x = y + idn
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1).contiguous()

    @torch.no_grad()
    def classify(self, feats):
        """Dynamic int8 fc on [N, 2048] fp32 features (device in, device out)."""
        with torch.cuda.device(self.device):
            w, s, ws, b = self.fc
            return ops.linear_dynamic(feats, w, s, ws, b, self.reduce_range)

    @torch.no_grad()
    def __call__(self, x):
        host = not x.is_cuda
        with torch.cuda.device(self.device):
            y = self.classify(self.features(x.to(self.device, torch.float32)))
            if host or self.host_io:
                return y.cpu()
            torch.cuda.current_stream(self.device).synchronize()
            return y

    forward = __call__

    def eval(self):
        return self

    def to(self, device):
        self.host_io = torch.device(device).type == "cpu"   # compute stays on the GPU
        return self

    def cpu(self):
        self.host_io = True
        return self

    def state_dict(self):
        """Every parameter the executor holds (fused fp32 body, int8 fc)."""
        sd = {"stem.weight": self.stem[0], "stem.bias": self.stem[1]}
        for i, blk in enumerate(self.blocks):
            sd[f"block{i}.conv1.weight"] = blk["c1"]
            for k, v in zip(("mean", "var", "weight", "bias"), blk["bn1"]):
                sd[f"block{i}.bn1.{k}"] = v
            for name in ("c2", "c3", "ds"):
                if name in blk:
                    sd[f"block{i}.{name}.weight"], sd[f"block{i}.{name}.bias"] = blk[name]
        sd["fc.weight_int8"], sd["fc.scale"], _, sd["fc.bias"] = self.fc
        return {k: v.cpu() for k, v in sd.items()}


class OptimizedCustomQuantization:
    def __init__(self, state_dict=None, device="cuda"):
        self.fp32_model = resnet50()
        if state_dict is not None:
            self.fp32_model.load_state_dict(state_dict)
        self.quantized_model = None
        self.device = device
        from qconvnet import _lib
        try:
            _lib.load()
        except _lib.QcnError as e:   # the reference raises when no engine exists (:17-22)
            raise RuntimeError("No supported quantization engine found: " + str(e)) from e

    def quantize(self, model):
        model = model.cpu().eval()
        self.quantized_model = DynamicFcResNet(model, self.device)
        return self.quantized_model

    def get_model_size(self, model):
        """Serialized state_dict size in MB (:129-135), in memory."""
        buf = io.BytesIO()
        torch.save(model.state_dict(), buf)
        return buf.getbuffer().nbytes / (1024 * 1024)
