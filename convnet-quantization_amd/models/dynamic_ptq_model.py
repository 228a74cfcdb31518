"""DynamicPTQModel — drop-in for /root/reference/models/dynamic_ptq_model.py:218-317.

Reference behaviour: duck-typed model (load_state_dict, eval, cpu, to, forward,
__call__ :234-279); quantize() folds conv_i+bn_i and fc1+bn7 (:289-299) then
``quantize_dynamic({Linear, Conv2d}, qint8)`` (:302-306).  torch has no dynamic
mapping for Conv2d, so the effect is BN-folded fp32 convs + dynamic int8
fc1/fc2.

MI355X version: fc1 and fc2 run ``quantized::linear_dynamic`` semantics in the
HIP kernel (device-side min/max -> ChooseQuantizationParams with reduce_range
-> LEGACY quantize -> u8 x s8 MFMA GEMM -> y = fmaf(acc, s_x*s_w, b)), bit-exact
with FBGEMM for the same fp32 input.  The six fp32 convolutions are the
reference's fp32 ops and run through torch (MIOpen) on the same device — an
fp32 conv is outside this path's int8 scope (SURVEY §8(f) row 1 lists the
batch-exact dynamic path as the next step).  The ResNet-50
``CustomDynamicQuantization`` of :13-216 needs torchvision and a weight
download and is out of scope.
"""
from __future__ import annotations

import io

import numpy as np
import torch
import torch.nn.functional as F

from models.baseline_model import CONV_TABLE, SimpleConvNet, load_checkpoint_state
from qconvnet import ops
from qconvnet import quant as Q
from qconvnet.qmodel import cuda_device, fold_state_dict

F32 = np.float32


class DynamicQuantConvNet:
    """fp32 convs (+ optional BN fold) and dynamic-int8 fc1/fc2 on the GPU."""

    def __init__(self, state_dict, fold=True, device="cuda", reduce_range=True):
        self.device = cuda_device(device)
        self.reduce_range = reduce_range
        self.sharded = False   # True: batch-exact across ranks (see _range)
        self.quantized = True
        self.host_io = False
        g = {k: v.detach().cpu().numpy() for k, v in state_dict.items() if torch.is_tensor(v)}
        if fold:
            f = fold_state_dict(state_dict)
            convs = [(f[f"conv{i}.w"], f[f"conv{i}.b"], None) for i in range(1, 7)]
            fc1w, fc1b, self.bn7 = f["fc1.w"], f["fc1.b"], None
        else:
            convs = [(g[f"conv{i}.weight"], g[f"conv{i}.bias"],
                      tuple(g[f"bn{i}.{k}"] for k in ("running_mean", "running_var", "weight", "bias")))
                     for i in range(1, 7)]
            fc1w, fc1b = g["fc1.weight"], g["fc1.bias"]
            # bn7 in ATen's CPU op order (fma(x, alpha, beta')), so the dynamic
            # fc2 sees bit-identical input to the reference's CPU model
            self.bn7 = tuple(self._t(a) for a in Q.bn_eval_affine(
                *(g[f"bn7.{k}"] for k in ("running_mean", "running_var", "weight", "bias"))))
        self.convs = [(self._t(w), self._t(b), tuple(self._t(a) for a in bn) if bn else None)
                      for w, b, bn in convs]
        self.fc = []
        for w, b in ((fc1w, fc1b), (g["fc2.weight"], g["fc2.bias"])):
            s_w = Q.qparams_symmetric(w.min(), w.max())     # default_weight_observer
            wq = Q.quantize_weight(w, s_w)
            self.fc.append((self._t(wq), self._t(np.atleast_1d(s_w)),
                            self._t(wq.astype(np.int64).sum(1).astype(np.int32)), self._t(b)))

    def _t(self, a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def _range(self, x):
        """None (each call uses its own batch range, quantize_dynamic's
        semantics) unless ``sharded`` is set — this process runs one shard of a
        batch split over the ranks (qconvnet.dist.sharded_forward): then the
        range is all-reduced so every shard quantizes exactly as the whole
        batch would (one 2-float RCCL all-reduce per dynamic Linear; every rank
        must make the same calls)."""
        import torch.distributed as dist
        if not self.sharded or not (dist.is_available() and dist.is_initialized()) \
                or dist.get_world_size() == 1:
            return None
        from qconvnet.dist import global_minmax
        return global_minmax(ops.minmax_range(x))

    @torch.no_grad()
    def __call__(self, x):
        with torch.cuda.device(self.device):   # ops launch on this device's current stream
            return self._forward(x)

    def features(self, x):
        """fp32 convs (+BN, ReLU, pools) -> the [N, 4096] NCHW-flatten fc1 input."""
        for i, (w, b, bn) in enumerate(self.convs):
            x = F.conv2d(x, w, b, padding=1)
            if bn is not None:
                x = F.batch_norm(x, bn[0], bn[1], bn[2], bn[3], False, 0.0, 1e-5)
            x = F.relu(x)
            if CONV_TABLE[i][2]:
                x = F.max_pool2d(x, 2, 2)
        return x.reshape(x.shape[0], -1).contiguous()

    @torch.no_grad()
    def classify(self, feats):
        """dynamic-int8 fc1 -> [bn7] -> ReLU -> dynamic-int8 fc2 on [N, 4096]
        fp32 features (device tensor in, device logits out, no sync)."""
        with torch.cuda.device(self.device):
            w, s, ws, b = self.fc[0]
            x = ops.linear_dynamic(feats, w, s, ws, b, self.reduce_range, minmax=self._range(feats))
            if self.bn7 is not None:
                x = ops.channel_affine(x, self.bn7[0], self.bn7[1], relu=True)
            else:
                x = F.relu(x).contiguous()
            w, s, ws, b = self.fc[1]
            return ops.linear_dynamic(x, w, s, ws, b, self.reduce_range, minmax=self._range(x))

    def _forward(self, x):
        host = not x.is_cuda
        x = x.to(self.device, torch.float32)
        y = self.classify(self.features(x))
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


class DynamicPTQModel:
    def __init__(self, device="cuda"):
        self.fp32_model = SimpleConvNet()
        self.quantized_model = None
        self.device = device

    def load_state_dict(self, state_dict):
        self.fp32_model.load_state_dict(load_checkpoint_state(state_dict))

    def eval(self):
        (self.quantized_model or self.fp32_model).eval()
        return self

    def cpu(self):
        if self.quantized_model is not None:
            self.quantized_model.cpu()
        else:
            self.fp32_model = self.fp32_model.cpu()
        return self

    def to(self, device):
        if self.quantized_model is not None:
            self.quantized_model.to(device)
        else:
            self.fp32_model = self.fp32_model.to(device)
        return self

    def forward(self, x):
        if self.quantized_model is not None:
            return self.quantized_model(x)
        return self.fp32_model(x)

    def __call__(self, x):
        return self.forward(x)

    def quantize(self):
        self.fp32_model = self.fp32_model.cpu().eval()
        self.quantized_model = DynamicQuantConvNet(self.fp32_model.state_dict(), fold=True,
                                                   device=self.device)
        return self.quantized_model

    def get_model_size(self):
        buf = io.BytesIO()
        torch.save([t for fc in self.quantized_model.fc for t in fc], buf)
        return buf.tell() / (1024 * 1024)
