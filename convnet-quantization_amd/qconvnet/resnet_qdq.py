"""ResNet bottleneck network in the reference's own semantics — SURVEY §8(f)2,
BASELINE config 5, ``CustomQuantizedResNet50(mode="reference")``.

Reference: ``CustomQuantizedBottleneck`` / ``CustomQuantizedResNet50``
(/root/reference/models/custom_quantization_model.py:34-45, 60-143).  Every
conv (stem, conv1-3, downsample) and the fc is wrapped QuantStub -> op ->
DeQuantStub; BN, ReLU, the stem's max-pool, the float-domain residual add
(:95-101) and the average pool run in fp32 BETWEEN the int8 ops.  Nothing is
folded.  As shipped the reference never converts those stubs (its model
stays fp32); here they are live, as torch.ao eager prepare/convert makes them:
each stub's MinMax observer sees the fp32 network's activations during
calibration, each int8 conv requantizes to its own output observer's qparams
(no ReLU in the int8 op), per-channel symmetric s8 weights.  The outer
QuantStub / DeQuantStub pair (:107-108) stays an identity — converted, it
would feed conv1's own QuantStub a quantized tensor, which torch rejects.
The oracle is ``oracle.qref.resnet_qdq_forward``, pinned to torch.ao by
tests/golden/net_resnet_qdq.npz (oracle/make_golden.py gen_resnet_qdq_net).

Device pipeline per forward (every launch a hand-written HIP kernel):
  stem_pack (stem QuantStub + 7-tap rows) -> conv 7x1 -> dq_bn_relu_maxpool
  (fp32 block input + its u8 quantize) -> per block [conv1 -> dq_bn_q ->
  conv2 -> dq_bn_q -> conv3 (, downsample conv) -> qdq_join (fp32 block
  output + next block's u8 input)] -> avgpool_f32 -> fc QuantStub -> int8 fc
  -> DeQuantStub.  Activations between blocks are fp32 NHWC (the identity
  path of the next block reads them), every conv input is u8 NHWC.
"""
from __future__ import annotations

import re

import numpy as np
import torch
import torch.nn.functional as F

from . import ops
from . import quant as Q
from .qmodel import _DevLayer, _Range, _weight_scale, cuda_device

F32 = np.float32


def _np(v):
    return v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)


def unfolded_state(sd):
    """torchvision-layout ResNet state_dict -> {"stem": conv, "blocks": [{c1, c2,
    c3[, ds]}], "fc": (w, b)}, conv = (w, stride, pad, bn), bn = (mean, var,
    gamma, beta, eps) — nothing folded (the reference keeps BN in fp32)."""
    g = {k: _np(v) for k, v in sd.items()}

    def bn(p):
        return (g[p + ".running_mean"], g[p + ".running_var"], g[p + ".weight"], g[p + ".bias"], 1e-5)

    out = {"stem": (np.asarray(g["conv1.weight"], F32), 2, 3, bn("bn1")), "blocks": []}
    keys = sorted({(int(m.group(1)), int(m.group(2)))
                   for k in g for m in [re.match(r"layer(\d)\.(\d+)\.conv1\.weight$", k)] if m})
    for li, bi in keys:
        p = f"layer{li}.{bi}."
        s = 2 if (bi == 0 and li > 1) else 1
        blk = {}
        for j, (st, pad) in enumerate(((1, 0), (s, 1), (1, 0)), start=1):
            blk[f"c{j}"] = (np.asarray(g[p + f"conv{j}.weight"], F32), st, pad, bn(p + f"bn{j}"))
        if p + "downsample.0.weight" in g:
            blk["ds"] = (np.asarray(g[p + "downsample.0.weight"], F32), s, 0, bn(p + "downsample.1"))
        out["blocks"].append(blk)
    out["fc"] = (np.asarray(g["fc.weight"], F32), np.asarray(g["fc.bias"], F32))
    return out


def calibrate(net, batches, device="cpu"):
    """The observers of the live-stub model: fp32 forward of the unfolded net
    (torch's own conv / batch_norm / pooling ops, as torch.ao's prepared model
    runs during calibration) recording, per int8 op, its QuantStub's input
    range ("<name>.in") and its output range ("<name>.out")."""
    dev = torch.device(device)

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    rng = {}

    def obs(key, x):
        if key not in rng:
            rng[key] = _Range(dev)
        rng[key](x)

    def qconv(name, x, layer):
        w, st, pad, (m, v, g, b, eps) = layer
        obs(name + ".in", x)
        y = F.conv2d(x, t(w), None, stride=st, padding=pad)
        obs(name + ".out", y)
        return F.batch_norm(y, t(m), t(v), t(g), t(b), False, 0.0, eps)

    with torch.no_grad():
        for xb in batches:
            x = xb.to(dev, torch.float32)
            x = F.max_pool2d(F.relu(qconv("stem", x, net["stem"])), 3, 2, 1)
            for i, blk in enumerate(net["blocks"]):
                out = F.relu(qconv(f"b{i}.c1", x, blk["c1"]))
                out = F.relu(qconv(f"b{i}.c2", out, blk["c2"]))
                out = qconv(f"b{i}.c3", out, blk["c3"])
                idn = qconv(f"b{i}.ds", x, blk["ds"]) if "ds" in blk else x
                x = F.relu(out + idn)
            x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
            obs("fc.in", x)
            obs("fc.out", F.linear(x, t(net["fc"][0]), t(net["fc"][1])))
    return {k: r.values() for k, r in rng.items()}


def build_spec(net, ranges, per_channel=True):
    """Host description of the live-stub int8 net (numpy) — the format
    oracle.qref.resnet_qdq_forward reads."""
    def conv(name, layer):
        w, st, pad, (m, v, g, b, eps) = layer
        s_w = _weight_scale(w, per_channel)
        s_x, z_x = Q.qparams_affine(*ranges[name + ".in"])
        s_y, z_y = Q.qparams_affine(*ranges[name + ".out"])
        return dict(w=Q.quantize_weight(w, s_w), b=np.zeros(w.shape[0], F32), s_w=s_w, s_x=s_x,
                    z_x=z_x, s_y=s_y, z_y=z_y, stride=(st, st), pad=(pad, pad),
                    bn=Q.bn_eval_affine(m, v, g, b, eps))

    spec = {"per_channel": bool(per_channel), "stem": conv("stem", net["stem"]), "blocks": []}
    for i, blk in enumerate(net["blocks"]):
        e = {k: conv(f"b{i}.{k}", blk[k]) for k in ("c1", "c2", "c3")}
        e["ds"] = conv(f"b{i}.ds", blk["ds"]) if "ds" in blk else None
        spec["blocks"].append(e)
    w, b = net["fc"]
    s_w = _weight_scale(w, per_channel)
    s_x, z_x = Q.qparams_affine(*ranges["fc.in"])
    s_y, z_y = Q.qparams_affine(*ranges["fc.out"])
    spec["fc"] = dict(w=Q.quantize_weight(w, s_w), b=np.asarray(b, F32), s_w=s_w, s_x=s_x, z_x=z_x,
                      s_y=s_y, z_y=z_y)
    return spec


def quantize_resnet_reference(model, calib_batches, device="cuda", per_channel=True,
                              calibration_device="cpu"):
    """fp32 ResNet (torchvision layout) -> QuantizedResNetQDQ on `device`."""
    net = unfolded_state(model.state_dict())
    ranges = calibrate(net, calib_batches, calibration_device)
    return QuantizedResNetQDQ(build_spec(net, ranges, per_channel), device)


class QuantizedResNetQDQ:
    """Duck-typed live-stub int8 ResNet (eval / cpu / to / __call__): fp32
    [N,3,H,W] in, fp32 [N,num_classes] logits out."""

    def __init__(self, spec, device="cuda"):
        self.spec = spec
        self.device = cuda_device(device)
        self.quantized = True
        self.host_io = False
        self._upload()

    def _t(self, a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def _layer(self, e, stem=False):
        d = _DevLayer()
        w = np.asarray(e["w"], np.int8)
        if stem:
            w = ops.stem_weight_rows(w)
            d.sy, d.sx, d.py, d.px = e["stride"][0], 1, e["pad"][0], 0
        else:
            (d.sy, d.sx), (d.py, d.px) = e["stride"], e["pad"]
        packed, wsum = ops.pack_conv_kmajor(w)
        d.cout, _, d.kh, d.kw = w.shape
        u, v, mult = Q.epilogue_constants(e["s_x"], e["s_w"], e["s_y"], e["b"])
        d.w = self._t(packed)
        d.u, d.v, d.mult = self._t(u), self._t(v), self._t(mult)
        d.corr = self._t(((128 - int(e["z_x"])) * wsum.astype(np.int64)).astype(np.int32))
        d.z_x, d.s_x, d.z_y, d.s_y, d.relu = int(e["z_x"]), F32(e["s_x"]), int(e["z_y"]), F32(e["s_y"]), False
        d.alpha, d.beta = (self._t(np.asarray(a, F32)) for a in e["bn"])
        return d

    def _upload(self):
        sp = self.spec
        self.stem = self._layer(sp["stem"], stem=True)
        self.blocks = []
        for e in sp["blocks"]:
            b = {k: (self._layer(e[k]) if e.get(k) is not None else None) for k in ("c1", "c2", "c3", "ds")}
            if b["ds"] is not None and (b["ds"].s_x, b["ds"].z_x) != (b["c1"].s_x, b["c1"].z_x):
                raise ValueError("conv1's and the downsample's QuantStubs observe the same tensor "
                                 "and must agree on their qparams")
            self.blocks.append(b)
        fc = sp["fc"]
        d = _DevLayer()
        w = np.asarray(fc["w"], np.int8)
        u, v, mult = Q.epilogue_constants(fc["s_x"], fc["s_w"], fc["s_y"], fc["b"])
        d.w = self._t(w)
        d.u, d.v, d.mult = self._t(u), self._t(v), self._t(mult)
        d.corr = self._t(((128 - int(fc["z_x"])) * w.astype(np.int64).sum(1)).astype(np.int32))
        d.s_x, d.z_x, d.z_y, d.s_y = F32(fc["s_x"]), int(fc["z_x"]), int(fc["z_y"]), F32(fc["s_y"])
        self.fc = d
        self.num_classes = w.shape[0]

    def run(self, x, keep=False):
        if x.device != self.device:
            raise ValueError(f"input on {x.device}, model on {self.device}")
        with torch.cuda.device(self.device):
            return self._run(x, keep)

    def _run(self, x, keep):
        inter = {}
        st = self.stem
        first = self.blocks[0]["c1"] if self.blocks else None
        y = ops.conv(ops.stem_pack(x, st.s_x, st.z_x), st.z_x, st)
        xf, xq = ops.dq_bn_relu_maxpool(y, st.s_y, st.z_y, st.alpha, st.beta,
                                        first.s_x if first else None, first.z_x if first else 0)
        if keep:
            inter["stem.q"], inter["stem"] = y, xf
        for i, b in enumerate(self.blocks):
            c1, c2, c3, ds = b["c1"], b["c2"], b["c3"], b["ds"]
            y1 = ops.conv(xq, c1.z_x, c1)
            y2 = ops.conv(ops.dq_bn_q(y1, c1.s_y, c1.z_y, c1.alpha, c1.beta, True, c2.s_x, c2.z_x), c2.z_x, c2)
            y3 = ops.conv(ops.dq_bn_q(y2, c2.s_y, c2.z_y, c2.alpha, c2.beta, True, c3.s_x, c3.z_x), c3.z_x, c3)
            if ds is not None:
                yd = ops.conv(xq, ds.z_x, ds)
                ident = (yd, ds.s_y, ds.z_y, ds.alpha, ds.beta)
            else:
                ident = xf
            nxt = self.blocks[i + 1]["c1"] if i + 1 < len(self.blocks) else None
            xf, xq = ops.qdq_join(y3, c3.s_y, c3.z_y, c3.alpha, c3.beta, ident,
                                  nxt.s_x if nxt else None, nxt.z_x if nxt else 0)
            if keep:
                inter.update({f"block{i}.c1": y1, f"block{i}.c2": y2, f"block{i}.c3": y3, f"block{i}": xf})
                if ds is not None:
                    inter[f"block{i}.ds"] = yd
        p = ops.avgpool_f32(xf)
        f = self.fc
        q = ops.quantize(p.view(p.shape[0], p.shape[1], 1, 1), f.s_x, f.z_x, nhwc=False).view(p.shape)
        qy, logits = ops.linear_u8(q, f.z_x, f.w, f.u, f.v, f.mult, f.corr, f.z_y, False,
                                   y_scale=f.s_y, want_fp32=True)
        if keep:
            inter["pool"], inter["fc.q"] = p, qy
            return logits, inter
        return logits

    @torch.no_grad()
    def forward(self, x):
        host = not x.is_cuda
        xd = x.to(self.device, torch.float32).contiguous()
        out = self.run(xd).clone()
        if host or self.host_io:
            return out.cpu()
        torch.cuda.current_stream(self.device).synchronize()
        return out

    __call__ = forward

    def eval(self):
        return self

    def train(self, mode=True):
        if mode:
            raise RuntimeError("QuantizedResNetQDQ is inference-only")
        return self

    def to(self, device):
        self.host_io = torch.device(device).type == "cpu"   # compute stays on the GPU
        return self

    def cpu(self):
        self.host_io = True
        return self

    def cuda(self, device=None):
        self.host_io = False
        return self
