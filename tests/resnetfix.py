"""Rebuild the §8(f)2 whole-net golden ResNet (tests/golden/net_resnet_int8.npz,
written by oracle/make_golden.py gen_resnet_net) from version-stable inputs:
numpy-PCG64 weights (oracle/torch_ref.resnet_state_dict) plus the BN running
statistics and qparams stored in the fixture.  BN folding and int8 weight
quantization are done by the PRODUCT host code (qconvnet.resnet / quant) and
checked against torch.ao's int8 weights by hash."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import torch

from oracle import torch_ref

F32 = np.float32
HERE = os.path.dirname(os.path.abspath(__file__))
IMAGENET = dict(mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load(name="net_resnet_int8.npz"):
    return dict(np.load(os.path.join(HERE, "golden", name)))


def load_qdq():
    """The reference-semantics (live per-layer stubs) fixture,
    oracle/make_golden.py gen_resnet_qdq_net."""
    return load("net_resnet_qdq.npz")


def qdq_spec(z, fixture_qparams=False):
    """Product spec (qconvnet.resnet_qdq.build_spec) from the fixture's
    regenerated fp32 model, calibrated by the PRODUCT host code on the
    fixture's calibration images.  fixture_qparams=True then overwrites every
    stub's and conv's qparams with the fixture's: the calibration's fp32 CPU
    convs differ in the last bits between host CPUs (the GPU box's is not this
    container's), so GPU tests take torch.ao's qparams as given, as
    spec() does for the static net; the CPU test pins the calibration here."""
    from qconvnet import resnet_qdq
    net = resnet_qdq.unfolded_state(fp32_model(z).state_dict())
    ranges = resnet_qdq.calibrate(net, [torch.from_numpy(images(z, "calib"))], "cpu")
    sp = resnet_qdq.build_spec(net, ranges, True)
    if fixture_qparams:
        def put(name, e):
            e["s_x"], e["z_x"] = F32(z[name + ".s_x"]), int(z[name + ".z_x"])
            e["s_y"], e["z_y"] = F32(z[name + ".s_y"]), int(z[name + ".z_y"])
        put("stem", sp["stem"])
        for i, e in enumerate(sp["blocks"]):
            for k in ("c1", "c2", "c3", "ds"):
                if e[k] is not None:
                    put(f"b{i}.{k}", e[k])
        put("fc", sp["fc"])
    return sp


def check_qdq_spec(sp, z):
    """Names whose qparams or int8 weights differ from torch.ao's."""
    bad = []

    def cmp(name, e):
        for k in ("s_x", "z_x", "s_y", "z_y"):
            if np.asarray(e[k]) != np.asarray(z[f"{name}.{k}"]):
                bad.append(f"{name}.{k}")
        if sha(e["w"]) != str(z[f"{name}.w_sha"]):
            bad.append(f"{name}.w")
    cmp("stem", sp["stem"])
    for i, e in enumerate(sp["blocks"]):
        for k in ("c1", "c2", "c3", "ds"):
            if e[k] is not None:
                cmp(f"b{i}.{k}", e[k])
    cmp("fc", sp["fc"])
    return bad


def fp32_model(z):
    m = torch_ref.ResNetRef(tuple(int(v) for v in z["layers"]), int(z["num_classes"]))
    sd = torch_ref.resnet_state_dict(m, 0)
    for k in sd:
        if "sd." + k in z:
            sd[k] = torch.from_numpy(z["sd." + k])
    m.load_state_dict(sd)
    return m.eval()


def images(z, which="x"):
    hw = int(z["hw"])
    if which == "x":
        x = torch_ref.synthetic_images(int(z["batch"]), 5, hw=hw, **IMAGENET)
    else:
        x = torch_ref.synthetic_images(8, 4, hw=hw, **IMAGENET)
    assert sha(x) == str(z[f"{which}_sha"]), "synthetic input generator drifted"
    return x


def spec(z):
    """Product spec (qconvnet.resnet.build_spec's format) with the fixture's
    qparams and the product's own folded / quantized weights."""
    from qconvnet import quant as Q
    from qconvnet.qmodel import _weight_scale
    from qconvnet.resnet import fold_state_dict
    folded = fold_state_dict(fp32_model(z).state_dict())

    def layer(wb, name, s_x, z_x, relu):
        w, b, st, pad = wb
        s_w = _weight_scale(w, True)
        return dict(w=Q.quantize_weight(w, s_w), b=np.asarray(b, F32), s_w=s_w, s_x=F32(s_x),
                    z_x=int(z_x), s_y=F32(z[name + ".s_y"]), z_y=int(z[name + ".z_y"]), relu=relu,
                    stride=(st, st), pad=(pad, pad))

    sp = {"per_channel": True, "blocks": [], "in": (F32(z["in_scale"]), int(z["in_zp"]))}
    w, b = folded["stem"]
    sp["stem"] = layer((w, b, 2, 3), "stem", *sp["in"], True)
    s_x, z_x = sp["stem"]["s_y"], sp["stem"]["z_y"]
    for i, blk in enumerate(folded["blocks"]):
        e = {"c1": layer(blk["c1"], f"b{i}.c1", s_x, z_x, True)}
        e["c2"] = layer(blk["c2"], f"b{i}.c2", e["c1"]["s_y"], e["c1"]["z_y"], True)
        e["c3"] = layer(blk["c3"], f"b{i}.c3", e["c2"]["s_y"], e["c2"]["z_y"], False)
        e["ds"] = layer(blk["ds"], f"b{i}.ds", s_x, z_x, False) if "ds" in blk else None
        e["out"] = (F32(z[f"b{i}.out_scale"]), int(z[f"b{i}.out_zp"]))
        sp["blocks"].append(e)
        s_x, z_x = e["out"]
    w, b = folded["fc"]
    s_w = _weight_scale(w, True)
    sp["fc"] = dict(w=Q.quantize_weight(w, s_w), b=np.asarray(b, F32), s_w=s_w, s_x=s_x, z_x=z_x,
                    s_y=F32(z["fc.s_y"]), z_y=int(z["fc.z_y"]), relu=False)
    return sp


def check_weights(sp, z):
    """Layer names whose product-quantized int8 weights differ from torch.ao's."""
    bad = [] if sha(sp["stem"]["w"]) == str(z["stem.w_sha"]) else ["stem"]
    for i, e in enumerate(sp["blocks"]):
        for k in ("c1", "c2", "c3", "ds"):
            if e[k] is not None and sha(e[k]["w"]) != str(z[f"b{i}.{k}.w_sha"]):
                bad.append(f"b{i}.{k}")
    if sha(sp["fc"]["w"]) != str(z["fc.w_sha"]):
        bad.append("fc")
    return bad
