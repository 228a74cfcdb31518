"""Rebuild the golden whole-net quantized model from version-stable inputs:
numpy-PCG64 weights (oracle/torch_ref.make_state_dict), the BN statistics and
activation qparams stored in tests/golden/net_static_int8*.npz.  The int8
weights are re-derived by the PRODUCT host code (qconvnet.quant) and checked
against the torch.ao weight hashes in the fixture."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import torch

from oracle import qref, torch_ref
from qconvnet import quant as Q
from qconvnet import qmodel

F32 = np.float32
HERE = os.path.dirname(os.path.abspath(__file__))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load(per_channel=False):
    name = "net_static_int8_pc.npz" if per_channel else "net_static_int8.npz"
    return dict(np.load(os.path.join(HERE, "golden", name)))


def state_dict(z):
    sd = torch_ref.make_state_dict(0)
    for i in range(1, 8):
        sd[f"bn{i}.running_mean"] = torch.from_numpy(z[f"bn{i}_mean"])
        sd[f"bn{i}.running_var"] = torch.from_numpy(z[f"bn{i}_var"])
    return sd


def static_spec(z):
    """Product qspec (static mode) from the fixture's qparams."""
    per_channel = bool(int(z["per_channel"]))
    folded = qmodel.fold_state_dict(state_dict(z))
    spec = {"mode": "static", "per_channel": per_channel,
            "in": (F32(z["qm_in_scale"]), int(z["qm_in_zp"]))}
    s_x, z_x = spec["in"]
    for name in [f"conv{i}" for i in range(1, 7)] + ["fc1", "fc2"]:
        w = folded[f"{name}.w"]
        s_w = np.asarray(z[f"qm_{name}_s_w"], F32)
        if s_w.size == 1:
            s_w = F32(s_w.reshape(-1)[0])
        wq = Q.quantize_weight(w, s_w)
        spec[name] = dict(w=wq, b=folded[f"{name}.b"], s_w=s_w, s_x=s_x, z_x=z_x,
                          s_y=F32(z[f"qm_{name}_scale"]), z_y=int(z[f"qm_{name}_zp"]),
                          relu=name != "fc2")
        s_x, z_x = spec[name]["s_y"], spec[name]["z_y"]
    return spec, folded


def check_weights(spec, z):
    """int8 weights re-derived by the product == torch.ao's (by hash)."""
    bad = []
    for name in [f"conv{i}" for i in range(1, 7)] + ["fc1", "fc2"]:
        w = spec[name]["w"]
        if name.startswith("conv"):
            w = np.ascontiguousarray(w.transpose(0, 2, 3, 1))
        if name == "fc1":
            w = np.ascontiguousarray(w[:, qref.flatten_perm_nhwc_to_nchw()])
        if sha(w) != str(z[f"{name}_w_sha"]):
            bad.append(name)
        if not np.array_equal(spec[name]["b"], z[f"qm_{name}_b"]):
            bad.append(name + ".b")
    return bad


def oracle_dict(spec):
    """qref.static_int8_forward's dict from a product spec."""
    qm = {"in_scale": spec["in"][0], "in_zp": spec["in"][1]}
    for name in [f"conv{i}" for i in range(1, 7)] + ["fc1", "fc2"]:
        e = spec[name]
        w = e["w"]
        if name.startswith("conv"):
            w = np.ascontiguousarray(w.transpose(0, 2, 3, 1))
        if name == "fc1":
            w = np.ascontiguousarray(w[:, qref.flatten_perm_nhwc_to_nchw()])
        u, v, mult = qref.requant_constants(e["s_x"], e["s_w"], e["s_y"], e["b"])
        qm.update({name + "_w": w, name + "_u": u, name + "_v": v, name + "_mult": mult,
                   name + "_zp": e["z_y"], name + "_scale": e["s_y"]})
    return qm


def qdq_spec(z):
    """Product qspec (per-layer QDQ mode) from the fixture's QDQ qparams."""
    per_channel = bool(int(z["per_channel"]))
    folded = qmodel.fold_state_dict(state_dict(z))
    spec = {"mode": "qdq", "per_channel": per_channel}
    for i in range(1, 7):
        w = folded[f"conv{i}.w"]
        flat = w.reshape(w.shape[0], -1)
        s_w = Q.qparams_symmetric(flat.min(1), flat.max(1)) if per_channel else \
            Q.qparams_symmetric(w.min(), w.max())
        spec[f"conv{i}"] = dict(w=Q.quantize_weight(w, s_w), b=folded[f"conv{i}.b"], s_w=s_w,
                                s_x=F32(z[f"qdq_conv{i}_in_scale"]), z_x=int(z[f"qdq_conv{i}_in_zp"]),
                                s_y=F32(z[f"qdq_conv{i}_out_scale"]),
                                z_y=int(z[f"qdq_conv{i}_out_zp"]), relu=False)
    w = folded["fc1.w"]
    s_w = Q.qparams_symmetric(w.reshape(w.shape[0], -1).min(1), w.reshape(w.shape[0], -1).max(1)) \
        if per_channel else Q.qparams_symmetric(w.min(), w.max())
    spec["fc1"] = dict(w=Q.quantize_weight(w, s_w), b=folded["fc1.b"], s_w=s_w,
                       s_x=F32(z["qdq_fc1_in_scale"]), z_x=int(z["qdq_fc1_in_zp"]),
                       s_y=F32(z["qdq_fc1_out_scale"]), z_y=int(z["qdq_fc1_out_zp"]), relu=False)
    spec["fc2"] = dict(w=folded["fc2.w"], b=folded["fc2.b"])
    for i in range(1, 6):
        spec[f"conv{i}"]["next"] = (spec[f"conv{i + 1}"]["s_x"], spec[f"conv{i + 1}"]["z_x"])
    spec["conv6"]["next"] = (spec["fc1"]["s_x"], spec["fc1"]["z_x"])
    return spec


def images(z):
    x = torch_ref.synthetic_images(int(z["batch"]), 0)
    assert sha(x) == str(z["x_sha"]), "synthetic input generator drifted"
    return x
