"""Debug: the classifier head (static and QDQ) at m rows against the
per-layer linear kernels; prints mismatch positions."""
import os
import sys
from types import SimpleNamespace as NS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "convnet-quantization_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from qconvnet import _lib, ops  # noqa: E402
from qconvnet import quant as Q  # noqa: E402

F32 = np.float32
_lib.load()
dev = torch.device("cuda")
rng = np.random.default_rng(5)
k, n1, n2 = 4096, 512, 10
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
for m in (256, 1024):
    qx = rng.integers(0, 256, (m, k), dtype=np.uint8)
    w1 = rng.integers(-128, 128, (n1, k), dtype=np.int8)
    w2 = rng.integers(-128, 128, (n2, n1), dtype=np.int8)
    s_x, s_y1, s_y2, s_w1, s_w2 = F32(0.02), F32(0.05), F32(0.11), F32(2e-4), F32(2e-3)
    b1 = rng.normal(0, 0.5, n1).astype(F32)
    b2 = rng.normal(0, 0.5, n2).astype(F32)
    zx, z1, z2 = 3, 0, 120
    u1, v1, m1 = Q.epilogue_constants(s_x, s_w1, s_y1, b1)
    u2, v2, m2 = Q.epilogue_constants(s_y1, s_w2, s_y2, b2)
    corr1 = ((128 - zx) * w1.astype(np.int64).sum(1)).astype(np.int32)
    corr2 = ((128 - z1) * w2.astype(np.int64).sum(1)).astype(np.int32)
    y1_ref = ops.linear_u8(T(qx), zx, T(w1), T(u1), T(v1), T(m1), T(corr1), z1, True)
    y2_ref, y2f_ref = ops.linear_u8(y1_ref, z1, T(w2), T(u2), T(v2), T(m2), T(corr2), z2, False,
                                    y_scale=s_y2, want_fp32=True)
    l1 = NS(w=T(w1), wk=T(ops.pack_fc_kmajor(w1)), u=T(u1), v=T(v1), mult=T(m1), corr=T(corr1),
            z_y=z1, relu=True)
    l2 = NS(w=T(w2), u=T(u2), v=T(v2), mult=T(m2), z_y=z2, relu=False, s_y=s_y2)
    ws = ops.classifier_workspace(m, n1, dev)
    y1 = torch.empty((m, n1), dtype=torch.uint8, device=dev)
    y2 = torch.zeros((m, n2), dtype=torch.uint8, device=dev)
    y2f = torch.zeros((m, n2), dtype=torch.float32, device=dev)
    ok = ops.classifier(ops.to_kmajor(T(qx)), l1, l2, ws, y1, y2, y2f)
    torch.cuda.synchronize()
    d1 = (y1 != y1_ref).nonzero()
    d2 = (y2 != y2_ref).nonzero()
    print(f"static m={m} ok={ok} y1 mismatches {len(d1)} y2 mismatches {len(d2)}", d2[:10].tolist())
    # QDQ: fc1 -> dequantize -> relu -> fp32 fc2
    w2f = (rng.standard_normal((n2, n1)) * 0.05).astype(F32)
    b2f = rng.standard_normal(n2).astype(F32)
    l2q = NS(w=T(w2f), b=T(b2f))
    y1q = torch.empty((m, n1), dtype=torch.uint8, device=dev)
    yq = torch.zeros((m, n2), dtype=torch.float32, device=dev)
    l1q = NS(w=T(w1), wk=T(ops.pack_fc_kmajor(w1)), u=T(u1), v=T(v1), mult=T(m1), corr=T(corr1),
             z_y=z1, relu=False, s_y=s_y1)
    y1r = ops.linear_u8(T(qx), zx, T(w1), T(u1), T(v1), T(m1), T(corr1), z1, False)
    xf = torch.relu((y1r.float() - z1) * float(s_y1))
    ref = xf @ T(w2f).t() + T(b2f)
    try:
        okq = ops.classifier_qdq(ops.to_kmajor(T(qx)), l1q, l2q, ws, y1q, yq)
    except Exception as e:  # noqa: BLE001
        print("qdq call failed:", e)
        continue
    torch.cuda.synchronize()
    err = (yq - ref).abs()
    print(f"qdq m={m} ok={okq} y1 mismatches {(y1q != y1r).sum().item()} max err {err.max().item():.3g} "
          f"rows bad {(err.max(1).values > 1e-3).nonzero().flatten()[:20].tolist()} "
          f"cols bad {(err.max(0).values > 1e-3).nonzero().flatten().tolist()}")
