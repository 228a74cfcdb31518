"""Time one ResNet 1x1 conv launch (default: layer-1 expand 64->256 at 56x56,
batch 512, with the fused residual join) through the C ABI, 50 launches;
prints ms and the algorithmic HBM rate.  Env: SHAPE=n,hw,cin,cout  RESID=0/1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "convnet-quantization_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from qconvnet import _lib, ops  # noqa: E402
from qconvnet import quant as Q  # noqa: E402
from qconvnet.qmodel import _DevLayer  # noqa: E402

n, hw, cin, cout = (int(t) for t in os.environ.get("SHAPE", "512,56,64,256").split(","))
resid = os.environ.get("RESID", "1") == "1"
_lib.load()
dev = torch.device("cuda")
rng = np.random.default_rng(0)
wq = rng.integers(-127, 128, (cout, cin, 1, 1)).astype(np.int8)
packed, wsum = ops.pack_conv_kmajor(wq)
d = _DevLayer()
d.cout, d.kh, d.kw, d.sy, d.sx, d.py, d.px = cout, 1, 1, 1, 1, 0, 0
u, v, mult = Q.epilogue_constants(np.float32(0.02), np.full(cout, 0.001, np.float32), np.float32(0.1),
                                  rng.standard_normal(cout).astype(np.float32))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
d.w, d.u, d.v, d.mult = T(packed), T(u), T(v), T(mult)
d.corr = T(((128 - 3) * wsum.astype(np.int64)).astype(np.int32))
d.z_y, d.relu, d.s_y = 7, not resid, np.float32(0.1)
x = torch.randint(0, 256, (n, hw, hw, cin), dtype=torch.uint8, device=dev)
r = torch.randint(0, 256, (n, hw, hw, cout), dtype=torch.uint8, device=dev)
out = torch.empty((n, hw, hw, cout), dtype=torch.uint8, device=dev)
rs = (r, np.float32(0.03), 5, np.float32(0.05), 0) if resid else None
for _ in range(5):
    ops.conv(x, 3, d, out=out, resid=rs)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    ops.conv(x, 3, d, out=out, resid=rs)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 50
byts = n * hw * hw * (cin + cout * (2 if resid else 1))
print(f"{os.environ.get('QCN_GEMM_STREAM', '1')=} {n=} {hw=} {cin=} {cout=} {resid=}: "
      f"{ms:.3f} ms  {byts / ms / 1e9:.2f} TB/s")
