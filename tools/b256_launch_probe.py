"""Per-launch HIP-event times at batch B (default 256) of the one launch
(convnet_convs_sm_kernel: one image per workgroup) and of the three-launch
forward (conv12, conv3+4, conv5+6 with its own tiling), per-layer QDQ and
static nets, 500 forwards each with marks and no host sync between them
(diagnostic: is conv5+6 cheaper as its own launch at this batch?).

    python tools/b256_launch_probe.py [B]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import netfix  # noqa: E402
from oracle import torch_ref  # noqa: E402  (input images only; not the measured path)
from qconvnet.qmodel import QuantizedConvNet  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda:0")
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    for mode in ("qdq", "static"):
        spec = netfix.qdq_spec(netfix.load()) if mode == "qdq" else netfix.static_spec(netfix.load(False))[0]
        model = QuantizedConvNet(spec, dev)
        for fuse in (True, False):
            model.fuse_convs = fuse
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 1.5:
                for _ in range(50):
                    model.run(x)
                torch.cuda.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2000):
                model.run(x)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / 2000 * 1e6
            names = model.kernel_names(x.shape)
            marks = []
            for _ in range(500):
                m = []
                model.run(x, marks=m)
                marks.append(m)
            torch.cuda.synchronize()
            per = {n: np.mean([m[i].elapsed_time(m[i + 1]) * 1e3 for m in marks]) for i, n in enumerate(names)}
            print(f"{mode:6s} {'one launch' if fuse else 'separate  '} batch {B}: {us:6.1f} us/forward; "
                  + ", ".join(f"{n} {v:.2f}" for n, v in per.items()), flush=True)


if __name__ == "__main__":
    main()
