"""Same-process A/B of the static forward at batch B (diagnostic): conv1 ..
conv6 in one launch (convnet_convs16_kernel, 512-thread workgroups) against
conv12 + conv3 .. conv6 in one launch of one-wave-per-SIMD workgroups
(convs36_w4_kernel), interleaved rounds of ITERS forwards each, plus the
per-launch HIP-event times of each form.

    python tools/w4_ab.py [B] [ITERS] [ROUNDS]
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda:0")
    spec, _ = netfix.static_spec(netfix.load(False))
    model = QuantizedConvNet(spec, dev)
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    forms = {"one-launch": False, "w4": True}
    res = {k: [] for k in forms}
    for name, flag in forms.items():
        model.convs_w4 = flag
        for _ in range(300):
            model.run(x)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for name, flag in forms.items():
            model.convs_w4 = flag
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                model.run(x)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / iters * 1e6)
    for name, v in res.items():
        print(f"{name:11s} batch {B}: " + " ".join(f"{t:6.1f}" for t in v)
              + f" us/forward; best {B / min(v):.3f} M img/s", flush=True)
    for name, flag in forms.items():
        model.convs_w4 = flag
        names = model.kernel_names(x.shape)
        per = {n: [] for n in names}
        for _ in range(200):
            m = []
            model.run(x, marks=m)
            torch.cuda.synchronize()
            for i, n in enumerate(names):
                per[n].append(m[i].elapsed_time(m[i + 1]) * 1e3)
        print(f"{name:11s} per launch (HIP events, mean us): "
              + ", ".join(f"{n} {np.mean(v):.1f}" for n, v in per.items()), flush=True)


if __name__ == "__main__":
    main()
