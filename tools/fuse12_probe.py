"""Same-box A/B of the fused conv12 launch (fuse12=True) against conv1 and
conv2 as two launches (a1 through HBM), per batch size and mode: at one image
per CU (config 2, batch 256) the fused kernel runs three pipeline stages for
two half-image tiles.

    python tools/fuse12_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

from oracle import torch_ref  # noqa: E402  (weights only; not the measured path)
from qconvnet.qmodel import QuantizedConvNet, build_qspec, calibrate, fold_state_dict  # noqa: E402


def timed(model, x, iters=400):
    t_end = time.perf_counter() + 0.3   # load the chip first
    while time.perf_counter() < t_end:
        model.run(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        model.run(x)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    fp = torch_ref.reference_fp32_model(0, torch_ref.synthetic_images(64, 1))
    folded = fold_state_dict(fp.state_dict())
    ranges = calibrate(folded, [torch.from_numpy(torch_ref.synthetic_images(64, 1))], "cpu")
    for mode in ("qdq", "static"):
        spec = build_qspec(folded, ranges, mode)
        models = {f: QuantizedConvNet(spec, dev, fuse12=f) for f in (True, False)}
        for B in (256, 512, 1024):
            x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
            ref = models[True].run(x).clone()
            same = torch.equal(ref, models[False].run(x))
            for rep in range(2):
                ms = {f: timed(m, x) for f, m in models.items()}
                print(f"{mode:6s} batch {B:5d}: fused {ms[True]*1e3:7.1f} us  split {ms[False]*1e3:7.1f} us"
                      f"  ({B / ms[True] / 1e3:.2f} vs {B / ms[False] / 1e3:.2f} M img/s)  logits equal {same}",
                      flush=True)


if __name__ == "__main__":
    main()
