"""Experiment: do two full 1024-image forwards on two HIP streams overlap at
the kernel edges (ramp / drain / launch boundaries)?  Compares images/s of
(a) one stream, batches back to back and (b) two streams, one batch each in
flight, same model weights, same kernels.

    python tools/twostream.py [ITERS]
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


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    fp = torch_ref.reference_fp32_model(0, torch_ref.synthetic_images(64, 1))
    folded = fold_state_dict(fp.state_dict())
    ranges = calibrate(folded, [torch.from_numpy(torch_ref.synthetic_images(64, 1))], "cpu")
    spec = build_qspec(folded, ranges, "static")
    ma, mb = QuantizedConvNet(spec, dev), QuantizedConvNet(spec, dev)
    xa = torch.from_numpy(torch_ref.synthetic_images(1024, 0)).to(dev)
    xb = torch.from_numpy(torch_ref.synthetic_images(1024, 1)).to(dev)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for _ in range(10):
        ma.run(xa)
        mb.run(xb)
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(iters):
            ma.run(xa)
        torch.cuda.synchronize()
        one = 1024 * iters / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        for _ in range(iters // 2):
            with torch.cuda.stream(sa):
                ma.run(xa)
            with torch.cuda.stream(sb):
                mb.run(xb)
        torch.cuda.synchronize()
        two = 1024 * (iters // 2) * 2 / (time.perf_counter() - t0)
        print(f"one stream {one / 1e6:.3f} M img/s   two streams {two / 1e6:.3f} M img/s", flush=True)


if __name__ == "__main__":
    main()
