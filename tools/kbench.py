"""Forward-only kernel timing loop for profiling passes (no training, no CPU
baselines): random-init SimpleConvNet (BN recalibrated), calibrated on 64
synthetic images, then ITERS forwards at batch B on cuda:0.

    python tools/kbench.py [B] [ITERS] [MODE]     (MODE: static | qdq)

Under rocprofv3 every dispatch is one of the product kernels, so PMC passes
(e.g. GRBM_GUI_ACTIVE for the effective clock) are not diluted by the
bench's training kernels.
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    mode = sys.argv[3] if len(sys.argv) > 3 else "static"
    dev = torch.device("cuda:0")
    fp = torch_ref.reference_fp32_model(0, torch_ref.synthetic_images(64, 1))
    folded = fold_state_dict(fp.state_dict())
    ranges = calibrate(folded, [torch.from_numpy(torch_ref.synthetic_images(64, 1))], "cpu")
    model = QuantizedConvNet(build_qspec(folded, ranges, mode), dev)
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    for _ in range(5):
        model.run(x)
    torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        for _ in range(iters):
            model.run(x)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"batch {B} x {iters}: {dt / iters * 1e3:.3f} ms/forward, "
              f"{B * iters / dt / 1e6:.3f} M img/s", flush=True)


if __name__ == "__main__":
    main()
