"""Same-process A/B of the static forward at batch B: conv1 .. conv6 in one
persistent launch (QuantizedConvNet.fuse_convs) against conv12 -> conv3+4 ->
conv5+6, interleaved rounds of ITERS forwards each (diagnostic).

    python tools/c16_ab.py [B] [ITERS] [ROUNDS]
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
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda:0")
    fp = torch_ref.reference_fp32_model(0, torch_ref.synthetic_images(64, 1))
    folded = fold_state_dict(fp.state_dict())
    ranges = calibrate(folded, [torch.from_numpy(torch_ref.synthetic_images(64, 1))], "cpu")
    model = QuantizedConvNet(build_qspec(folded, ranges, "static"), dev)
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    res = {True: [], False: []}
    for flag in (True, False):
        model.fuse_convs = flag
        for _ in range(300):
            model.run(x)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for flag in (True, False):
            model.fuse_convs = flag
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                model.run(x)
            torch.cuda.synchronize()
            res[flag].append((time.perf_counter() - t0) / iters * 1e6)
    for flag, v in res.items():
        print(f"{'one launch ' if flag else 'three      '} batch {B}: "
              + " ".join(f"{t:6.1f}" for t in v) + f" us/forward; best {B / min(v):.3f} M img/s",
              flush=True)
    model.fuse_convs = True
    print("names", model.kernel_names(x.shape))


if __name__ == "__main__":
    main()
