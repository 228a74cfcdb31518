"""Same-process A/B of conv1's requant in one fma (QuantizedConvNet sets
L[0].one_mult / one_add when qcn_requant_one_fma proves the form) against the
two-op fast requant, static net at batch B: interleaved rounds of ITERS
back-to-back forwards, logits compared bit for bit (diagnostic).

    python tools/one_fma_ab.py [B] [ITERS] [ROUNDS] [--per-channel]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import netfix  # noqa: E402
from oracle import torch_ref  # noqa: E402  (input images only; not the measured path)
from qconvnet.qmodel import QuantizedConvNet  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    pc = "--per-channel" in sys.argv
    B = int(args[0]) if args else 1024
    iters = int(args[1]) if len(args) > 1 else 1000
    rounds = int(args[2]) if len(args) > 2 else 4
    dev = torch.device("cuda:0")
    spec, _ = netfix.static_spec(netfix.load(pc))
    one, two = QuantizedConvNet(spec, dev), QuantizedConvNet(spec, dev)
    print("conv1 one-fma form:", one.L[0].one_mult is not None, flush=True)
    two.L[0].one_mult = two.L[0].one_add = None
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    forms = {"one-fma": one, "two-op": two}
    for m in forms.values():
        for _ in range(300):
            m.run(x)
    torch.cuda.synchronize()
    assert torch.equal(one.run(x).clone(), two.run(x).clone()), "logits differ"
    res = {k: [] for k in forms}
    for _ in range(rounds):
        for k, m in forms.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                m.run(x)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / iters * 1e6)
    for k, v in res.items():
        print(f"{k:8s} batch {B}: " + " ".join(f"{t:6.1f}" for t in v) + f" us/forward; best {B / min(v):.3f} M img/s",
              flush=True)
    print("logits equal", flush=True)


if __name__ == "__main__":
    main()
