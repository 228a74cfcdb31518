"""Forward time and per-launch time of the static net at batch B with the
library QCN_LIB points at (diagnostic; run once per library variant, e.g. the
grid-barrier probes of tools/gpu_grid_probe.sh): ROUNDS x ITERS back-to-back
forwards, then 500 forwards with HIP-event marks and no host sync between them
(so no host latency enters the per-launch means).  With --save / --check PATH
the logits of the last forward are written / compared bit for bit.

    QCN_LIB=... python tools/grid_probe_ab.py NAME [B] [ITERS] [ROUNDS] [--qdq] [--save P | --check P]

--qdq: the per-layer QDQ net (configs[1]) instead of the static one.
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
    args = [a for a in sys.argv[1:] if a != "--qdq"]
    qdq = "--qdq" in sys.argv[1:]
    save = check = None
    if "--save" in args:
        save = args[args.index("--save") + 1]
        args = args[:args.index("--save")]
    if "--check" in args:
        check = args[args.index("--check") + 1]
        args = args[:args.index("--check")]
    name = args[0]
    B = int(args[1]) if len(args) > 1 else 1024
    iters = int(args[2]) if len(args) > 2 else 1000
    rounds = int(args[3]) if len(args) > 3 else 3
    dev = torch.device("cuda:0")
    spec = netfix.qdq_spec(netfix.load()) if qdq else netfix.static_spec(netfix.load(False))[0]
    model = QuantizedConvNet(spec, dev)
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.5:
        for _ in range(50):
            model.run(x)
        torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            model.run(x)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / iters * 1e6)
    names = model.kernel_names(x.shape)
    marks = []
    for _ in range(500):
        m = []
        model.run(x, marks=m)
        marks.append(m)
    torch.cuda.synchronize()
    per = {n: np.mean([m[i].elapsed_time(m[i + 1]) * 1e3 for m in marks]) for i, n in enumerate(names)}
    out = model.run(x).clone()
    torch.cuda.synchronize()
    ok = ""
    if save:
        np.save(save, out.cpu().numpy())
    if check:
        ok = " logits " + ("equal" if np.array_equal(np.load(check), out.cpu().numpy()) else "DIFFER")
    print(f"{name:6s} batch {B}: " + " ".join(f"{t:6.1f}" for t in res)
          + f" us/forward (best {B / min(res):.3f} M img/s); per launch "
          + ", ".join(f"{n} {v:.2f}" for n, v in per.items()) + ok, flush=True)


if __name__ == "__main__":
    main()
