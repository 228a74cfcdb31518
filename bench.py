"""Benchmark: images/sec of the full static-PTQ int8 SimpleConvNet at batch 1024
(3x32x32) per MI355X — BASELINE.json's metric on configs[2] (N=1) and
configs[3] (batch 8192 = 8 x 1024 sharded, RCCL all-gather of logits, N=8).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

A step = one forward of the whole int8 net over this rank's 1024 resident
images (fp32 NCHW in HBM -> quantize+conv1 ... fc2 -> fp32 logits) plus, for
N > 1, the all-gather of every rank's logits.  Weak scaling: 1024 images per
GPU.  Weights: random-init SimpleConvNet with BN statistics recalibrated on
synthetic CIFAR-normalised images (no trained checkpoint or dataset offline),
calibrated once on rank 0 and broadcast.

Prints ONE JSON line on rank 0 with value (whole-job images/sec), a
``roofline`` object for the dominant kernel (HIP-event per-kernel timing over
a second timed pass) and, at N = 1, ``cpu_baseline`` (the reference's
StaticPTQModel path — torch.ao quantize_dynamic — timed on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec at batch 1024 (3×32×32) int8 static-PTQ, 1/2/4/8 MI355X; top-1 delta"
PEAK_INT8_TOPS = 5033.0   # 256 CU x 4 SIMD x 2048 int8 op/clk x 2.4 GHz (dense)
PEAK_HBM_GBS = 8000.0
# MAC per image per kernel
MAC_PER_IMAGE = {"conv1": 1_769_472, "conv2": 37_748_736, "conv3": 18_874_368,
                 "conv4": 37_748_736, "conv5": 18_874_368, "conv6": 37_748_736,
                 "fc1": 2_097_152, "fc2": 5_120}
MAC_PER_IMAGE["conv12"] = MAC_PER_IMAGE["conv1"] + MAC_PER_IMAGE["conv2"]
MAC_PER_IMAGE["fc12"] = MAC_PER_IMAGE["fc1"] + MAC_PER_IMAGE["fc2"]
MAC_PER_IMAGE["conv34"] = MAC_PER_IMAGE["conv3"] + MAC_PER_IMAGE["conv4"]
MAC_PER_IMAGE["conv56"] = MAC_PER_IMAGE["conv5"] + MAC_PER_IMAGE["conv6"]
MAC_PER_IMAGE["net"] = sum(MAC_PER_IMAGE[f"conv{i}"] for i in range(1, 7))
# algorithmic HBM bytes per image (u8 activations, fp32 input/logits)
BYTES_PER_IMAGE = {"conv1": 3 * 32 * 32 * 4 + 32 * 32 * 64,
                   "conv2": 32 * 32 * 64 + 16 * 16 * 64,
                   "conv3": 16 * 16 * 64 + 16 * 16 * 128,
                   "conv4": 16 * 16 * 128 + 8 * 8 * 128,
                   "conv5": 8 * 8 * 128 + 8 * 8 * 256,
                   "conv6": 8 * 8 * 256 + 4 * 4 * 256,
                   "fc1": 4096 + 512, "fc2": 512 + 10 + 40,
                 "conv12": 3 * 32 * 32 * 4 + 16 * 16 * 64,
                 "fc12": 4096 + 512 + 10 + 40,
                 "conv34": 16 * 16 * 64 + 8 * 8 * 128,
                 "conv56": 8 * 8 * 128 + 4 * 4 * 256,
                 "net": 3 * 32 * 32 * 4 + 4 * 4 * 256}
HBM_BOUND = {"conv1"}


def build_model(rank, device, per_channel=False):
    from models.baseline_model import trained_synthetic_model
    from qconvnet import data
    from qconvnet.dist import broadcast_object
    from qconvnet.qmodel import QuantizedConvNet, build_qspec, calibrate, fold_state_dict
    payload = None
    if rank == 0:
        # trained on the synthetic 10-class task (no CIFAR-10 / checkpoint offline)
        x_cal, _ = data.synthetic_task(512, 1)
        calib = torch.from_numpy(x_cal)
        fp = trained_synthetic_model(0, device=device)
        folded = fold_state_dict(fp.state_dict())
        ranges = calibrate(folded, [calib], "cpu")
        payload = (build_qspec(folded, ranges, "static", per_channel), fp.state_dict())
    spec, sd = broadcast_object(payload)
    return QuantizedConvNet(spec, device), sd


def cpu_baselines(state_dict, qmodel_gpu, seconds):
    """Reference CPU paths on the host cores (rank 0, N = 1 only)."""
    from oracle import torch_ref
    from qconvnet import data
    fp = torch_ref.SimpleConvNetRef()
    fp.load_state_dict(state_dict)
    fp.eval()
    threads = torch.get_num_threads()
    out = {}
    # (1) StaticPTQModel as the reference builds it (static_ptq_model.py:19-34):
    #     quantize_dynamic({Linear, Conv2d}, qint8) -> fp32 convs + dynamic int8 fc
    sp = torch_ref.build_static_ptq_cpu(fp)
    bs = 32
    x = torch.from_numpy(data.synthetic_images(bs, 11))
    with torch.no_grad():
        for _ in range(3):
            sp(x)
        total, iters = 0.0, 0
        while total < seconds:
            t0 = time.time()
            sp(x)
            total += time.time() - t0
            iters += 1
    out["static_ptq"] = {"value": bs * iters / total, "unit": "images/sec", "cores": threads,
                         "kind": "port",
                         "sample": f"reference StaticPTQModel path (torch.ao quantize_dynamic "
                                   f"{{Linear,Conv2d}} qint8 on our SimpleConvNet restatement), "
                                   f"batch {bs} x {iters} iters, time.time() loop as "
                                   f"utils/inference_benchmark.py:92-100"}
    # (2) full static int8 on the CPU (torch.ao eager, fbgemm) — apples to apples
    calib = torch.from_numpy(data.synthetic_task(512, 1)[0])   # the GPU model's calibration set
    q = torch_ref.build_static_int8_cpu(fp, [calib])
    bs2 = 256
    x2 = torch.from_numpy(data.synthetic_images(bs2, 12))
    with torch.no_grad():
        q(x2)
        total, iters = 0.0, 0
        while total < seconds / 2:
            t0 = time.time()
            q(x2)
            total += time.time() - t0
            iters += 1
    out["static_int8"] = {"value": bs2 * iters / total, "unit": "images/sec", "cores": threads,
                          "kind": "port",
                          "sample": f"torch.ao eager static int8 (fbgemm), batch {bs2} x {iters} iters"}
    # (3) top-1 on a held-out synthetic test set with true labels (the fp32
    #     model was trained on the same task; CIFAR-10 is not available offline)
    xe_np, ye_np = data.synthetic_task(4096, 77)
    xe, lab = torch.from_numpy(xe_np), torch.from_numpy(ye_np)
    with torch.no_grad():
        fp_pred = fp(xe).argmax(1)
        ref_pred = sp(xe).argmax(1)
        gpu_pred = qmodel_gpu(xe).argmax(1)
        cpu_int8_pred = q(xe).argmax(1)
    # the reference's own StaticPTQModel semantics on the GPU (fp32 convs +
    # HIP dynamic int8 Linear, models/static_ptq_model.py mode="reference")
    from models.static_ptq_model import StaticPTQModel
    rm = StaticPTQModel(device=qmodel_gpu.device, mode="reference")
    rm.load_state_dict(state_dict)
    rq = rm.quantize()
    with torch.no_grad():
        gpu_ref_pred = rq(xe.to(qmodel_gpu.device)).argmax(1).cpu()

    def acc(p):
        return (p == lab).float().mean().item() * 100

    out["top1"] = {"labels": "true labels of 4096 held-out images of the synthetic 10-class task "
                             "the fp32 SimpleConvNet was trained on (qconvnet.data.synthetic_task)",
                   "fp32": acc(fp_pred), "gpu_int8_static": acc(gpu_pred),
                   "cpu_reference_static_ptq": acc(ref_pred),
                   "cpu_torchao_static_int8": acc(cpu_int8_pred),
                   "gpu_reference_mode_static_ptq": acc(gpu_ref_pred),
                   "delta_vs_reference_pct": acc(gpu_pred) - acc(ref_pred),
                   "delta_reference_mode_pct": acc(gpu_ref_pred) - acc(ref_pred),
                   "gpu_int8_equals_torchao_static_int8": bool(torch.equal(gpu_pred, cpu_int8_pred)),
                   "agreement_gpu_int8_vs_fp32_pct": (gpu_pred == fp_pred).float().mean().item() * 100}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024, help="images per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--per-channel", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay the forward as one HIP graph (measured: no gain, the launch "
                         "queue already runs back to back)")
    ap.add_argument("--workload", choices=("convnet", "resnet50"), default="convnet",
                    help="convnet: BASELINE configs[2]/[3] (the metric); resnet50: configs[4]")
    args = ap.parse_args()
    if args.workload == "resnet50":
        return main_resnet(args)

    from qconvnet import data
    from qconvnet import dist as qd

    rank, world, local = qd.init()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world != args.gpus and rank == 0:
        print(f"# note: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)

    model, sd = build_model(rank, dev, args.per_channel)
    B = args.batch
    x = torch.from_numpy(data.synthetic_images(B, 100 + rank)).to(dev)
    gathered = torch.empty((world * B, 10), dtype=torch.float32, device=dev) if world > 1 else None

    use_graph = args.graph
    if use_graph:   # the forward's launches as one HIP graph (same kernels, no launch gaps)
        model.capture_graph(x)

    def step(marks=None):
        if marks is None and use_graph:
            logits = model.replay(B)
        else:
            logits = model.run(x, marks=marks)
        if world > 1:
            qd.gather_logits(logits, gathered)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- timed region A: the metric
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    images = world * B * args.steps
    value = images / elapsed

    # ---- timed region B: per-kernel HIP events (same steps, same stream)
    marks_all = []
    barrier()
    torch.cuda.synchronize()
    for _ in range(args.steps):
        m = []
        step(m)
        marks_all.append(m)
    torch.cuda.synchronize()
    names = model.kernel_names(x.shape)
    per = {n: [] for n in names}
    for m in marks_all:
        for i, n in enumerate(names):
            per[n].append(m[i].elapsed_time(m[i + 1]))
    kern = {}
    for n in names:
        ms = float(np.mean(per[n]))
        ops_ = 2.0 * MAC_PER_IMAGE[n] * B
        byts = BYTES_PER_IMAGE[n] * B
        kern[n] = {"ms": ms, "tops": ops_ / (ms * 1e-3) / 1e12,
                   "gbs": byts / (ms * 1e-3) / 1e9,
                   "bound": "hbm" if n in HBM_BOUND else "mfma"}
        kern[n]["frac"] = (kern[n]["gbs"] / PEAK_HBM_GBS if n in HBM_BOUND
                           else kern[n]["tops"] / PEAK_INT8_TOPS)
    dom = max(names, key=lambda n: kern[n]["ms"])
    k = kern[dom]
    if k["bound"] == "mfma":
        roof = {"kernel": dom, "bound": "mfma", "achieved": k["tops"], "peak": PEAK_INT8_TOPS,
                "unit": "TFLOP/s", "frac": k["frac"], "traffic": None,
                "note": "int8 TOPS reported in the TFLOP/s slot; achieved = 2*MAC*1024 / mean HIP-event duration"}
    else:
        roof = {"kernel": dom, "bound": "hbm", "achieved": k["gbs"], "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": k["frac"], "traffic": None}

    result = {
        "metric": METRIC, "value": value, "unit": "images/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int8", "data": "synthetic",
        "config": {"workload": "full static-PTQ SimpleConvNet, all conv+linear int8 (u8 x s8 -> i32), "
                               "NHWC, per-tensor weights" + (" [per-channel]" if args.per_channel else ""),
                   "global_batch": world * B, "per_gpu_batch": B, "image": [3, 32, 32],
                   "parallelism": f"dp{world}", "collective": "all_gather logits (RCCL)" if world > 1 else None},
        "roofline": roof,
        "kernels": {n: {kk: round(vv, 4) if isinstance(vv, float) else vv for kk, vv in kern[n].items()}
                    for n in names},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        cb = cpu_baselines(sd, model, args.cpu_seconds)
        result["cpu_baseline"] = cb["static_ptq"]
        result["cpu_static_int8"] = cb["static_int8"]
        result["top1"] = cb["top1"]
        result["gpu_vs_cpu_ratio"] = value / cb["static_ptq"]["value"]
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# ============================================================ configs[4]
METRIC_RESNET = "images/sec at batch 512 (3×224×224) ResNet-50 bottleneck blocks, per-channel int8"


def resnet_cpu_baseline(model_fp, seconds):
    """torch.ao FX static int8 (fbgemm, per-channel weights) of the same
    ResNet-50 on the host cores, and the fp32 model the reference's
    CustomQuantizedResNet50 effectively runs (its stubs are never converted)."""
    from torch.ao.quantization import get_default_qconfig_mapping
    from torch.ao.quantization.quantize_fx import convert_fx, prepare_fx
    from models.resnet import synthetic_images
    fp = model_fp.cpu().eval()
    threads = torch.get_num_threads()
    xc = torch.from_numpy(synthetic_images(8, 21))
    with torch.no_grad():
        pq = prepare_fx(fp, get_default_qconfig_mapping("fbgemm"), example_inputs=(xc,))
        pq(xc)
        q = convert_fx(pq)
    bs = 32
    x = torch.from_numpy(synthetic_images(bs, 22))
    out = {}
    for name, m, budget in (("static_int8", q, seconds), ("fp32", fp, seconds / 2)):
        with torch.no_grad():
            m(x)
            total, iters = 0.0, 0
            while total < budget:
                t0 = time.time()
                m(x)
                total += time.time() - t0
                iters += 1
        out[name] = {"value": bs * iters / total, "unit": "images/sec", "cores": threads,
                     "kind": "port", "sample": f"batch {bs} x {iters} iters"}
    out["static_int8"]["sample"] = ("torch.ao FX static int8 (fbgemm, per-channel) of the same "
                                    "ResNet-50, " + out["static_int8"]["sample"])
    out["fp32"]["sample"] = ("fp32 ResNet-50 (what CustomQuantizedResNet50 runs: its stubs are "
                             "never converted), " + out["fp32"]["sample"])
    return out, q


def main_resnet(args):
    from models.resnet import synthetic_images, synthetic_resnet
    from qconvnet import dist as qd
    from qconvnet.resnet import quantize_resnet

    rank, world, local = qd.init()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B = args.batch if args.batch != 1024 else 512
    fp = synthetic_resnet(0, device=dev, calib_images=32)
    calib = [torch.from_numpy(synthetic_images(32, 1 + i)) for i in range(2)]
    model = quantize_resnet(fp, calib, dev, per_channel=True)
    x = torch.from_numpy(synthetic_images(B, 100 + rank)).to(dev)
    gathered = torch.empty((world * B, model.num_classes), dtype=torch.float32,
                           device=dev) if world > 1 else None

    use_graph = args.graph
    if use_graph:   # the forward's launches as one HIP graph (same kernels, no launch gaps)
        model.capture_graph(x)

    def step(marks=None):
        if marks is None and use_graph:
            logits = model.replay(B)
        else:
            logits = model.run(x, marks=marks)
        if world > 1:
            qd.gather_logits(logits, gathered)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    value = world * B * args.steps / elapsed

    # MACs per image of every conv launch, in forward order
    convs = model.conv_layers()
    hh = (x.shape[2] + 2 * convs[0].py - convs[0].kh) // convs[0].sy + 1   # stem output
    sizes = [hh * hh]
    hh = (hh - 1) // 2 + 1                                                   # maxpool
    for b in model.blocks:   # launch order: [ds], c1, c2, c3 (conv_layers())
        ho = (hh + 2 * b["c2"].py - b["c2"].kh) // b["c2"].sy + 1
        sizes += ([ho * ho] if b["ds"] is not None else []) + [hh * hh, ho * ho, ho * ho]
        hh = ho
    mac_img = [sz * d.cout * d.w.shape[0] * 32 for sz, d in zip(sizes, convs)]  # K = chunks*32
    per_name = {}
    n_rep = max(3, min(args.steps, 10))
    conv_ms = []
    for _ in range(n_rep):
        m = []
        step(m)
        torch.cuda.synchronize()
        tot_conv = 0.0
        for (_, e0), (n1, e1) in zip(m[:-1], m[1:]):
            ms = e0.elapsed_time(e1)
            per_name.setdefault(n1, []).append(ms)
            if n1 == "conv":
                tot_conv += ms
        conv_ms.append(tot_conv)
    conv_ms = float(np.mean(conv_ms))
    conv_ops = 2.0 * sum(mac_img) * B
    tops = conv_ops / (conv_ms * 1e-3) / 1e12
    roof = {"kernel": "conv_gemm_kernel (all 53 conv launches)", "bound": "mfma", "achieved": tops,
            "peak": PEAK_INT8_TOPS, "unit": "TFLOP/s", "frac": tops / PEAK_INT8_TOPS, "traffic": None,
            "note": "int8 TOPS in the TFLOP/s slot; achieved = 2*sum(conv MAC)*batch / summed "
                    "HIP-event conv time; stem MACs counted at the packed K=224 actually issued"}
    result = {
        "metric": METRIC_RESNET, "value": value, "unit": "images/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int8",
        "data": "synthetic",
        "config": {"workload": "ResNet-50 (stem, 16 bottleneck blocks, avgpool, fc) static int8, "
                               "per-channel weights, u8 NHWC activations",
                   "global_batch": world * B, "per_gpu_batch": B, "image": [3, 224, 224],
                   "parallelism": f"dp{world}"},
        "roofline": roof,
        "launch_ms": {k: round(float(np.sum(v) / n_rep), 4) for k, v in per_name.items()},
        "conv_gmac_per_image": sum(mac_img) / 1e9,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        cb, q_cpu = resnet_cpu_baseline(fp, args.cpu_seconds)
        result["cpu_baseline"] = cb["static_int8"]
        result["cpu_fp32"] = cb["fp32"]
        xe = synthetic_images(64, 31)
        with torch.no_grad():
            lab = fp.cpu()(torch.from_numpy(xe)).argmax(1)
            g = model(torch.from_numpy(xe)).argmax(1)
            c = q_cpu(torch.from_numpy(xe)).argmax(1)
        result["top1_vs_fp32"] = {"gpu_int8": (g == lab).float().mean().item() * 100,
                                  "cpu_torchao_int8": (c == lab).float().mean().item() * 100,
                                  "images": 64}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
