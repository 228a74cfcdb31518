"""In-kernel clock of the SimpleConvNet conv launches (diagnostic, not product).

Loads tools/clock/libqconvnet_clock.so (QCN_LIB) — the product library with
the three conv launches replaced by stamped copies of the same kernels — runs
the bench's forward back to back for >= 2 s (MI355X_MICROARCH.md 'DVFS
give-back' item 6), then K more steps with HIP events between launches, and
reads the last launch's per-workgroup stamps:

    clock  = (s_memtime delta) / (s_memrealtime delta) x 100 MHz, median over workgroups
    issue  = frac_at_2.4GHz x 2.4 / clock   (MFMA issue fraction at the held clock)

    python tools/clock_probe.py [--batch 1024] [--workload convnet|qdq] [--spec-file F]

Prints one JSON line.  bench.py runs it as a child with the parent's model.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG_LIB = os.environ.get("QCN_CLOCK_LIB", os.path.join(ROOT, "tools", "clock", "libqconvnet_clock.so"))
os.environ["QCN_LIB"] = DIAG_LIB   # before qconvnet is imported
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

KINDS = {"conv12": 0, "conv34": 1, "conv56": 2, "conv1_6": 3}
MFMA_MAC_PER_CLK_SIMD = 1024   # v_mfma_i32_32x32x32_i8: 32768 MAC per 32 cycles


def grid_of(name, n, ncu):
    if name == "conv1_6":              # one launch: one image per workgroup, else persistent
        return n if n <= ncu else ncu
    if name == "conv12":
        return min(n, ncu)
    if name == "conv34":               # persistent wave-specialised kernel from two images
        return ncu if n >= 2 * ncu else n      # per CU, else one image per workgroup
    if n <= ncu:                       # cout-split: two workgroups per pair of images
        return 2 * ((n + 1) // 2)
    if n >= 4 * ncu:                   # persistent wave-specialised kernel
        return ncu
    return (n + 1) // 2                # two 8x8 images per 4-wave workgroup (convpair_ga_kernel)


def layer_table(lib, g, img_per_wg, s12, T12, phases, B):
    """conv1 .. conv6 each against its own bound, from the
    stamped copy's role stamps.  Inside the one launch the two convs of a
    phase run on different waves of the same SIMDs at the same time, so each
    layer's row is its role's BUSY time (median over workgroups, summed over
    its tiles): conv1 the conv12 producer waves (4, 5), conv2 the consumer
    (wave 0: main loop + pooled epilogue), conv3 / conv5 the A-role wave 0
    (job + requant into B's patch + the next input's hand-off), conv4 / conv6
    the B-role wave 4 (pooled epilogue + job).  mfma_issue_while_busy = the
    layer's MFMA cycles per SIMD over those busy cycles, frac_at_2p4 = that x
    the phase's held clock / 2.4 GHz: the int8 rate the layer runs at while it
    runs (co-running with its phase partner).  conv1 is HBM-bound (SURVEY
    §8(d)): its row also carries its algorithmic bytes per busy time against
    8 TB/s."""
    import bench
    from qconvnet import _lib
    out, periods = {}, {}
    mfma = lambda n: bench.MAC_PER_IMAGE[n] * img_per_wg / (4 * MFMA_MAC_PER_CLK_SIMD)   # noqa: E731
    clk12 = phases.get("conv12", {}).get("clock_ghz")
    if clk12:
        c2 = np.sum(s12[:, 0, 1:T12 + 1, 1] - s12[:, 0, 1:T12 + 1, 0], axis=1)
        c1 = np.sum(0.5 * ((s12[:, 1, :T12, 1] - s12[:, 1, :T12, 0]) + (s12[:, 2, :T12, 1] - s12[:, 2, :T12, 0])), axis=1)
        for name, busy in (("conv1", c1), ("conv2", c2)):
            bc = float(np.median(busy))
            row = {"role": "conv12 producer waves 4-7" if name == "conv1" else "conv12 consumer waves 0-3",
                   "busy_cycles": bc, "mfma_cycles_per_simd": mfma(name), "clock_ghz": clk12,
                   "mfma_issue_while_busy": mfma(name) / bc, "frac_at_2p4": mfma(name) / bc * clk12 / 2.4,
                   "bound": "mfma"}
            if name == "conv1":
                gbs = bench.BYTES_PER_IMAGE["conv1"] * img_per_wg * g / (bc / (clk12 * 1e9)) / 1e9
                row.update({"bound": "hbm", "achieved_gbs": gbs, "hbm_frac": gbs / bench.PEAK_HBM_GBS,
                            "mfma_frac_at_2p4": row["frac_at_2p4"], "frac_at_2p4": gbs / bench.PEAK_HBM_GBS,
                            "frac_note": "conv1 is HBM-bound (SURVEY §8(d)): frac_at_2p4 here is its algorithmic "
                                         "bytes (fp32 input + u8 output) per busy time over 8 TB/s"})
            out[name] = row
    if hasattr(lib, "qcn_clock_read_ws16"):
        f = lib.qcn_clock_read_ws16
        f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
        w = np.zeros((g, 2, 2, 8, 3), np.uint64)
        _lib.check(f(w.ctypes.data, g), "qcn_clock_read_ws16")
        w = w.astype(np.float64)
        for ph, (a, b_, segs) in enumerate((("conv3", "conv4", 1), ("conv5", "conv6", 2))):
            pn = "conv34" if ph == 0 else "conv56"
            clk = phases.get(pn, {}).get("clock_ghz")
            T = int(np.ceil(img_per_wg / segs))
            if not clk or T + 1 >= 8:
                continue
            x = w[:, ph]
            busy_a = np.sum(x[:, 0, :T, 2] - x[:, 0, :T, 0], axis=1)
            busy_b = np.sum(x[:, 1, 1:T + 1, 2] - x[:, 1, 1:T + 1, 0], axis=1) + (x[:, 1, T + 1, 0] - x[:, 1, T, 2])
            for name, busy, role in ((a, busy_a, "A-role waves 0-3"), (b_, busy_b, "B-role waves 4-7")):
                bc = float(np.median(busy))
                out[name] = {"role": role, "busy_cycles": bc, "mfma_cycles_per_simd": mfma(name), "clock_ghz": clk,
                             "mfma_issue_while_busy": mfma(name) / bc, "frac_at_2p4": mfma(name) / bc * clk / 2.4,
                             "bound": "mfma"}
            # the pipeline's periods (median over workgroups, cycles from the
            # phase's first stamp): A runs tile p, B tile p - 1; period T is B only
            t0 = np.minimum(x[:, 0, 0, 0], x[:, 1, 0, 0])
            per = []
            for p in range(T + 1):
                row = {"period": p}
                if p < T:
                    row.update({"a_start": float(np.median(x[:, 0, p, 0] - t0)),
                                "a_job": float(np.median(x[:, 0, p, 1] - x[:, 0, p, 0])),
                                "a_epi_handoff": float(np.median(x[:, 0, p, 2] - x[:, 0, p, 1]))})
                if p >= 1:
                    row.update({"b_start": float(np.median(x[:, 1, p, 0] - t0)),
                                "b_epi": float(np.median(x[:, 1, p, 1] - x[:, 1, p, 0])),
                                "b_job": float(np.median(x[:, 1, p, 2] - x[:, 1, p, 1]))})
                per.append(row)
            per.append({"period": "end", "b_last_epi_done": float(np.median(x[:, 1, T + 1, 0] - t0))})
            periods[pn] = per
    return out, periods


def main():
    import bench
    from qconvnet import _lib, data
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--workload", choices=("convnet", "qdq"), default="convnet")
    ap.add_argument("--spec-file", default=None)
    ap.add_argument("--heat-s", type=float, default=2.5)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    B = args.batch or (1024 if args.workload == "convnet" else 256)
    lib = _lib.load()
    assert os.path.samefile(_lib.LIB_PATH, DIAG_LIB), "the diagnostic library must be the one loaded"
    fn = lib.qcn_clock_read
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    fn16 = lib.qcn_clock_read_c16
    fn16.restype, fn16.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mode = "qdq" if args.workload == "qdq" else "static"
    model, _ = bench.build_model(0, dev, False, args.spec_file, mode)
    x = torch.from_numpy(data.synthetic_images(B, 100)).to(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count

    # heat: >= heat_s of back-to-back forwards
    t0 = time.perf_counter()
    k = 0
    while True:
        model.run(x)
        k += 1
        if k % 50 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() - t0 >= args.heat_s:
                break
    names = model.kernel_names(x.shape)
    per = {n: [] for n in names}
    for _ in range(args.steps):
        m = []
        model.run(x, marks=m)
        for i, n in enumerate(names):
            per[n].append(m[i])
            per[n].append(m[i + 1])
    torch.cuda.synchronize()
    out = {"batch": B, "workload": args.workload, "heat_s": time.perf_counter() - t0,
           "heat_steps": k, "kernels": {}}
    for n in names:
        evs = per[n]
        ms = float(np.mean([evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(len(evs) // 2)]))
        rec = {"ms": ms}
        if n in KINDS:
            g = grid_of(n, B, ncu)
            buf = np.zeros((g, 4), np.uint64)
            _lib.check(fn(KINDS[n], buf.ctypes.data, g), "qcn_clock_read")
            t0_, t1_, r0_, r1_ = (buf[:, i].astype(np.float64) for i in range(4))
            cyc, rt = t1_ - t0_, r1_ - r0_
            ok = rt > 0
            ghz = cyc[ok] / rt[ok] * 0.1
            frac = 2.0 * bench.MAC_PER_IMAGE[n] * B / (ms * 1e-3) / 1e12 / bench.PEAK_INT8_TOPS
            clock = float(np.median(ghz))
            # MFMA cycles per SIMD of one workgroup (its images' MACs over its 4 SIMDs)
            img_per_wg = B / g
            mac_wg = bench.MAC_PER_IMAGE[n] * img_per_wg
            if n == "conv56" and B <= ncu:   # cout-split: conv5 of two images + half of conv6's
                mac_wg = 2 * (bench.MAC_PER_IMAGE["conv5"] + bench.MAC_PER_IMAGE["conv6"] / 2)
            mfma_cyc_wg = mac_wg / (4 * MFMA_MAC_PER_CLK_SIMD)
            rec.update({"clock_ghz": clock, "clock_ghz_p10": float(np.percentile(ghz, 10)),
                        "clock_ghz_p90": float(np.percentile(ghz, 90)),
                        "workgroups": int(g), "wg_cycles_median": float(np.median(cyc[ok])),
                        "wg_mfma_cycles_per_simd": mfma_cyc_wg,
                        "launch_span_us": float((r1_.max() - r0_.min()) / 100.0),
                        "frac_at_2p4": frac, "mfma_issue_at_clock": frac * 2.4 / clock})
            if n == "conv1_6":   # per-phase cycles of the one launch (median over workgroups)
                b16 = np.zeros((g, 8), np.uint64)
                _lib.check(fn16(b16.ctypes.data, g), "qcn_clock_read_c16")
                t = b16[:, :4].astype(np.float64)
                r = b16[:, 4:].astype(np.float64)
                rec["phase_cycles_median"] = {
                    ph: float(np.median(t[:, i + 1] - t[:, i]))
                    for i, ph in enumerate(("conv12", "conv34", "conv56"))}
                # every phase against its own bound.  A phase's MFMA
                # cycles per SIMD are its images' MACs over the workgroup's 4
                # SIMDs at 1024 MAC / clk; issue = those / the phase's cycles (at
                # the clock the chip holds in it), frac = issue x clock / 2.4 GHz
                # (the fraction of the 2.4 GHz int8 peak the phase runs at)
                table = {}
                for i, ph in enumerate(("conv12", "conv34", "conv56")):
                    cyc_p = t[:, i + 1] - t[:, i]
                    rt_p = r[:, i + 1] - r[:, i]
                    okp = rt_p > 0
                    clk_p = float(np.median(cyc_p[okp] / rt_p[okp] * 0.1))
                    cyc_med = float(np.median(cyc_p))
                    if cyc_med <= 0:   # a phase this launch does not run (a separate launch)
                        continue
                    mfma_p = bench.MAC_PER_IMAGE[ph] * img_per_wg / (4 * MFMA_MAC_PER_CLK_SIMD)
                    issue = mfma_p / cyc_med
                    table[ph] = {"us_median": float(np.median(rt_p)) / 100.0,
                                 "gop": 2.0 * bench.MAC_PER_IMAGE[ph] * B / 1e9,
                                 "cycles_median": cyc_med, "mfma_cycles_per_simd": mfma_p,
                                 "clock_ghz": clk_p, "mfma_issue_at_clock": issue,
                                 "frac_at_2p4": issue * clk_p / 2.4}
                rec["phase_table"] = table
                if hasattr(lib, "qcn_clock_read_c12"):   # conv12p per-iteration stamps
                    f12 = lib.qcn_clock_read_c12
                    f12.restype, f12.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
                    b12 = np.zeros((g, 3, 12, 3), np.uint64)
                    _lib.check(f12(b12.ctypes.data, g), "qcn_clock_read_c12")
                    s = b12.astype(np.float64)
                    T = int(round(2 * img_per_wg))   # tiles of the full workgroups
                    full = s[:, 0, T, 1] > 0
                    s = s[full]
                    it = {}
                    for j in range(T + 1):
                        top = s[:, 0, j, 0]
                        nxt = s[:, 0, j + 1, 0] if j < T else s[:, 0, j, 1]
                        it[str(j)] = {
                            "iter_cycles": float(np.median(nxt - top)),
                            "consumer_busy": float(np.median(s[:, 0, j, 1] - s[:, 0, j, 0])),
                            "consumer_mainloop": float(np.median(s[:, 0, j, 2] - s[:, 0, j, 0])) if j > 0 else 0.0,
                            "producer_w4_busy": float(np.median(s[:, 1, j, 1] - s[:, 1, j, 0])),
                            "producer_w5_busy": float(np.median(s[:, 2, j, 1] - s[:, 2, j, 0])),
                        }
                    rec["conv12_iterations"] = {"workgroups": int(full.sum()), "tiles": T, "per_iteration": it}
                    rec["layer_table"], rec["pair_periods"] = layer_table(lib, g, img_per_wg, s, T, table, B)
        out["kernels"][n] = rec
    print(json.dumps(out))
    for n, r in out["kernels"].items():
        if "clock_ghz" in r:
            print(f"# {n}: {r['ms'] * 1e3:.1f} us, clock {r['clock_ghz']:.3f} GHz "
                  f"(p10 {r['clock_ghz_p10']:.3f}, p90 {r['clock_ghz_p90']:.3f}), frac@2.4 "
                  f"{r['frac_at_2p4']:.3f}, MFMA issue at the held clock {r['mfma_issue_at_clock']:.3f}, "
                  f"WG {r['wg_cycles_median']:.0f} cyc vs {r['wg_mfma_cycles_per_simd']:.0f} MFMA cyc/SIMD",
                  file=sys.stderr)
        ci = r.get("conv12_iterations")
        if ci:
            for j, v in ci["per_iteration"].items():
                print(f"#   conv12 iter {j}: {v['iter_cycles']:.0f} cyc, consumer busy {v['consumer_busy']:.0f} (main loop {v['consumer_mainloop']:.0f}), "
                      f"producer w4 {v['producer_w4_busy']:.0f}, w5 {v['producer_w5_busy']:.0f}", file=sys.stderr)
        for ph, t in r.get("phase_table", {}).items():
            print(f"#   {ph}: {t['us_median']:.1f} us, {t['cycles_median']:.0f} cyc vs {t['mfma_cycles_per_simd']:.0f} "
                  f"MFMA cyc/SIMD, clock {t['clock_ghz']:.3f} GHz, issue {t['mfma_issue_at_clock']:.3f}, "
                  f"frac@2.4 {t['frac_at_2p4']:.3f}", file=sys.stderr)


if __name__ == "__main__":
    main()
