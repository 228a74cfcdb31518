"""InferenceBenchmark — drop-in for /root/reference/utils/inference_benchmark.py:6-157.

Same constructor, methods, arguments and return values as the reference
(warm_up :14-28, measure_inference_time :30-79, measure_throughput :81-105,
compare_models :107-157).  One deliberate difference: the
reference brackets ``model(data)`` with ``time.time()`` and never synchronizes
the device, which on a GPU times only the kernel launches.  Here every timed
call is bracketed by a device synchronization when the data lives on a GPU, so
the numbers are real images/sec.  Messages are in English.
"""
from __future__ import annotations

import time
import warnings

import numpy as np
import torch


def _sync(device):
    if torch.cuda.is_available() and str(device).startswith("cuda"):
        torch.cuda.synchronize()


class InferenceBenchmark:
    def __init__(self, test_loader, device="cpu"):
        self.test_loader = test_loader
        self.device = device

    def _timed(self, model, data):
        _sync(self.device)
        t0 = time.time()
        model(data)
        _sync(self.device)
        return time.time() - t0

    def warm_up(self, model, num_iterations=10):
        print("Warming up model...")
        model.eval()
        model.to(self.device)
        data, _ = next(iter(self.test_loader))
        data = data.to(self.device)
        with torch.no_grad():
            for _ in range(num_iterations):
                model(data)
        _sync(self.device)

    def measure_inference_time(self, model, batch_size=1, num_iterations=100, verbose=True):
        model.eval()
        model.to(self.device)
        data, _ = next(iter(self.test_loader))
        single = data[0].unsqueeze(0).to(self.device)
        with torch.no_grad():
            single_times = [self._timed(model, single) * 1000 for _ in range(num_iterations)]
        single_mean, single_std = float(np.mean(single_times)), float(np.std(single_times))
        if verbose:
            print(f"Single-image latency: {single_mean:.2f} ± {single_std:.2f} ms")
        batch_data, _ = next(iter(self.test_loader))
        batch_data = batch_data[:batch_size].to(self.device)
        with torch.no_grad():
            batch_times = [self._timed(model, batch_data) * 1000 for _ in range(num_iterations)]
        batch_mean, batch_std = float(np.mean(batch_times)), float(np.std(batch_times))
        per_image = batch_mean / batch_size
        if verbose:
            print(f"Batch {batch_size} latency: {batch_mean:.2f} ± {batch_std:.2f} ms")
            print(f"Per-image latency (batched): {per_image:.4f} ms")
        return {"single": (single_mean, single_std), "batch": (batch_mean, batch_std),
                "per_image": per_image}

    def measure_throughput(self, model, batch_size=1, num_iterations=100, verbose=True):
        """images/sec = batch_size * iterations / sum(per-call time) (:100)."""
        model.eval()
        model.to(self.device)
        data, _ = next(iter(self.test_loader))
        data = data[:batch_size].to(self.device)
        n = data.shape[0]
        if n < batch_size:
            # the reference runs on the smaller slice (:90) but counts batch_size
            # images per call (:100); run the same slice and count what ran
            warnings.warn(f"loader batch {n} < requested batch_size {batch_size}: "
                          f"measuring at batch {n}")
        total = 0.0
        with torch.no_grad():
            for _ in range(num_iterations):
                total += self._timed(model, data)
        throughput = n * num_iterations / total
        if verbose:
            print(f"Throughput at batch {batch_size}: {throughput:.2f} images/sec")
        return throughput

    def compare_models(self, models_dict, batch_size=32, num_iterations=100, verbose=True):
        print("\nComparing model inference speed...")
        results = {}
        for name, model in models_dict.items():
            print(f"\nBenchmarking {name}...")
            self.warm_up(model)
            times = self.measure_inference_time(model, batch_size=batch_size,
                                                num_iterations=num_iterations, verbose=verbose)
            self.warm_up(model)
            t1 = self.measure_throughput(model, batch_size=1, num_iterations=num_iterations,
                                         verbose=verbose)
            t32 = self.measure_throughput(model, batch_size=32, num_iterations=num_iterations,
                                          verbose=verbose)
            results[name] = {"single_inference_time": times["single"][0],
                             "batch_inference_time": times["batch"][0],
                             "per_image_time": times["per_image"],
                             "throughput_1": t1, "throughput_32": t32}
        print("\n=== Inference speed comparison ===")
        for name, r in results.items():
            print(f"\n{name}:\n  single-image latency: {r['single_inference_time']:.2f} ms"
                  f"\n  per-image latency (batched): {r['per_image_time']:.4f} ms"
                  f"\n  throughput (batch 32): {r['throughput_32']:.2f} images/sec")
        return {name: r["throughput_32"] for name, r in results.items()}
