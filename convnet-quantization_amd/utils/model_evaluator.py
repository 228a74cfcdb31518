"""ModelEvaluator — drop-in for /root/reference/utils/model_evaluator.py:10-204.

* ``evaluate_accuracy`` (:15-55): top-1/top-5 with ``topk(5, 1, True, True)``
  (ties -> lowest index);
* ``evaluate_class_accuracy`` (:57-119): per-class top-1 (``torch.max``
  argmax), sorted by accuracy, descending;
* ``compare_models`` (:121-204): overall and per-class accuracy per model.

The reference moves every quantized model to the CPU (:20, :78-81, :139-142).
Here ``model.cpu()`` on our int8 models switches only their I/O to host
tensors — the HIP kernels still do the compute — so the reference's calling
pattern runs unchanged; with ``device="cuda"`` inputs go to the GPU and no
host round trip is made (the GPU counterpart of SURVEY §8(f) row 4).
Messages are in English; the tqdm progress bars are dropped."""
from __future__ import annotations

import torch


def _model_type(model):
    if hasattr(model, "quantized"):
        return ("custom quantized model" if getattr(model, "is_custom_quantized", False)
                else "quantized model")
    return "FP32 model"


class ModelEvaluator:
    def __init__(self, test_loader, device="cpu"):
        self.test_loader = test_loader
        self.device = device

    def _place(self, model):
        """(model, input device): every model goes to self.device.  The reference
        forces quantized models to the CPU (:78-84) because fbgemm runs there;
        our int8 models compute on the GPU, and with self.device == "cpu" they
        take host tensors and keep their compute on the GPU (model.cpu())."""
        model.eval()
        if str(self.device) == "cpu":
            return model.cpu(), torch.device("cpu")
        model.to(self.device)
        return model, torch.device(self.device)

    def _predict(self, model, device):
        with torch.no_grad():
            for images, labels in self.test_loader:
                out = model(images.to(device))
                yield out.cpu(), labels.cpu()

    def evaluate_accuracy(self, model, verbose=True):
        model, device = self._place(model)
        c1 = c5 = total = 0
        for out, labels in self._predict(model, device):
            _, pred = out.topk(5, 1, True, True)
            pred = pred.t()
            correct = pred.eq(labels.view(1, -1).expand_as(pred))
            c1 += correct[0].sum().item()
            c5 += correct.sum().item()
            total += labels.size(0)
        top1, top5 = 100.0 * c1 / total, 100.0 * c5 / total
        if verbose:
            print(f"Top-1 Accuracy: {top1:.2f}%\nTop-5 Accuracy: {top5:.2f}%")
        return top1, top5

    def _class_counts(self, model, device, n_classes):
        correct = torch.zeros(n_classes, dtype=torch.float64)
        total = torch.zeros(n_classes, dtype=torch.float64)
        for out, target in self._predict(model, device):
            _, predicted = torch.max(out, 1)
            total += torch.bincount(target, minlength=n_classes)[:n_classes].double()
            hit = target[predicted == target]
            correct += torch.bincount(hit, minlength=n_classes)[:n_classes].double()
        return correct, total

    @staticmethod
    def _sorted_class_acc(classes, correct, total):
        acc = {classes[i]: 100.0 * correct[i].item() / total[i].item()
               for i in range(len(classes)) if total[i] > 0}
        return dict(sorted(acc.items(), key=lambda kv: kv[1], reverse=True))

    def evaluate_class_accuracy(self, model, classes, verbose=True):
        kind = _model_type(model)
        model, device = self._place(model)
        correct, total = self._class_counts(model, device, len(classes))
        res = self._sorted_class_acc(classes, correct, total)
        if verbose:
            print(f"\n[{kind}] per-class accuracy (top 20 classes):")
            for i, (name, a) in enumerate(res.items()):
                if i >= 20:
                    break
                print(f"{name}: {a:.2f}%")
        return res

    def compare_models(self, models_dict, classes):
        results = {}
        print("\n=== Model accuracy comparison ===")
        for name, model in models_dict.items():
            kind = _model_type(model)
            m, device = self._place(model)
            correct, total = self._class_counts(m, device, len(classes))
            accuracy = 100.0 * correct.sum().item() / total.sum().item()
            results[name] = {"accuracy": accuracy,
                             "class_accuracies": self._sorted_class_acc(classes, correct, total)}
            print(f"[{kind}] {name} accuracy: {accuracy:.2f}%")
        print("\n=== Summary ===")
        for name, r in results.items():
            print(f"[{_model_type(models_dict[name])}] {name}: {r['accuracy']:.2f}%")
        return results

    def agreement(self, model_a, model_b):
        """Share of inputs where the two models' argmax agree (%)."""
        same = total = 0
        with torch.no_grad():
            for images, _ in self.test_loader:
                a = model_a(images).cpu().argmax(1)
                b = model_b(images).cpu().argmax(1)
                same += (a == b).sum().item()
                total += images.shape[0]
        return 100.0 * same / total
