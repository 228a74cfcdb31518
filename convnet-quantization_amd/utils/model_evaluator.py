"""ModelEvaluator — top-1/top-5 of /root/reference/utils/model_evaluator.py:15-55
(``topk(5, 1, True, True)``; ties -> lowest index), and the GPU counterpart the
reference lacks: ``device=None`` keeps each model on its
own device instead of forcing ``model.cpu()`` (:20, :30-31).  The reference's
class-accuracy/compare helpers (:57-204) reduce to the same argmax."""
from __future__ import annotations

import torch


class ModelEvaluator:
    def __init__(self, test_loader, device="cpu"):
        self.test_loader = test_loader
        self.device = device

    def evaluate_accuracy(self, model, verbose=True):
        model.eval()
        if self.device == "cpu":
            model = model.cpu()  # reference semantics; our int8 models keep GPU compute
        c1 = c5 = total = 0
        with torch.no_grad():
            for images, labels in self.test_loader:
                out = model(images if self.device == "cpu" else images.to(self.device))
                out = out.cpu()
                _, pred = out.topk(5, 1, True, True)
                pred = pred.t()
                correct = pred.eq(labels.cpu().view(1, -1).expand_as(pred))
                c1 += correct[0].sum().item()
                c5 += correct.sum().item()
                total += labels.size(0)
        top1, top5 = 100.0 * c1 / total, 100.0 * c5 / total
        if verbose:
            print(f"Top-1 Accuracy: {top1:.2f}%\nTop-5 Accuracy: {top5:.2f}%")
        return top1, top5

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
