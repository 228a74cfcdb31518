"""fp32 SimpleConvNet — drop-in for /root/reference/models/baseline_model.py.

Same topology and parameter names as the reference (:13-40) so its
``state_dict`` (and checkpoints in the ``{'model_state_dict', ...}`` format of
main.py:22-26 / model_trainer.py:93-99) load unchanged; same Kaiming fan_out
init statistics (:45-56).  This fp32 module is the calibration source of the
int8 path and the fp32 accuracy baseline; the int8 hot path runs in
``qconvnet.qmodel.QuantizedConvNet``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

# (in_channels, out_channels, pool after this conv) for conv1..conv6
CONV_TABLE = ((3, 64, False), (64, 64, True), (64, 128, False), (128, 128, True),
              (128, 256, False), (256, 256, True))
FLAT = 256 * 4 * 4


class SimpleConvNet(nn.Module):
    def __init__(self):
        super().__init__()
        for idx, (cin, cout, _) in enumerate(CONV_TABLE, start=1):
            self.add_module(f"conv{idx}", nn.Conv2d(cin, cout, kernel_size=3, padding=1))
            self.add_module(f"bn{idx}", nn.BatchNorm2d(cout))
        for blk in (1, 2, 3):
            self.add_module(f"pool{blk}", nn.MaxPool2d(2, 2))
            self.add_module(f"dropout{blk}", nn.Dropout(0.25))
        self.fc1 = nn.Linear(FLAT, 512)
        self.bn7 = nn.BatchNorm1d(512)
        self.dropout4 = nn.Dropout(0.5)
        self.fc2 = nn.Linear(512, 10)
        self._init_params()

    def _init_params(self):
        for mod in self.modules():
            if isinstance(mod, (nn.Conv2d, nn.Linear)):
                nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
                nn.init.zeros_(mod.bias)
            elif isinstance(mod, nn.BatchNorm2d):
                nn.init.ones_(mod.weight)
                nn.init.zeros_(mod.bias)

    def forward(self, x):
        blk = 0
        for idx, (_, _, pool) in enumerate(CONV_TABLE, start=1):
            x = F.relu(getattr(self, f"bn{idx}")(getattr(self, f"conv{idx}")(x)))
            if pool:
                blk += 1
                x = getattr(self, f"dropout{blk}")(getattr(self, f"pool{blk}")(x))
        x = x.reshape(-1, FLAT)
        x = self.dropout4(F.relu(self.bn7(self.fc1(x))))
        return self.fc2(x)


def load_checkpoint_state(obj):
    """Accept a bare state_dict or the reference's checkpoint dict
    ({'model_state_dict': ..., 'best_accuracy': ...}, main.py:22-26)."""
    if isinstance(obj, dict) and "model_state_dict" in obj:
        return obj["model_state_dict"]
    return obj


def recalibrate_bn(model, images):
    """Synthetic-weight helper (random-init BN statistics make
    the argmax degenerate): set every BatchNorm's running stats to the batch
    statistics of ``images`` (train-mode forward, cumulative average), then
    return the model in eval mode.  Parameters are not touched."""
    model.train()
    for m in model.modules():
        if isinstance(m, nn.Dropout):
            m.eval()
    bns = [m for m in model.modules() if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d))]
    saved = [m.momentum for m in bns]
    for m in bns:
        m.reset_running_stats()
        m.momentum = None
    with torch.no_grad():
        model(images)
    for m, mom in zip(bns, saved):
        m.momentum = mom
    return model.eval()


def synthetic_model(seed=0, calib_images=None):
    """Random-init SimpleConvNet (torch seed) with BN recalibrated on
    ``calib_images`` — the benchmark's stand-in for trained weights."""
    torch.manual_seed(seed)
    model = SimpleConvNet()
    if calib_images is not None:
        recalibrate_bn(model, calib_images)
    return model.eval()


def trained_synthetic_model(seed=0, steps=400, batch=256, device="cuda", lr=2e-3):
    """SimpleConvNet trained on the synthetic 10-class task
    (qconvnet.data.synthetic_task) — a bench/test fixture standing in for the
    reference's trained CIFAR-10 checkpoint (model_trainer.py), which is not
    available offline.  A trained net has real decision margins, so top-1
    deltas between quantization schemes mean what they mean on CIFAR-10."""
    from qconvnet import data
    torch.manual_seed(seed)
    dev = torch.device(device)
    model = SimpleConvNet().to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, steps)
    model.train()
    for it in range(steps):
        x, y = data.synthetic_task(batch, 10_000 + seed * 100_003 + it)
        x, y = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
        loss = torch.nn.functional.cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        sched.step()
    return model.eval().cpu()


def test_model():
    model = SimpleConvNet()
    y = model(torch.randn(1, 3, 32, 32))
    print(f"Output shape: {tuple(y.shape)}")
    return model


if __name__ == "__main__":
    test_model()
