"""StaticPTQModel — drop-in for /root/reference/models/static_ptq_model.py:7-43.

Reference behaviour: a plain wrapper holding ``fp32_model`` / ``quantized_model``;
``quantize(calibration_data_loader=None)`` returns the quantized model and
``get_model_size(model)`` reports MB.  The reference's quantize() actually calls
``quantize_dynamic`` (only fc1/fc2 become int8).  Here
``quantize`` does what the class name and BASELINE config 3 promise: true
static PTQ of the whole net — BN folded, MinMax-calibrated activations, every
conv and linear int8 on the MI355X (``QuantizedConvNet``, static mode), with
torch.ao/fbgemm numerics bit for bit.  The calibration loader is used (the
reference ignores it); with none, 512 synthetic CIFAR images are used.
"""
from __future__ import annotations

import io

import torch

from models.baseline_model import SimpleConvNet, load_checkpoint_state
from qconvnet import data
from qconvnet.qmodel import QuantizedConvNet, build_qspec, calibrate, fold_state_dict


class StaticPTQModel:
    """mode="static" (default): full static int8 on the MI355X.
    mode="reference": the reference's actual semantics — quantize_dynamic on the
    unfolded net (fp32 convs + BN, dynamic int8 fc1/fc2; the dynamic Linear on
    the HIP kernel)."""

    def __init__(self, device="cuda", mode="static"):
        if mode not in ("static", "reference"):
            raise ValueError(f"unknown mode {mode!r}")
        self.fp32_model = SimpleConvNet()
        self.quantized_model = None
        self.device = device
        self.mode = mode

    def load_state_dict(self, state_dict):
        self.fp32_model.load_state_dict(load_checkpoint_state(state_dict))

    def quantize(self, calibration_data_loader=None, per_channel=False, calibration_device="cpu",
                 max_batches=None):
        """Calibrate (fp32, BN folded — the reference quantizes on the CPU, so
        does the default here) and build the int8 GPU model."""
        self.fp32_model.eval()
        if self.mode == "reference":
            from models.dynamic_ptq_model import DynamicQuantConvNet
            self.quantized_model = DynamicQuantConvNet(self.fp32_model.state_dict(), fold=False,
                                                       device=self.device)
            return self.quantized_model
        folded = fold_state_dict(self.fp32_model.state_dict())
        batches = data.calibration_batches(calibration_data_loader, max_batches)
        ranges = calibrate(folded, batches, calibration_device)
        spec = build_qspec(folded, ranges, "static", per_channel)
        self.quantized_model = QuantizedConvNet(spec, self.device)
        return self.quantized_model

    def get_model_size(self, model):
        """MB of the serialized parameters (the reference writes temp_model.pth
        into the CWD, static_ptq_model.py:36-43; this uses an in-memory buffer)."""
        buf = io.BytesIO()
        if isinstance(model, QuantizedConvNet):
            torch.save({k: v for k, v in model.spec.items()}, buf)
        else:
            torch.save(model.state_dict(), buf)
        return buf.tell() / (1024 * 1024)
