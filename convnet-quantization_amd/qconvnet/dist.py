"""Multi-GPU inference: one process per GPU, images sharded
into contiguous per-rank slices, weights and calibrated qparams replicated
(calibrated once on rank 0 and broadcast), and ONE exchange per batch: an
all-gather of the fp32 logits ([shard, 10] per rank) over RCCL/xGMI
(backend "nccl" is RCCL on ROCm).  The static int8 path is batch-independent,
so the gathered logits equal a single-GPU run bit for bit.  The dynamic
(reference-mode) path adds one 2-float all-reduce per dynamic Linear
(``global_minmax``) so its activation qparams are the whole batch's.

Everything here also runs on CPU with the gloo backend (tests)."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), \
        int(os.environ.get("LOCAL_RANK", 0))


def init(backend=None):
    """Initialise the default process group from torchrun's env (no-op at
    WORLD_SIZE 1).  Returns (rank, world, local_rank)."""
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend is None:   # QCN_DIST_BACKEND=gloo: rehearsal of N ranks on one GPU
            backend = os.environ.get("QCN_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard(total, world, rank):
    """Contiguous [start, stop) of ``total`` items for ``rank`` (balanced,
    the first total % world ranks take one extra)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_object(obj, src=0):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def gather_logits(local, out=None):
    """All-gather equal-size per-rank logits into [world * shard, C] (rank
    order == image order).  ``out`` may be a preallocated buffer."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    world = dist.get_world_size()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


def gather_logits_async(local, out):
    """gather_logits without blocking: the all-gather is enqueued behind the
    current stream's work (RCCL runs it on its own stream) and the current
    stream only waits for it at ``work.wait()``, so the next batch's forward
    overlaps it (its logits must go to another buffer meanwhile).  Returns
    the work handle, or None at world size 1."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return None
    return dist.all_gather_into_tensor(out, local.contiguous(), async_op=True)


def global_minmax(mm):
    """All-reduce a [min, max] pair over the ranks (one 2-float collective:
    MIN over [min, -max]; negation is exact).  This is the exchange that makes
    a sharded dynamic-int8 Linear batch-exact: every rank then
    derives the same ChooseQuantizationParams as a single-GPU run over the
    whole batch.  Returns a new tensor on mm's device."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return mm
    t = torch.stack([mm[0], -mm[1]])
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return torch.stack([t[0], -t[1]])


def sharded_forward(model_fn, x_global, out=None):
    """Run ``model_fn`` on this rank's contiguous slice of ``x_global`` and
    all-gather the logits.  Requires the batch to divide evenly (fixed-shape
    collective); the caller pads otherwise."""
    rank = dist.get_rank() if dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_initialized() else 1
    if x_global.shape[0] % world:
        raise ValueError("global batch must be a multiple of the world size")
    s, e = shard(x_global.shape[0], world, rank)
    return gather_logits(model_fn(x_global[s:e]), out)
