"""CPU, world_size 2 (gloo): the multi-GPU data path of qconvnet.dist —
contiguous sharding, rank-0 qspec broadcast, logits all-gather — reproduces
the single-process result exactly.  The per-rank "model" is the numpy oracle
(CPU restatement), standing in for the GPU forward."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "convnet-quantization_amd"), root, here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import netfix
        from oracle import qref
        from qconvnet import dist as qd
        r, w, _ = qd.init("gloo")
        assert (r, w) == (rank, world)
        z = netfix.load(False)
        spec = None
        if rank == 0:
            spec, _ = netfix.static_spec(z)
        spec = qd.broadcast_object(spec)
        qm = netfix.oracle_dict(spec)
        x = torch.from_numpy(netfix.images(z)[:8])

        def model_fn(xs):
            return torch.from_numpy(qref.static_int8_forward(xs.numpy(), qm)[0])

        out = qd.sharded_forward(model_fn, x)
        # bench.py's N > 1 loop: two batches' all-gathers in flight at once
        s, e = qd.shard(x.shape[0], world, rank)
        bufs = [torch.empty_like(out), torch.empty_like(out)]
        works = [qd.gather_logits_async(model_fn(x[s:e]), bufs[k]) for k in range(2)]
        for wk in works:
            wk.wait()
        for bf in bufs:
            assert torch.equal(bf, out)
        q.put((rank, out.numpy()))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, repr(e)))


def test_shard_bounds():
    from qconvnet.dist import shard
    for total in (0, 1, 7, 8192, 8193):
        for world in (1, 2, 3, 8):
            spans = [shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gather_matches_single_process():
    import netfix
    from oracle import qref
    z = netfix.load(False)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    assert np.array_equal(res[0], res[1])
    assert np.array_equal(res[0], z["logits"][:8])


def _range_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "convnet-quantization_amd"), root, here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from oracle import qref
        from qconvnet import dist as qd
        qd.init("gloo")
        x, qw, s_w, b = _dyn_case()
        s, e = qd.shard(x.shape[0], world, rank)
        lo, hi = torch.aminmax(torch.from_numpy(x[s:e]))   # stands in for the device observer
        mm = qd.global_minmax(torch.stack([lo, hi]))
        y = qref.linear_dynamic(x[s:e], qw, s_w, b, True, (mm[0].item(), mm[1].item()))
        q.put((rank, (mm.numpy(), y)))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as ex:
        q.put((rank, repr(ex)))


def _dyn_case():
    rng = np.random.default_rng(9)
    x = rng.standard_normal((16, 256)).astype(np.float32)
    x[3] *= 6.0          # the batch extremes sit on rank 0's shard only
    w = (rng.standard_normal((32, 256)) * 0.05).astype(np.float32)
    from oracle import qref
    s_w = qref.qparams_symmetric(w.min(), w.max())[0]
    return x, qref.quantize_weight(w, s_w), s_w, (rng.standard_normal(32) * 0.1).astype(np.float32)


def test_sharded_dynamic_linear_is_batch_exact():
    """§8(f)1: with the 2-float all-reduce of the activation range, the shards
    of a dynamic-int8 Linear reproduce the whole-batch result exactly (and
    differ from per-shard ranges, so the exchange is what makes it exact)."""
    from oracle import qref
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_range_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    x, qw, s_w, b = _dyn_case()
    full = qref.linear_dynamic(x, qw, s_w, b, True)
    assert np.array_equal(res[0][0], np.array([x.min(), x.max()], np.float32))
    assert np.array_equal(np.concatenate([res[0][1], res[1][1]]), full)
    per_shard = qref.linear_dynamic(x[8:], qw, s_w, b, True)
    assert not np.array_equal(per_shard, full[8:])
