"""GPU, world_size 2 over gloo, both ranks on cuda:0: the PRODUCT multi-GPU
path of qconvnet.dist — rank-0 spec broadcast, contiguous shards through
``QuantizedConvNet`` (the HIP kernels), ``sharded_forward`` / ``gather_logits``
— reproduces the single-process forward bit for bit (the dynamic path's
range exchange is covered by test_dist_gloo and
test_gpu_parity::test_linear_dynamic_shards_with_global_range).  RCCL itself needs
one GPU per rank, so on this one-GPU box the collective is gloo; bench.py
runs the same calls over RCCL under torchrun."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _setup(rank, port):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "convnet-quantization_amd"), root, here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK="0")


def _static_worker(rank, port, q):
    _setup(rank, port)
    try:
        import netfix
        from oracle import torch_ref
        from qconvnet import dist as qd
        from qconvnet.qmodel import QuantizedConvNet
        qd.init("gloo")
        spec = netfix.static_spec(netfix.load(False))[0] if rank == 0 else None
        spec = qd.broadcast_object(spec)
        model = QuantizedConvNet(spec, "cuda:0")
        x = torch.from_numpy(torch_ref.synthetic_images(2048, 3))   # host batch, like the harness
        out = qd.sharded_forward(model, x)                           # each rank: 1024 on the GPU
        q.put((rank, out.numpy()))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, repr(e)))


def _run(target):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
    for r in range(WORLD):
        assert not isinstance(res[r], str), res[r]
    assert np.array_equal(res[0], res[1])
    return res[0]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qconvnet import _lib
    _lib.load()
    return torch.device("cuda:0")


def test_two_rank_static_product_equals_one_process(dev):
    import netfix
    from oracle import torch_ref
    from qconvnet.qmodel import QuantizedConvNet
    got = _run(_static_worker)
    model = QuantizedConvNet(netfix.static_spec(netfix.load(False))[0], dev)
    want = model(torch.from_numpy(torch_ref.synthetic_images(2048, 3))).numpy()
    assert np.array_equal(got, want)



def _bench_worker(rank, port, q):
    """bench.py's own N = 2 path (rank-0 model build + spec broadcast, per-rank
    resident batch, HIP forward, logits all-gather inside the timed step,
    barrier + max-over-ranks timing), both ranks on cuda:0 over gloo."""
    _setup(rank, port)
    os.environ["QCN_DIST_BACKEND"] = "gloo"
    try:
        import contextlib
        import io
        import json
        import sys
        import bench
        sys.argv = ["bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "256",
                    "--no-cpu", "--no-pmc"]
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            bench.main()
        line = next((ln for ln in buf.getvalue().splitlines() if ln.startswith("{")), None)
        q.put((rank, json.loads(line) if line else None))
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, repr(e)))


def test_bench_two_ranks_rehearsal(dev):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
    for r in range(WORLD):
        assert not isinstance(res[r], str), res[r]
    d = res[0]
    assert res[1] is None   # one JSON line, from rank 0
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 512 and d["value"] > 0
    assert d["config"]["collective"]
    # compute vs collective: every rank's step time and the all-gather's own time
    assert len(d["rank_ms_per_step"]) == 2 and all(t > 0 for t in d["rank_ms_per_step"])
    assert d["rank_ms_spread"] >= 0
    assert abs(d["ms_per_step"] - max(d["rank_ms_per_step"])) < 1e-6
    assert d["allgather"]["ms_mean"] > 0 and d["allgather"]["bytes_per_rank"] == 256 * 10 * 4
