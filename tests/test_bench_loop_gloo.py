"""CPU, world_size 2 (gloo): bench.py's N > 1 timed step itself — the
StepLoop the metric runs (two logits slots, the all-gather of batch k issued
asynchronously while batch k+1 computes, a slot's gather waited for before
its reuse, everything drained before the clock stops) — driven through
qconvnet.dist on gloo.  The per-rank forward is the numpy oracle (the GPU
forward's CPU restatement) on the rank's contiguous shard.  Checks: the
gathered logits of the last step equal a single-process run over the whole
batch, and the fields the N > 1 bench line carries (rank_ms_per_step,
allgather) come out of the same code."""
import os
import socket

import numpy as np
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
        import bench
        import netfix
        from oracle import qref
        from qconvnet import dist as qd
        r, w, _ = qd.init("gloo")
        assert (r, w) == (rank, world)
        z = netfix.load(False)
        spec = netfix.static_spec(z)[0] if rank == 0 else None
        spec = qd.broadcast_object(spec)          # rank 0 calibrates, the rest receive
        qm = netfix.oracle_dict(spec)
        x = netfix.images(z)[:8]
        s, e = qd.shard(x.shape[0], world, rank)
        xs = x[s:e]
        calls = []

        def forward(marks=None, slot=0):
            calls.append(slot)
            return torch.from_numpy(qref.static_int8_forward(xs, qm)[0])

        loop = bench.StepLoop(forward, world, "cpu")
        warm = bench.ramp_warmup(loop.step, loop.drain, 2, world, "cpu", min_s=0.0, sync=loop.sync)
        elapsed, rank_ms = loop.timed(3)
        sus = loop.sustained(elapsed / 3, 3, xs.shape[0], seconds=0.0)
        gather = loop.allgather_timing(forward(), 3)
        got = loop.gathered[loop.last_slot].numpy()
        q.put((rank, dict(got=got, rank_ms=rank_ms, gather=gather, warm=warm, sus=sus, slots=calls,
                          elapsed=elapsed)))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


def test_bench_step_loop_two_ranks_matches_single_process():
    import netfix
    from oracle import qref
    z = netfix.load(False)
    spec, _ = netfix.static_spec(z)
    want = qref.static_int8_forward(netfix.images(z)[:8], netfix.oracle_dict(spec))[0]
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
        assert isinstance(res[r], dict), res[r]
        d = res[r]
        assert np.array_equal(d["got"], want)              # rank order == image order
        assert len(d["rank_ms"]) == world and all(v > 0 for v in d["rank_ms"])
        assert d["elapsed"] * 1e3 / 3 >= max(d["rank_ms"]) - 1e-6   # the max over ranks
        assert set(d["gather"]) >= {"ms_mean", "ms_min", "bytes_per_rank"}
        assert d["gather"]["bytes_per_rank"] == 4 * 10 * 4   # [4, 10] fp32 logits per rank
        assert d["warm"] == 2 + 5                           # W steps + the 5-step probe (min_s 0)
        assert d["sus"]["steps"] == 3
        # two slots alternate at N > 1 (slot k % 2 for step k), the last call is the timing forward
        assert d["slots"][:-1] == [k % 2 for k in range(len(d["slots"]) - 1)]
    # every rank took the same number of steps (their all-gathers paired up)
    assert len(res[0]["slots"]) == len(res[1]["slots"])


def test_bench_gpus_2_without_torchrun_starts_two_ranks():
    """`python bench.py --gpus 2` with no torchrun env starts torch.distributed.run
    with two ranks as a child (never one rank labelled two): the line reports
    n_gpus 2 and both ranks' step times.  The rehearsal mode runs the harness
    on CPU over gloo with a stand-in forward."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--rehearse",
                        "--steps", "3", "--warmup", "1", "--batch", "4"], cwd=root, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert len(d["rank_ms_per_step"]) == 2 and all(v > 0 for v in d["rank_ms_per_step"])
    assert d["config"]["global_batch"] == 8
    assert d["allgather"]["bytes_per_rank"] == 4 * 10 * 4
