"""CPU, world_size 2 (gloo): the data-parallel gradient path.

GradReducer all-reduces flat gradient arenas bucket by bucket as layers report ready (out of order
readiness, an unused parameter, tail segments), and the result equals the average of the per-rank
gradients after the 1/world scale AdamW applies. Also checks init_distributed's env rendezvous."""

import os

import torch
import torch.multiprocessing as mp
import torch.nn as nn


def _worker(rank, world, port, q, overlap=True):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        from vjepa2_amd.distributed import GradReducer, init_distributed

        w, r = init_distributed(backend="gloo")
        assert (w, r) == (world, rank)
        torch.manual_seed(0)
        mods = [nn.Linear(64, 64) for _ in range(5)]  # same structure on every rank
        weights = [m.weight for m in mods]
        biases = [m.bias for m in mods]
        flat_w = torch.zeros(5 * 4096)
        flat_b = torch.zeros(5 * 64)
        for i in range(5):
            flat_w[i * 4096:(i + 1) * 4096] = (rank + 1) * (i + 1)  # rank-specific "gradients"
            flat_b[i * 64:(i + 1) * 64] = (rank + 1) * 10.0
        red = GradReducer([(flat_w, [(p, i * 4096, 4096) for i, p in enumerate(weights)])],
                          tail_segments=[(flat_b, [(p, i * 64, 64) for i, p in enumerate(biases)])],
                          bucket_mb=32e3 / (1 << 20), overlap=overlap)  # ~2 params per bucket
        order = [4, 3, 1, 0]  # module 2 never reports (unused parameter)
        for i in order:
            red.mark_ready(mods[i])
        red.finish()
        ok_w = all(torch.all(flat_w[i * 4096:(i + 1) * 4096] == sum(k + 1 for k in range(world)) * (i + 1))
                   for i in range(5))
        ok_b = bool(torch.all(flat_b == 10.0 * sum(k + 1 for k in range(world))))
        q.put((rank, ok_w, ok_b))
        import torch.distributed as dist

        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


import pytest  # noqa: E402


@pytest.mark.parametrize("overlap", [True, False])
def test_grad_reducer_two_ranks(overlap):
    """overlap=False (VJ_ALLREDUCE=end): every bucket goes out at finish(), same result."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 400) + (0 if overlap else 401)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ok_w, ok_b in res:
        assert ok_w is True and ok_b is True, (rank, ok_w, ok_b)


def _two_reducers_worker(rank, world, port, q):
    """Two armed GradReducers in one process whose backward hooks interleave differently on the two
    ranks, on the weight-gradient-stream path (collectives queued until the next stream join; the
    stream calls stubbed, since this runs on the CPU). Each reducer's collectives must pair with the
    same reducer's on the other rank, and a reset() after a failed backward must drop what it queued."""
    try:
        import contextlib

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        from vjepa2_amd import functions
        from vjepa2_amd.distributed import GradReducer, init_distributed

        class _Side:
            def wait_stream(self, s):
                pass

        functions.wgrad_stream = lambda: _Side()
        torch.cuda.current_stream = lambda *a: None
        torch.cuda.stream = lambda s: contextlib.nullcontext()
        init_distributed(backend="gloo")

        def build(tag):
            mods = [nn.Linear(32, 32, bias=False) for _ in range(4)]
            flat = torch.zeros(4 * 1024)
            red = GradReducer([(flat, [(m.weight, i * 1024, 1024) for i, m in enumerate(mods)])],
                              bucket_mb=4096 / (1 << 20))  # one bucket per module, all the same size
            return mods, flat, red

        A, B = build("A"), build("B")

        def fill(flat, base):
            for i in range(4):
                flat[i * 1024:(i + 1) * 1024] = (rank + 1) * (base + i)

        # a backward that fails after queueing a bucket (rank 0 only): reset() must drop it
        if rank == 0:
            A[2].mark_ready(A[0][0])
            assert len(A[2]._after_join) == 1
            A[2].reset()
            assert len(A[2]._after_join) == 0
        fill(A[1], 1)
        fill(B[1], 100)
        order = [(A, 0), (B, 0), (A, 1), (B, 1), (A, 2), (B, 2), (A, 3), (B, 3)]
        if rank == 1:  # the other rank's hooks interleave the other way round
            order = [(B, 0), (A, 0), (B, 1), (A, 1), (B, 2), (A, 2), (B, 3), (A, 3)]
        for k, (r, i) in enumerate(order):
            r[2].mark_ready(r[0][i])
            if k == 3:
                functions._drain_join_queues()  # a weight-gradient stream join in the middle
        A[2].finish()
        B[2].finish()
        s = sum(k + 1 for k in range(world))
        ok_a = all(torch.all(A[1][i * 1024:(i + 1) * 1024] == s * (1 + i)) for i in range(4))
        ok_b = all(torch.all(B[1][i * 1024:(i + 1) * 1024] == s * (100 + i)) for i in range(4))
        q.put((rank, ok_a, ok_b))
        import torch.distributed as dist

        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


def test_two_armed_reducers_one_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29100 + (os.getpid() % 300)
    ps = [ctx.Process(target=_two_reducers_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ok_a, ok_b in res:
        assert ok_a is True and ok_b is True, (rank, ok_a, ok_b)
