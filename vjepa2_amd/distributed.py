"""Process-group init and bucketed gradient all-reduce (data parallel only, like the reference).

init_distributed follows src/utils/distributed.py:17-51 (env:// rendezvous, "nccl" = RCCL on ROCm,
fallback to a world of 1). GradReducer replaces the DDP reducer (app/vjepa/train.py:279-281):
gradients already live in flat arenas ordered by backward readiness, so a bucket is a contiguous
slice; when the last layer writing into a bucket finishes its backward, the bucket's all-reduce
(SUM; the 1/world average is folded into the AdamW kernel) is issued asynchronously. With the
"nccl" backend RCCL runs it on its own HIP stream, ordered after the compute stream's work so far,
so it overlaps the rest of the backward over xGMI. Buckets are issued strictly in order, so every
rank issues the same collective sequence.
"""

import logging
import os

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)


def init_distributed(port=37129, rank_and_world_size=(None, None), backend=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    rank, world = rank_and_world_size
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if rank is None or world is None:
        env = os.environ
        if "RANK" in env and "WORLD_SIZE" in env:
            rank, world = int(env["RANK"]), int(env["WORLD_SIZE"])
        elif "SLURM_NTASKS" in env:
            rank, world = int(env["SLURM_PROCID"]), int(env["SLURM_NTASKS"])
        else:
            return 1, 0
    if world == 1:
        return 1, 0
    os.environ.setdefault("MASTER_PORT", str(port))
    if backend is None:  # VJ_DIST_BACKEND=gloo: rehearse several ranks on one device (RCCL refuses that)
        backend = os.environ.get("VJ_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    kw = {}
    if backend == "nccl" and torch.cuda.is_available():
        # the caller has bound this rank's GPU (torch.cuda.set_device(LOCAL_RANK)); RCCL connects
        # eagerly on it, so binding afterwards would put every rank on the same device
        kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    try:
        dist.init_process_group(backend=backend, world_size=world, rank=rank, **kw)
    except Exception as e:
        # The reference falls back to a single process here (distributed.py:47-49). With a world
        # size > 1 explicitly requested that silently trains unsynchronised replicas, so raise.
        raise RuntimeError(f"init_process_group({backend}, world={world}, rank={rank}) failed: {e}") from e
    return world, rank


class _Bucket:
    __slots__ = ("view", "pending", "params", "work")

    def __init__(self, view, params):
        self.view, self.params, self.pending, self.work = view, params, set(), None


class GradReducer:
    """segments: list of (flat_grad_tensor, [(param, offset, numel), ...]) in readiness order.
    Params of `tail_segments` (tiny no-decay arenas) are reduced as one bucket each at finish()."""

    def __init__(self, segments, tail_segments=(), bucket_mb=64, group=None, reserve_cus=None, overlap=None):
        self.group = group
        # overlap=False (VJ_ALLREDUCE=end): every bucket is issued at finish(), after the backward,
        # instead of as soon as its last layer is done. The collectives are then exposed (~1.30 GB per
        # step at RCCL's bus bandwidth) but never share the CUs with the backward's kernels, which on
        # one GPU cost about 2.5x the CU-time they hold (DESIGN (e), profiles/r06_rccl_proxy_ab.txt).
        if overlap is None:
            overlap = os.environ.get("VJ_ALLREDUCE", "overlap") != "end"
        self.overlap = overlap
        # CUs the persistent GEMM grids leave to RCCL's channel kernels from the first bucket of a
        # backward to finish() (ops.set_reserved_cus; DESIGN (e)). VJ_RCCL_RESERVE_CUS overrides.
        if reserve_cus is None:
            reserve_cus = int(os.environ.get("VJ_RCCL_RESERVE_CUS", "0"))
        self.reserve_cus = reserve_cus
        self._reserving = False
        self.world = dist.get_world_size(group)
        self.buckets = []
        cap = int(bucket_mb * (1 << 20)) // 4
        for flat, plist in segments:
            cur, lo = [], None
            for p, off, n in plist:
                if lo is None:
                    lo = off
                cur.append(p)
                end = off + n
                if end - lo >= cap:
                    self.buckets.append(_Bucket(flat[lo:end], cur))
                    cur, lo = [], None
            if cur:
                end = plist[-1][1] + plist[-1][2]
                self.buckets.append(_Bucket(flat[lo:end], cur))
        self.tail = [_Bucket(flat[:plist[-1][1] + plist[-1][2]], [p for p, _, _ in plist])
                     for flat, plist in tail_segments if plist]
        self.owner = {}
        for i, b in enumerate(self.buckets):
            for p in b.params:
                self.owner[id(p)] = i
        from . import functions

        self._after_join = functions.join_queue()  # this reducer's collectives awaiting a stream join
        self.reset()

    def reset(self):
        self.armed = True  # False during the backward of all but the last frames-per-clip group
        # a backward that raised after queueing buckets must not leave them to fire in the next step
        # (one rank's extra collective would desync the collective order across ranks)
        self._after_join.clear()
        if getattr(self, "_reserving", False):
            from . import ops

            ops.set_reserved_cus(0)
            self._reserving = False
        for b in self.buckets + self.tail:
            b.pending = {id(p) for p in b.params}
            b.work = None
        self.next = 0

    def _all_reduce(self, b):
        b.work = dist.all_reduce(b.view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _issue(self, b):
        # With the weight-gradient stream on (functions.wgrad_stream), the bucket's weight gradients
        # may still be in flight there, and its LayerNorm / bias gradients were written on the current
        # stream. The collective is queued (in this reducer's own queue) to go out on the weight-gradient
        # stream right after that stream's next join with the current one (the next block's first
        # weight-gradient launch, a few launches later), so it sees both without a join of its own: a
        # join per bucket cost 2.8 % of the step (profiles/r05_reducer_joins_ab.txt). Queue order =
        # bucket order on every rank.
        from . import functions

        if self.reserve_cus and not self._reserving:
            from . import ops

            ops.set_reserved_cus(self.reserve_cus)
            self._reserving = True
        if functions.wgrad_stream() is None:
            self._all_reduce(b)
            return
        self._after_join.append(lambda b=b: self._all_reduce(b))

    def _flush(self):
        """Issue this reducer's queued collectives now (one join of the weight-gradient stream)."""
        from . import functions

        functions.drain_join_queue(self._after_join)

    def mark_ready(self, module):
        """Hook called when `module`'s backward has finished writing its parameter gradients."""
        if not self.armed or not self.overlap:
            return
        for p in module.parameters():
            i = self.owner.get(id(p))
            if i is not None:
                self.buckets[i].pending.discard(id(p))
        while self.next < len(self.buckets) and not self.buckets[self.next].pending:
            self._issue(self.buckets[self.next])
            self.next += 1

    def install(self, modules):
        for m in modules:
            m._vj_grad_ready = self.mark_ready

    def finish(self):
        """Issue what is left (unused params, tails) in order and make the current stream wait."""
        while self.next < len(self.buckets):
            self._issue(self.buckets[self.next])
            self.next += 1
        for b in self.tail:
            self._issue(b)
        self._flush()
        for b in self.buckets + self.tail:
            b.work.wait()
        if self._reserving:
            from . import ops

            ops.set_reserved_cus(0)
            self._reserving = False
        self.reset()
