"""Flat parameter arenas, fused AdamW and fused EMA (MI355X memory layout for the optimizer path).

Every trainable tensor of a model lives in ONE flat fp32 buffer (its nn.Parameter becomes a view),
with a parallel fp32 gradient buffer (param.grad views), AdamW moments and a bf16 shadow that the
GEMMs read. The optimizer and the EMA are then single grid-stride kernels over the arena
(12 B/param for EMA, 28 B/param + 2 B bf16 shadow for AdamW), not hundreds of small launches, and
the gradient buffer doubles as the data-parallel all-reduce buffer.

Layout choices (HBM, 288 GB per GPU): params ordered by backward readiness (last layer first) so
all-reduce buckets are contiguous slices that fill in order; every param padded to 8 elements so
every view is 16-B aligned for the bf16 DMA loads; weight-decay and no-decay params in separate
arenas (the reference's 4 AdamW param groups, app/vjepa/utils.py:224-237).

The optimizer's state_dict() is numbered exactly like torch.optim.AdamW's over the reference's
param groups (app/vjepa/utils.py:224-238: named_parameters() order per group, frozen parameters
included, no state for parameters that never received a gradient), so checkpoints interchange
with the reference's `opt` entry (app/vjepa/train.py:318-329, app/vjepa/utils.py:121).
"""

import numpy as np
import torch

from . import ops
from .functions import SHADOW_EPOCH

ALIGN = 8

# torch.optim.AdamW param-group defaults (torch 2.10), written into state_dict() groups so a
# torch.optim.AdamW built like the reference's init_opt loads them unchanged
_TORCH_ADAMW_KEYS = dict(amsgrad=False, maximize=False, foreach=None, capturable=False, differentiable=False,
                         fused=None, decoupled_weight_decay=True)


def wd_split(named_params):
    """app/vjepa/utils.py:224-237: weights decay, biases and 1-D params do not."""
    wd, nowd = [], []
    for n, p in named_params:
        (nowd if ("bias" in n) or (len(p.shape) == 1) else wd).append((n, p))
    return wd, nowd


def readiness_order(named_params):
    """Backward produces gradients last-layer-first: reverse registration order."""
    return list(reversed(list(named_params)))


def _padded(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


class FlatArena:
    def __init__(self, named_params, device, grads=True, opt_state=True, name=""):
        self.name = name
        self.names = [n for n, _ in named_params]
        self.params = [p for _, p in named_params]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _padded(p.numel())
        self.numel = max(off, ALIGN)
        f32 = dict(dtype=torch.float32, device=device)
        self.data = torch.zeros(self.numel, **f32)
        self.bf16 = torch.zeros(self.numel, dtype=torch.bfloat16, device=device)
        self.grad = torch.zeros(self.numel, **f32) if grads else None
        self.exp_avg = torch.zeros(self.numel, **f32) if opt_state else None
        self.exp_avg_sq = torch.zeros(self.numel, **f32) if opt_state else None
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            view = self.data[o:o + n].view(p.shape)
            view.copy_(p.data.to(device=device, dtype=torch.float32))
            p.data = view
            if grads:
                p.grad = self.grad[o:o + n].view(p.shape)
                p._vj_arena = self
                p._vj_gepoch = 0
            p._vj_bf16 = self.bf16[o:o + n].view(p.shape)
        self.epoch = 0  # gradient epoch: bumped by zero_grad(); a param's grad is current iff its epoch matches
        self.sync_bf16()

    def sync_bf16(self):
        """Refresh the bf16 shadow after the fp32 params were changed outside the fused kernels."""
        ops.cast_bf16(self.data, out=self.bf16)
        SHADOW_EPOCH[0] += 1

    def index(self, p):
        return next(i for i, q in enumerate(self.params) if q is p)

    def segment(self, p):
        i = self.index(p)
        return self.offsets[i], self.params[i].numel()

    def span(self, i, j):
        """[lo, hi) of params i .. j-1 (contiguous, padding included)."""
        return self.offsets[i], self.offsets[j - 1] + _padded(self.params[j - 1].numel())

    def zero_grad(self):
        """Zero the gradients, lazily for the weights that a weight-gradient GEMM overwrites on its
        first write of a step (functions.wgrad_buf marks them): those keep their old values until
        then (no fill pass over ~1.3 GB of ViT-L gradients, and the GEMM epilogue does not read them
        back). Every other gradient is zeroed here, in contiguous runs.

        Consequence for callers: between zero_grad() and finalize_grads() (run by compute_grads /
        check_finite / step) the .grad of a marked weight is NOT valid (it holds the previous step's
        values until its first write). Write such gradients only through functions.wgrad_buf /
        grad_buf, which zero or overwrite on the first touch; an external `p.grad += ...` (e.g. a
        torch AccumulateGrad) before that first touch would add onto stale data."""
        if self.grad is None:
            return
        self.epoch += 1
        ow = [getattr(p, "_vj_ow", False) for p in self.params]
        if not any(ow):
            self.grad.zero_()
            for p in self.params:
                p._vj_gepoch = self.epoch
            return
        i, n = 0, len(self.params)
        while i < n:
            if ow[i]:
                i += 1
                continue
            j = i
            while j < n and not ow[j]:
                self.params[j]._vj_gepoch = self.epoch
                j += 1
            lo, hi = self.span(i, j)
            self.grad[lo:hi].zero_()
            i = j

    def finalize_grads(self):
        """Zero the lazily zeroed gradients nothing wrote this step (their values are a previous
        step's): after the backward, before anything reads the whole gradient arena."""
        if self.grad is None:
            return
        for p in self.params:
            if p._vj_gepoch != self.epoch:
                p.grad.zero_()
                p._vj_gepoch = self.epoch


class FusedAdamW:
    """torch.optim.AdamW semantics (decoupled weight decay, bias correction) over arenas: one kernel
    launch per run of parameters with equal step count (normally one per arena = one per param
    group of app/vjepa/utils.py:207-255), bf16 shadow written in the same pass. `param_groups`
    mirrors torch's so the LR / WD schedulers drive it.

    Step counts are per parameter, as in torch: a parameter excluded from a step (an unused mask
    token, whose grad is None in the reference) does not advance, and a step skipped for an inf/NaN
    gradient (GradScaler.step, train.py:446-451) advances nothing. The skip is decided on the device
    (no host sync in the step); the host learns it lazily from a pinned copy of the flag at the next
    step() / state_dict()."""

    def __init__(self, arenas, wd_exclude, betas=(0.9, 0.999), eps=1e-8, lr=1e-3, weight_decay=1e-2,
                 ref_groups=None):
        self.arenas = arenas
        self.param_groups = []
        for a, ex in zip(arenas, wd_exclude):  # ex: None (no key: decayed group) or the WD_exclude flag
            g = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay if ex is None else 0.0,
                     **_TORCH_ADAMW_KEYS)
            if ex is not None:
                g["WD_exclude"] = bool(ex)
            g["params"] = a.params
            self.param_groups.append(g)
        # the reference's per-group parameter lists (named_parameters order, frozen params included)
        self.ref_groups = ref_groups if ref_groups is not None else [readiness_order(zip(a.names, a.params))
                                                                     for a in arenas]
        self.where = {}
        for i, a in enumerate(arenas):
            for j, p in enumerate(a.params):
                self.where[id(p)] = (i, j)
        self.pstep = [np.zeros(len(a.params), dtype=np.int64) for a in arenas]
        self.found_inf = None
        self._pending = None  # (pinned flag copy, event, [(arena, param indices advanced)])

    @property
    def steps(self):
        """Per-arena step count (of its first parameter; all equal unless some were excluded)."""
        self._resolve()
        return [int(s.max()) if len(s) else 0 for s in self.pstep]

    def _resolve(self):
        if self._pending is None:
            return
        flag, ev, advanced = self._pending
        ev.synchronize()
        if int(flag[0]) != 0:  # that step was skipped on the device
            for i, idx in advanced:
                self.pstep[i][idx] -= 1
        self._pending = None

    def step(self, grad_scale=1.0, found_inf=None, exclude=(), ema=None, stages=None):
        """One AdamW step over every arena. ema = (targets, momentum), targets[i] the target arena of
        arena i (same layout) or None: the EMA of train.py:456-465 is fused into the AdamW pass of that
        arena (the online parameters are read once); an arena with excluded parameters gets the plain
        EMA after its AdamW instead.

        stages: optional list of parameter lists in the order the next forward uses them (e.g. patch
        embedding, block 0, block 1, ...): the update is issued stage by stage (every arena's slice of a
        stage, then the next stage) and a HIP event is recorded on the current stream after each;
        returns those events (parameters in no stage form a last stage). Each stage's parameters must be
        consecutive in every arena (they are: arenas hold named_parameters() order reversed). Without
        stages: one pass per arena (None returned)."""
        self._resolve()
        for a in self.arenas:
            a.finalize_grads()
        ex = {id(p) for p in exclude}
        advanced = []
        late_ema = []
        work = []  # per arena: (arena index, active mask, fuse, target arena)
        for i, (g, a) in enumerate(zip(self.param_groups, self.arenas)):
            act = np.array([id(p) not in ex for p in a.params], dtype=bool)
            tgt = ema[0][i] if ema is not None else None
            fuse = tgt is not None and bool(act.all()) and tgt.numel == a.numel
            if tgt is not None and not fuse:
                late_ema.append((tgt, a))
            work.append((i, act, fuse, tgt))
        if stages is not None and late_ema:
            # the per-stage events would be recorded before these arenas' EMA writes, so a reader
            # waiting on them (the next target forward) would race with it. Checked before any step
            # count advances, so a caller may catch this and retry without stages.
            raise ValueError("stages: every EMA'd arena must take the fused AdamW + EMA pass (no excluded "
                             "parameters, equal layout)")
        for i, act, _, _ in work:
            self.pstep[i][act] += 1
            advanced.append((i, np.nonzero(act)[0]))

        def run(i, act, fuse, tgt, j, n):
            # maximal runs of active params with equal step count in params [j, n) of arena i
            g, a, st = self.param_groups[i], self.arenas[i], self.pstep[i]
            b1, b2 = g["betas"]
            wd = 0.0 if g.get("WD_exclude", False) else g["weight_decay"]
            while j < n:
                if not act[j]:
                    j += 1
                    continue
                k = j + 1
                while k < n and act[k] and st[k] == st[j]:
                    k += 1
                lo, hi = a.span(j, k)
                if fuse:
                    ops.adamw_ema(a.data[lo:hi], a.grad[lo:hi], a.exp_avg[lo:hi], a.exp_avg_sq[lo:hi], a.bf16[lo:hi],
                                  g["lr"], b1, b2, g["eps"], wd, int(st[j]), tgt.data[lo:hi], tgt.bf16[lo:hi], ema[1],
                                  grad_scale=grad_scale, found_inf=found_inf)
                else:
                    ops.adamw(a.data[lo:hi], a.grad[lo:hi], a.exp_avg[lo:hi], a.exp_avg_sq[lo:hi], a.bf16[lo:hi],
                              g["lr"], b1, b2, g["eps"], wd, int(st[j]), grad_scale=grad_scale, found_inf=found_inf)
                j = k

        events = None
        if stages is None:
            for i, act, fuse, tgt in work:
                run(i, act, fuse, tgt, 0, len(act))
        else:
            events = []
            ranges = self._stage_ranges(stages)
            for s in range(len(ranges)):
                for i, act, fuse, tgt in work:
                    j, n = ranges[s][i]
                    run(i, act, fuse, tgt, j, n)
                ev = torch.cuda.Event()
                ev.record()
                events.append(ev)
        for t, a in late_ema:
            ops.ema(t.data, a.data, ema[1], t.bf16)
        SHADOW_EPOCH[0] += 1  # the bf16 shadows changed: cached W^T copies are stale
        if found_inf is not None:
            flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
            flag.copy_(found_inf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pending = (flag, ev, advanced)
        return events

    def _stage_ranges(self, stages):
        """Per stage, per arena: the [j0, j1) parameter-index range of the stage's parameters
        (empty (0, 0) when the arena holds none); cached per stage list."""
        key = tuple(tuple(id(p) for p in st) for st in stages)
        if getattr(self, "_ranges_key", None) == key:
            return self._ranges
        sid = {}
        for s, st in enumerate(stages):
            for p in st:
                sid[id(p)] = s
        last = len(stages)
        ranges = [[(0, 0)] * len(self.arenas) for _ in range(last + 1)]
        for i, a in enumerate(self.arenas):
            per = {}
            for j, p in enumerate(a.params):
                per.setdefault(sid.get(id(p), last), []).append(j)
            for s, idx in per.items():
                if idx[-1] - idx[0] + 1 != len(idx):
                    raise ValueError(f"stage {s}: its parameters are not consecutive in arena {a.name!r}")
                ranges[s][i] = (idx[0], idx[-1] + 1)
        self._ranges_key, self._ranges = key, ranges
        return ranges

    def zero_grad(self, set_to_none=False):
        for a in self.arenas:
            a.zero_grad()

    def check_finite(self):
        """GradScaler inf/NaN detection over every gradient arena -> device flag (no host sync)."""
        for a in self.arenas:
            a.finalize_grads()
        if self.found_inf is None:
            self.found_inf = torch.zeros(1, dtype=torch.int32, device=self.arenas[0].data.device)
        self.found_inf.zero_()
        for a in self.arenas:
            ops.check_finite(a.grad, self.found_inf)
        return self.found_inf

    def state_dict(self):
        """torch.optim.AdamW.state_dict() of the reference's optimizer (app/vjepa/utils.py:224-239):
        parameters numbered across the 4 groups in named_parameters() order; state only for
        parameters that have taken a step."""
        self._resolve()
        state, groups, idx = {}, [], 0
        for g, refs in zip(self.param_groups, self.ref_groups):
            ids = []
            for _, p in refs:
                loc = self.where.get(id(p))
                if loc is not None and self.pstep[loc[0]][loc[1]] > 0:
                    i, j = loc
                    a = self.arenas[i]
                    o, n = a.offsets[j], p.numel()
                    state[idx] = dict(step=torch.tensor(float(self.pstep[i][j])),
                                      exp_avg=a.exp_avg[o:o + n].view(p.shape).detach().cpu().clone(),
                                      exp_avg_sq=a.exp_avg_sq[o:o + n].view(p.shape).detach().cpu().clone())
                ids.append(idx)
                idx += 1
            sg = {k: v for k, v in g.items() if k != "params"}
            sg["params"] = ids
            groups.append(sg)
        return dict(state=state, param_groups=groups)

    def load_state_dict(self, sd):
        """Accepts the reference's torch.optim.AdamW state (or ours): state entries are matched to
        parameters by their index in the reference numbering."""
        self._resolve()
        if len(sd["param_groups"]) != len(self.param_groups):
            raise ValueError(f"optimizer state has {len(sd['param_groups'])} param groups, expected "
                             f"{len(self.param_groups)}")
        for g, refs, sg in zip(self.param_groups, self.ref_groups, sd["param_groups"]):
            if len(sg["params"]) != len(refs):
                raise ValueError(f"param group of {len(sg['params'])} params in the state, {len(refs)} in the model")
            for k in ("lr", "weight_decay", "betas", "eps"):
                if k in sg:
                    g[k] = tuple(sg[k]) if k == "betas" else sg[k]
            for pid, (pname, p) in zip(sg["params"], refs):
                loc = self.where.get(id(p))
                st = sd["state"].get(pid, sd["state"].get(str(pid)))
                if loc is None:
                    continue
                i, j = loc
                a = self.arenas[i]
                o, n = a.offsets[j], p.numel()
                if not st:
                    self.pstep[i][j] = 0
                    a.exp_avg[o:o + n].zero_()
                    a.exp_avg_sq[o:o + n].zero_()
                    continue
                if st["exp_avg"].numel() != n:
                    raise ValueError(f"state of {pname}: {st['exp_avg'].numel()} elements, parameter has {n}")
                a.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
                a.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                self.pstep[i][j] = int(float(st["step"]))


def fused_ema(target_arenas, online_arenas, momentum):
    """train.py:456-465: target = target * m + (1 - m) * online, per arena, bf16 shadow refreshed."""
    for t, o in zip(target_arenas, online_arenas):
        ops.ema(t.data, o.data, momentum, t.bf16)
    SHADOW_EPOCH[0] += 1
