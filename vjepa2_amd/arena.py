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
"""

import torch

from . import ops

ALIGN = 8


def wd_split(named_params):
    """app/vjepa/utils.py:224-237: weights decay, biases and 1-D params do not."""
    wd, nowd = [], []
    for n, p in named_params:
        (nowd if ("bias" in n) or (len(p.shape) == 1) else wd).append((n, p))
    return wd, nowd


def readiness_order(named_params):
    """Backward produces gradients last-layer-first: reverse registration order."""
    return list(reversed(list(named_params)))


class FlatArena:
    def __init__(self, named_params, device, grads=True, opt_state=True, name=""):
        self.name = name
        self.names = [n for n, _ in named_params]
        self.params = [p for _, p in named_params]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
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
            p._vj_bf16 = self.bf16[o:o + n].view(p.shape)
        self.sync_bf16()

    def sync_bf16(self):
        """Refresh the bf16 shadow after the fp32 params were changed outside the fused kernels."""
        ops.cast_bf16(self.data, out=self.bf16)

    def segment(self, p):
        i = next(i for i, q in enumerate(self.params) if q is p)
        return self.offsets[i], self.params[i].numel()

    def ranges(self, exclude=()):
        """Contiguous [lo, hi) ranges covering the arena minus the segments of `exclude` params."""
        ex = sorted((self.segment(p)[0], self.segment(p)[0] + (p.numel() + ALIGN - 1) // ALIGN * ALIGN)
                    for p in exclude if any(p is q for q in self.params))
        out, lo = [], 0
        for a, b in ex:
            if a > lo:
                out.append((lo, a))
            lo = b
        if lo < self.numel:
            out.append((lo, self.numel))
        return out

    def zero_grad(self):
        if self.grad is not None:
            self.grad.zero_()


class FusedAdamW:
    """torch.optim.AdamW semantics (decoupled weight decay, bias correction) over arenas, one kernel
    launch per arena (the four param groups of app/vjepa/utils.py:207-255), bf16 shadow written in
    the same pass. `param_groups` mirrors torch's so the LR / WD schedulers drive it."""

    def __init__(self, arenas, wd_exclude, betas=(0.9, 0.999), eps=1e-8, lr=1e-3, weight_decay=1e-2):
        self.arenas = arenas
        self.param_groups = [dict(lr=lr, weight_decay=0.0 if ex else weight_decay, WD_exclude=ex, betas=tuple(betas),
                                  eps=eps, params=a.params) for a, ex in zip(arenas, wd_exclude)]
        self.steps = [0] * len(arenas)
        self.found_inf = None

    def step(self, grad_scale=1.0, found_inf=None, exclude=()):
        for i, (g, a) in enumerate(zip(self.param_groups, self.arenas)):
            self.steps[i] += 1
            b1, b2 = g["betas"]
            wd = 0.0 if g["WD_exclude"] else g["weight_decay"]
            for lo, hi in a.ranges(exclude):
                ops.adamw(a.data[lo:hi], a.grad[lo:hi], a.exp_avg[lo:hi], a.exp_avg_sq[lo:hi], a.bf16[lo:hi], g["lr"],
                          b1, b2, g["eps"], wd, self.steps[i], grad_scale=grad_scale, found_inf=found_inf)

    def zero_grad(self, set_to_none=False):
        for a in self.arenas:
            a.zero_grad()

    def check_finite(self):
        """GradScaler inf/NaN detection over every gradient arena -> device flag (no host sync)."""
        if self.found_inf is None:
            self.found_inf = torch.zeros(1, dtype=torch.int32, device=self.arenas[0].data.device)
        self.found_inf.zero_()
        for a in self.arenas:
            ops.check_finite(a.grad, self.found_inf)
        return self.found_inf

    def state_dict(self):
        """torch.optim.AdamW-style state (param index order = arena order within each group)."""
        state, groups, idx = {}, [], 0
        for i, (g, a) in enumerate(zip(self.param_groups, self.arenas)):
            ids = []
            for p, o in zip(a.params, a.offsets):
                n = p.numel()
                state[idx] = dict(step=torch.tensor(float(self.steps[i])),
                                  exp_avg=a.exp_avg[o:o + n].view(p.shape).clone(),
                                  exp_avg_sq=a.exp_avg_sq[o:o + n].view(p.shape).clone())
                ids.append(idx)
                idx += 1
            groups.append({k: v for k, v in g.items() if k != "params"} | dict(params=ids))
        return dict(state=state, param_groups=groups)

    def load_state_dict(self, sd):
        idx = 0
        for i, (g, a) in enumerate(zip(self.param_groups, self.arenas)):
            sg = sd["param_groups"][i]
            for k in ("lr", "weight_decay", "betas", "eps"):
                if k in sg:
                    g[k] = tuple(sg[k]) if k == "betas" else sg[k]
            for p, o in zip(a.params, a.offsets):
                st = sd["state"].get(idx, sd["state"].get(str(idx)))
                idx += 1
                if not st:
                    continue
                n = p.numel()
                a.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
                a.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                self.steps[i] = int(float(st["step"]))


def fused_ema(target_arenas, online_arenas, momentum):
    """train.py:456-465: target = target * m + (1 - m) * online, per arena, bf16 shadow refreshed."""
    for t, o in zip(target_arenas, online_arenas):
        ops.ema(t.data, o.data, momentum, t.bf16)
