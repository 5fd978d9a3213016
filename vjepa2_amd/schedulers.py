"""Host-side LR / weight-decay schedules (src/utils/schedulers.py:41-93).

Same step arithmetic as the reference; the optimizer argument may be any object with
`param_groups` (our FusedAdamW) so the schedules drive the fused kernels' scalars.
"""

import math


class WarmupCosineSchedule:
    def __init__(self, optimizer, warmup_steps, start_lr, ref_lr, T_max, last_epoch=-1, final_lr=0.0):
        self.optimizer = optimizer
        self.start_lr, self.ref_lr, self.final_lr = start_lr, ref_lr, final_lr
        self.warmup_steps = warmup_steps
        self.T_max = T_max - warmup_steps
        self._step = 0.0

    def step(self):
        self._step += 1
        if self._step < self.warmup_steps:
            frac = float(self._step) / float(max(1, self.warmup_steps))
            lr = self.start_lr + frac * (self.ref_lr - self.start_lr)
        else:
            frac = float(self._step - self.warmup_steps) / float(max(1, self.T_max))
            cos = 0.5 * (1.0 + math.cos(math.pi * frac))
            lr = max(self.final_lr, self.final_lr + (self.ref_lr - self.final_lr) * cos)
        for g in self.optimizer.param_groups:
            g["lr"] = lr
        return lr


class CosineWDSchedule:
    def __init__(self, optimizer, ref_wd, T_max, final_wd=0.0):
        self.optimizer = optimizer
        self.ref_wd, self.final_wd, self.T_max = ref_wd, final_wd, T_max
        self._step = 0.0

    def step(self):
        self._step += 1
        frac = self._step / self.T_max
        wd = self.final_wd + (self.ref_wd - self.final_wd) * 0.5 * (1.0 + math.cos(math.pi * frac))
        wd = max(self.final_wd, wd) if self.final_wd <= self.ref_wd else min(self.final_wd, wd)
        for g in self.optimizer.param_groups:
            if not g.get("WD_exclude", False):
                g["weight_decay"] = wd
        return wd
