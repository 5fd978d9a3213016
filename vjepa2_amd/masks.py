"""JEPA multi-block 3-D mask generation (host side, in the data-loader collate, like the reference).

Bit-exact with src/masks/multiseq_multiblock3d.py:16-239 for the same (iteration counter, torch
global RNG state): the block SIZE is drawn from a torch.Generator seeded with the shared iteration
counter; block POSITIONS from the global torch RNG, in the same call order (top, left, start per
block). Masks are sorted ascending int64 token ids, truncated to the batch minimum.
"""

import math
from multiprocessing import Value

import numpy as np
import torch


class MaskCollator:
    """multiseq_multiblock3d.py:16-76: one generator per (frames-per-clip, mask config)."""

    def __init__(self, cfgs_mask, dataset_fpcs, crop_size=(224, 224), patch_size=(16, 16), tubelet_size=2,
                 device_masks=False):
        # device_masks: the collate (a data-loader worker) only makes the reference's RNG draws and
        # returns MaskSpec objects; materialize() builds the masks on the GPU in the training process
        self.device_masks = device_masks
        self.mask_generators = {}
        for fpc in dataset_fpcs:
            self.mask_generators[fpc] = [
                _MaskGenerator(crop_size=crop_size, num_frames=fpc, spatial_patch_size=patch_size,
                               temporal_patch_size=tubelet_size, spatial_pred_mask_scale=m.get("spatial_scale"),
                               temporal_pred_mask_scale=m.get("temporal_scale"), aspect_ratio=m.get("aspect_ratio"),
                               npred=m.get("num_blocks"), max_context_frames_ratio=m.get("max_temporal_keep", 1.0),
                               max_keep=m.get("max_keep", None), full_complement=m.get("full_complement", False),
                               pred_full_complement=m.get("pred_full_complement", False),
                               inv_block=m.get("inv_block", False)) for m in cfgs_mask]

    def step(self):
        for gens in self.mask_generators.values():
            for g in gens:
                g.step()

    def __call__(self, batch):
        """batch: [(buffer, label, clip_indices)]; grouped by frames-per-clip (len of last clip index list)."""
        by_fpc = {fpc: [] for fpc in self.mask_generators}
        for sample in batch:
            by_fpc[len(sample[-1][-1])].append(sample)
        out = []
        for fpc, samples in by_fpc.items():
            if not samples:
                continue
            collated = torch.utils.data.default_collate(samples)
            if self.device_masks:
                out.append((collated, [gen.draw(len(samples)) for gen in self.mask_generators[fpc]], None))
                continue
            enc, pred = [], []
            for gen in self.mask_generators[fpc]:
                e, p = gen(len(samples))
                enc.append(e)
                pred.append(p)
            out.append((collated, enc, pred))
        return out


class _MaskGenerator:
    def __init__(self, crop_size=(224, 224), num_frames=16, spatial_patch_size=(16, 16), temporal_patch_size=2,
                 spatial_pred_mask_scale=(0.2, 0.8), temporal_pred_mask_scale=(1.0, 1.0), aspect_ratio=(0.3, 3.0),
                 npred=1, max_context_frames_ratio=1.0, max_keep=None, inv_block=False, full_complement=False,
                 pred_full_complement=False):
        crop = crop_size if isinstance(crop_size, tuple) else (crop_size, crop_size)
        psz = spatial_patch_size if isinstance(spatial_patch_size, tuple) else (spatial_patch_size,) * 2
        self.height, self.width = crop[0] // psz[0], crop[1] // psz[1]
        self.duration = num_frames // temporal_patch_size
        self.aspect_ratio = aspect_ratio
        self.spatial_pred_mask_scale = spatial_pred_mask_scale
        self.temporal_pred_mask_scale = temporal_pred_mask_scale
        self.npred = npred
        self.max_context_duration = max(1, int(self.duration * max_context_frames_ratio))
        self.max_keep = max_keep
        self.inv_block = inv_block
        self.full_complement = full_complement
        self.pred_full_complement = pred_full_complement
        self._itr_counter = Value("i", -1)  # shared across data-loader workers

    def step(self):
        with self._itr_counter.get_lock():
            self._itr_counter.value += 1
            return self._itr_counter.value

    def _block_size(self, g):
        """multiseq_multiblock3d.py:129-153: three draws from the seeded generator."""
        def draw(lo_hi):
            r = torch.rand(1, generator=g).item()
            return lo_hi[0] + r * (lo_hi[1] - lo_hi[0])

        t = max(1, int(self.duration * draw(self.temporal_pred_mask_scale)))
        keep = int(self.height * self.width * draw(self.spatial_pred_mask_scale))
        ar = draw(self.aspect_ratio)
        h = min(int(round(math.sqrt(keep * ar))), self.height)
        w = min(int(round(math.sqrt(keep / ar))), self.width)
        return t, h, w

    def _context_grid(self, size):
        """Product of npred 'ones except one block' grids (:155-171, :193-198); global RNG."""
        t, h, w = size
        grid = torch.ones((self.duration, self.height, self.width), dtype=torch.int32)
        for _ in range(self.npred):
            top = torch.randint(0, self.height - h + 1, (1,))
            left = torch.randint(0, self.width - w + 1, (1,))
            start = torch.randint(0, self.duration - t + 1, (1,))
            blk = torch.ones_like(grid)
            blk[start:start + t, top:top + h, left:left + w] = 0
            if self.max_context_duration < self.duration:
                blk[self.max_context_duration:] = 0
            grid *= blk
        return grid.flatten()

    def draw(self, batch_size):
        """The reference's RNG draws for one collate, nothing else (host, in the data-loader worker):
        the block size from the iteration-seeded generator, npred (top, left, start) positions per
        sample from the global RNG in the reference's call order, redrawn while a sample's context
        would be empty (:191-208; decided on a boolean grid). Returns a MaskSpec."""
        g = torch.Generator()
        g.manual_seed(self.step())
        t, h, w = self._block_size(g)
        boxes = np.empty((batch_size, self.npred, 3), dtype=np.int32)
        grid = np.empty((self.duration, self.height, self.width), dtype=bool)
        for b in range(batch_size):
            while True:
                grid.fill(True)
                grid[self.max_context_duration:] = False
                for j in range(self.npred):
                    top = int(torch.randint(0, self.height - h + 1, (1,)))
                    left = int(torch.randint(0, self.width - w + 1, (1,)))
                    start = int(torch.randint(0, self.duration - t + 1, (1,)))
                    boxes[b, j] = (start, top, left)
                    grid[start:start + t, top:top + h, left:left + w] = False
                if grid.any():
                    break
        return MaskSpec((self.duration, self.height, self.width), (t, h, w), self.max_context_duration, boxes,
                        self.max_keep, 1 if self.full_complement else (2 if self.pred_full_complement else 0),
                        self.inv_block)

    def __call__(self, batch_size):
        g = torch.Generator()
        g.manual_seed(self.step())
        size = self._block_size(g)
        enc, pred = [], []
        total = self.duration * self.height * self.width
        k_enc = k_pred = total
        for _ in range(batch_size):
            while True:
                grid = self._context_grid(size)
                keep = torch.nonzero(grid).reshape(-1)
                if keep.numel() == 0:
                    continue  # empty context: redraw (:191-208)
                drop = torch.nonzero(grid == 0).reshape(-1)
                k_enc, k_pred = min(k_enc, keep.numel()), min(k_pred, drop.numel())
                enc.append(keep)
                pred.append(drop)
                break
        if self.max_keep is not None:
            k_enc = min(k_enc, self.max_keep)
        enc = [m[:k_enc] for m in enc]
        pred = [m[:k_pred] for m in pred]
        if self.full_complement:
            pred = [_complement(m, total) for m in enc]
        elif self.pred_full_complement:
            enc = [_complement(m, total) for m in pred]
        enc, pred = torch.stack(enc), torch.stack(pred)
        return (pred, enc) if self.inv_block else (enc, pred)


def _complement(ids, total):
    keep = torch.ones(total, dtype=torch.bool)
    keep[ids] = False
    return torch.nonzero(keep).reshape(-1).to(ids.dtype)


class MaskSpec:
    """One mask config's draws for one collate (picklable, a few hundred bytes): grid (duration,
    height, width), block size (t, h, w), context frame limit, block positions int32 [B, npred, 3]
    as (start, top, left), max_keep, complement mode (0, 1 = full_complement, 2 =
    pred_full_complement), inv_block."""

    __slots__ = ("grid", "size", "max_ctx", "boxes", "max_keep", "mode", "inv_block")

    def __init__(self, grid, size, max_ctx, boxes, max_keep, mode, inv_block):
        self.grid, self.size, self.max_ctx, self.boxes = tuple(grid), tuple(size), int(max_ctx), boxes
        self.max_keep, self.mode, self.inv_block = max_keep, int(mode), bool(inv_block)

    def build(self, device):
        """(masks_enc, masks_pred) int64 [B, K] on `device` (vj_mask_count / vj_mask_emit), equal to
        what _MaskGenerator.__call__ returns for the same draws. One host sync: the batch-minimum
        lengths size the outputs."""
        from . import ops

        duration, height, width = self.grid
        t, h, w = self.size
        B, npred = self.boxes.shape[0], self.boxes.shape[1]
        N = duration * height * width
        boxes = torch.from_numpy(self.boxes).to(device)
        counts = torch.empty(B, dtype=torch.int32, device=device)
        ops.mask_count(B, duration, height, width, npred, boxes, t, h, w, self.max_ctx, counts)
        kept = counts.cpu()
        k_enc, k_pred = int(kept.min()), int(N - kept.max())
        if self.max_keep is not None:
            k_enc = min(k_enc, int(self.max_keep))
        le = N - k_pred if self.mode == 2 else k_enc
        lp = N - k_enc if self.mode == 1 else k_pred
        enc = torch.empty(B, le, dtype=torch.int64, device=device)
        pred = torch.empty(B, lp, dtype=torch.int64, device=device)
        ops.mask_emit(B, duration, height, width, npred, boxes, t, h, w, self.max_ctx, self.mode, k_enc, k_pred, enc,
                      pred)
        return (pred, enc) if self.inv_block else (enc, pred)


def materialize(entry, device):
    """One collated (fpc-group) entry -> (clips, masks_enc list, masks_pred list) with the masks on
    `device`: host masks are copied, MaskSpecs are built there."""
    collated, enc, pred = entry
    if pred is None:  # device_masks collate: enc holds one MaskSpec per mask config
        built = [spec.build(device) for spec in enc]
        return collated, [e for e, _ in built], [p for _, p in built]
    return (collated, [m.to(device, non_blocking=True) for m in enc],
            [m.to(device, non_blocking=True) for m in pred])
