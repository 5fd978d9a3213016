"""Multi-clip frozen-encoder wrapper of the video-classification evals
(evals/video_classification_frozen/modelcustom/vit_encoder_multiclip.py:87-162, ClipAggregation):
every (clip, view) goes through the encoder as one batch, the tokens of a view's clips are
concatenated along time, and an optional 1-D temporal sincos embedding is added at each clip's frame
indices. The encoder is the HIP VisionTransformer; the optional embedding add is vj_add_rows.
"""

import os

import numpy as np
import torch
import torch.nn as nn

from . import ops


def get_1d_sincos_pos_embed(embed_dim, grid_size):
    """src/models/utils/pos_embs.py:96-105 (float64 numpy, cls_token=False): [grid_size, embed_dim]."""
    pos = np.arange(grid_size, dtype=float)
    omega = np.arange(embed_dim // 2, dtype=np.float64)
    omega /= embed_dim / 2.0
    omega = 1.0 / 10000**omega
    out = np.einsum("m,d->md", pos.reshape(-1), omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1)


class ClipAggregation(nn.Module):
    """vit_encoder_multiclip.py:87-162: process each clip independently and concatenate all tokens."""

    def __init__(self, model, tubelet_size=2, max_frames=128, use_pos_embed=False):
        super().__init__()
        self.model = model
        self.tubelet_size = tubelet_size
        self.embed_dim = embed_dim = model.embed_dim
        self.num_heads = model.num_heads
        self.pos_embed = None
        if use_pos_embed:
            max_T = max_frames // tubelet_size
            self.pos_embed = nn.Parameter(torch.zeros(1, max_T, embed_dim), requires_grad=False)
            sincos = get_1d_sincos_pos_embed(embed_dim, max_T)
            with torch.no_grad():
                self.pos_embed.copy_(torch.from_numpy(sincos).float().unsqueeze(0))

    def forward(self, x, clip_indices=None):
        """x: list over clips of lists over views of [B, C, F, H, W]; clip_indices: list over clips of
        [B, F] frame indices. Returns a list over views of [B, num_clips * T * S, D] (f32)."""
        num_clips = len(x)
        num_views = len(x[0])
        B, C, Fr, H, W = x[0][0].size()
        xb = torch.cat([torch.cat(xi, dim=0) for xi in x], dim=0)
        outputs = self.model(xb)  # [num_clips * num_views * B, N, D]
        _, N, D = outputs.size()
        T = Fr // self.tubelet_size
        S = N // T
        eff_B = B * num_views
        views = []
        for j in range(num_views):
            # [num_clips, B, T*S, D] of this view -> [B, num_clips*T*S, D] (time-major concatenation)
            o = torch.stack([outputs[i * eff_B + j * B:i * eff_B + (j + 1) * B] for i in range(num_clips)], 1)
            o = o.reshape(B, num_clips * T * S, D).contiguous()
            if self.pos_embed is not None and clip_indices is not None:
                # row (b, c, t, s) += pos_embed[clip_indices[c][b, t * tubelet]] (apply_masks of the table)
                idx = torch.stack([ci[:, ::self.tubelet_size] for ci in clip_indices], 1)  # [B, clips, T]
                # CPU indices (the eval loaders' clip_indices) are validated here and raise as the
                # reference's gather would; device indices are not read back (no host sync per forward)
                # unless VJ_CHECK_INDICES=1 (debug): vj_add_rows never reads a table row outside
                # [0, rows) and leaves such a row unchanged
                if not idx.is_cuda or os.environ.get("VJ_CHECK_INDICES", "0") == "1":
                    lo, hi = int(idx.min()), int(idx.max())
                    if lo < 0 or hi >= self.pos_embed.shape[1]:
                        raise IndexError(f"clip index {hi if hi >= self.pos_embed.shape[1] else lo} out of range "
                                         f"for the temporal pos_embed of {self.pos_embed.shape[1]} frames")
                idx = idx.to(device=o.device, dtype=torch.int32)
                idx = idx.reshape(B, num_clips * T, 1).expand(B, num_clips * T, S).reshape(-1).contiguous()
                table = self.pos_embed[0].detach().float().contiguous()
                ops.add_rows(o.view(-1, D), table, idx=idx)
            views.append(o)
        return views
