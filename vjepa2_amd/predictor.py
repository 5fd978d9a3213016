"""V-JEPA 2 predictor on the gfx950 kernels (API of src/models/predictor.py).

The sort of [context | target] tokens by patch id (predictor.py:206-217) and its inverse
(:238-242) are never materialised as permuted copies: a HIP index kernel computes each token's
slot in the sorted sequence (stable rank == torch.argsort for unique ids), context rows are
scattered straight into their slots, the mask token is broadcast into the target slots, and after
the blocks only the target rows are gathered, normalised and projected.
"""

from functools import partial

import torch
import torch.nn as nn

from . import functions as fn
from . import ops
from .modules import Block, rescale_blocks, trunc_normal_
from .vision_transformer import sincos_3d_table


class PredictorLayout:
    """Index tables of one predictor pass over several (masks_x, masks_y) pairs (device int32)."""

    def __init__(self, masks_x, masks_y, N, device):
        self.B = masks_x[0].shape[0]
        self.pairs = [(int(mx.shape[1]), int(my.shape[1])) for mx, my in zip(masks_x, masks_y)]
        self.S = sum(self.B * (k + kp) for k, kp in self.pairs)
        self.R_ctx = sum(self.B * k for k, _ in self.pairs)
        self.R_tgt = sum(self.B * kp for _, kp in self.pairs)
        i32 = dict(dtype=torch.int32, device=device)
        self.pos = torch.empty(self.S, **i32)
        self.ctx_dst = torch.empty(self.R_ctx, **i32)
        self.tgt_rows = torch.empty(self.R_tgt, **i32)
        self.loss_rows = torch.empty(self.R_tgt, **i32)
        row0 = c0 = t0 = 0
        for (k, kp), mx, my in zip(self.pairs, masks_x, masks_y):
            # slots are absolute rows of the whole ragged sequence buffer (pos is indexed by slot)
            ops.pred_index(mx, my, row0, N, self.pos, self.ctx_dst[c0:c0 + self.B * k],
                           self.tgt_rows[t0:t0 + self.B * kp], self.loss_rows[t0:t0 + self.B * kp])
            row0 += self.B * (k + kp)
            c0 += self.B * k
            t0 += self.B * kp

    @property
    def groups(self):
        return [(self.B, k + kp) for k, kp in self.pairs]


class VisionTransformerPredictor(nn.Module):
    def __init__(self, img_size=(224, 224), patch_size=16, num_frames=1, tubelet_size=2, embed_dim=768,
                 predictor_embed_dim=384, depth=6, num_heads=12, mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                 drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0, norm_layer=nn.LayerNorm, init_std=0.02,
                 uniform_power=False, use_mask_tokens=False, num_mask_tokens=2, zero_init_mask_tokens=True,
                 use_silu=False, wide_silu=True, use_activation_checkpointing=False, return_all_tokens=False,
                 chop_last_n_tokens=0, use_rope=False, **kwargs):
        super().__init__()
        self.return_all_tokens = return_all_tokens
        self.chop_last_n_tokens = chop_last_n_tokens
        if chop_last_n_tokens:
            raise NotImplementedError("chop_last_n_tokens > 0 is not implemented (not used by V-JEPA configs)")
        self.predictor_embed = nn.Linear(embed_dim, predictor_embed_dim, bias=True)
        self.mask_tokens = None
        self.num_mask_tokens = 0
        if use_mask_tokens:
            self.num_mask_tokens = num_mask_tokens
            self.mask_tokens = nn.ParameterList(
                [nn.Parameter(torch.zeros(1, 1, predictor_embed_dim)) for _ in range(num_mask_tokens)])
        if isinstance(img_size, int):
            img_size = (img_size, img_size)
        self.img_height, self.img_width = img_size
        self.patch_size = patch_size
        self.num_frames = num_frames
        self.tubelet_size = tubelet_size
        self.is_video = num_frames > 1
        if not self.is_video:
            raise NotImplementedError("image predictors are outside the V-JEPA video train-step path")
        self.grid_height = img_size[0] // patch_size
        self.grid_width = img_size[1] // patch_size
        self.grid_depth = num_frames // tubelet_size
        self.use_activation_checkpointing = use_activation_checkpointing
        dpr = [v.item() for v in torch.linspace(0, drop_path_rate, depth)]
        self.num_patches = self.grid_depth * self.grid_height * self.grid_width
        self.uniform_power = uniform_power
        self.predictor_pos_embed = None
        if not use_rope:
            self.predictor_pos_embed = nn.Parameter(torch.zeros(1, self.num_patches, predictor_embed_dim),
                                                    requires_grad=False)
        self.use_rope = use_rope
        self.predictor_blocks = nn.ModuleList([
            Block(use_rope=use_rope, grid_size=self.grid_height, grid_depth=self.grid_depth, dim=predictor_embed_dim,
                  num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop_rate,
                  act_layer=nn.SiLU if use_silu else nn.GELU, wide_silu=wide_silu, attn_drop=attn_drop_rate,
                  drop_path=dpr[i], norm_layer=norm_layer) for i in range(depth)])
        self.predictor_norm = norm_layer(predictor_embed_dim)
        self.predictor_proj = nn.Linear(predictor_embed_dim, embed_dim, bias=True)
        if self.predictor_pos_embed is not None:
            t = sincos_3d_table(predictor_embed_dim, self.img_height // patch_size, self.grid_depth, uniform_power)
            self.predictor_pos_embed.data.copy_(torch.from_numpy(t).float().unsqueeze(0))
        self.init_std = init_std
        if not zero_init_mask_tokens:
            for mt in self.mask_tokens:
                trunc_normal_(mt, std=init_std)
        self.apply(self._init_weights)
        rescale_blocks(self.predictor_blocks)

    def _init_weights(self, m):
        # predictor.py:150-156
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=self.init_std)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    # ---------------------------------------------------------------------------------------------
    def layout(self, masks_x, masks_y, device, n_target=None):
        """n_target: tokens per clip of the target rows the JEPA loss gathers (loss_rows = b * n + id);
        the clip's own token count, which is below num_patches for clips shorter than num_frames
        (a frames-per-clip group with fewer frames than the model's maximum)."""
        mx = [m.to(device=device, dtype=torch.int64).contiguous() for m in masks_x]
        my = [m.to(device=device, dtype=torch.int64).contiguous() for m in masks_y]
        return PredictorLayout(mx, my, self.num_patches if n_target is None else int(n_target), device)

    def forward_ragged(self, z, masks_x, masks_y, mask_index=1, out_dtype=torch.bfloat16, layout=None,
                       n_target=None):
        """z: encoder tokens of all mask pairs, flat [sum_m B*K_m, D] (mask order). Returns
        (predictions of the target tokens, flat [sum_m B*Kp_m, D], PredictorLayout); n_target: the
        clips' tokens per sample (loss-row indexing, see layout())."""
        pl = layout if layout is not None else self.layout(masks_x, masks_y, z.device, n_target=n_target)
        e = fn.run_linear(z, self.predictor_embed, out_dtype=torch.float32)
        if self.mask_tokens is None:
            raise NotImplementedError("use_mask_tokens=False predictor is not on the V-JEPA 2 path")
        tok = self.mask_tokens[mask_index % self.num_mask_tokens]
        pos = None
        if self.predictor_pos_embed is not None:
            pos = self.predictor_pos_embed[0].float().contiguous()
        if torch.is_grad_enabled() and (e.requires_grad or tok.requires_grad):
            seq = fn._AssembleFn.apply(e, tok, pl.ctx_dst, pl.tgt_rows, pl.S, pos, pl.pos, self.mask_tokens)
        else:
            seq = fn._AssembleFn.forward(_NoCtx(), e, tok, pl.ctx_dst, pl.tgt_rows, pl.S, pos, pl.pos, self.mask_tokens)
        g = self.grid_height
        lay = fn.TokenLayout(pl.groups, ids=pl.pos, ids_mod=self.num_patches, tpf=g * g, tpr=g)
        for blk in self.predictor_blocks:
            seq = fn.run_block(seq, blk, lay)
        rows = seq if self.return_all_tokens else fn.gather_rows(seq, pl.tgt_rows)
        y = fn.run_layernorm(rows, self.predictor_norm, out_dtype=torch.bfloat16)
        return fn.run_linear(y, self.predictor_proj, out_dtype=out_dtype), pl

    def forward(self, x, masks_x, masks_y, mask_index=1, has_cls=False):
        """predictor.py:166-246 for one (masks_x, masks_y) pair per call (what the wrapper passes)."""
        if has_cls:
            raise NotImplementedError("has_cls is not used by V-JEPA pre-training")
        masks_x = masks_x if isinstance(masks_x, list) else [masks_x]
        masks_y = masks_y if isinstance(masks_y, list) else [masks_y]
        if len(masks_x) != 1 or len(masks_y) != 1:
            raise NotImplementedError("pass one mask pair per call (PredictorMultiSeqWrapper does); "
                                      "use forward_ragged for several pairs in one pass")
        B, K, D = x.shape
        z = x.reshape(B * K, D)
        if z.dtype != torch.bfloat16:
            z = ops.cast_bf16(z.float().contiguous()) if not z.requires_grad else _CastBF16.apply(z.float())
        y, pl = self.forward_ragged(z, masks_x, masks_y, mask_index=mask_index, out_dtype=torch.float32)
        n = pl.pairs[0][0] + pl.pairs[0][1] if self.return_all_tokens else pl.pairs[0][1]
        return y.reshape(B, n, -1)


class _NoCtx:
    def __setattr__(self, k, v):
        pass


class _CastBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return ops.cast_bf16(x.contiguous())

    @staticmethod
    def backward(ctx, dy):
        return dy.float()


def vit_predictor(**kwargs):
    """predictor.py:249-253."""
    return VisionTransformerPredictor(mlp_ratio=4, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                                      **kwargs)
