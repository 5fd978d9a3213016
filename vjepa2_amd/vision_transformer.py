"""Video VisionTransformer (V-JEPA 2 encoder) on the gfx950 kernels.

API-compatible with src/models/vision_transformer.py: same constructor keywords, factory functions
(vit_large, vit_giant_xformers, *_rope ...), attributes and state_dict() keys; forward(x, masks)
returns what the reference returns. Execution is token-major and ragged: all masks of a call run
as ONE pass (vision_transformer.py:188-203 runs them as one batch too, but needs equal K; the
train step runs masks of different K together through forward_ragged()).
"""

import math
from functools import partial

import numpy as np
import torch
import torch.nn as nn

from . import functions as fn
from . import ops
from .modules import Block, rescale_blocks, trunc_normal_


def _sincos_axis(dim, coords):
    # pos_embs.py:75-93: [sin(c * w_i), cos(c * w_i)], w_i = 1 / 10000^(i / (dim/2)), float64
    w = 1.0 / 10000 ** (np.arange(dim // 2, dtype=float) / (dim / 2.0))
    ang = coords.reshape(-1)[:, None] * w[None, :]
    return np.concatenate([np.sin(ang), np.cos(ang)], axis=1)


def sincos_3d_table(dim, grid, depth, uniform_power=False):
    """pos_embs.py:9-38: rows ordered (d, h, w); columns [depth | height | width] parts."""
    d, h, w = np.meshgrid(np.arange(depth, dtype=float), np.arange(grid, dtype=float), np.arange(grid, dtype=float),
                          indexing="ij")
    if uniform_power:
        dd = dh = dw = int(np.ceil(dim / 6) * 2)
    else:
        dd, dh, dw = dim // 2, dim // 4, dim // 4
    return np.concatenate([_sincos_axis(dd, d), _sincos_axis(dh, h), _sincos_axis(dw, w)], axis=1)[:, :dim]


def _wait_ready(mod):
    """Staged optimizer update (train.JEPATrainer.apply_update): make the current stream wait for the
    event after which this module's weights are current, when the trainer set one."""
    ev = getattr(mod, "_vj_ready", None)
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)


class PatchEmbed3D(nn.Module):
    """patch_embed.py:26-52: Conv3d with kernel = stride = (tubelet, patch, patch), run as
    im2col-of-kept-tubelets + MFMA GEMM."""

    def __init__(self, patch_size=16, tubelet_size=2, in_chans=3, embed_dim=768):
        super().__init__()
        self.patch_size = patch_size
        self.tubelet_size = tubelet_size
        self.proj = nn.Conv3d(in_channels=in_chans, out_channels=embed_dim,
                              kernel_size=(tubelet_size, patch_size, patch_size),
                              stride=(tubelet_size, patch_size, patch_size))


class VisionTransformer(nn.Module):
    def __init__(self, img_size=(224, 224), patch_size=16, num_frames=1, tubelet_size=2, in_chans=3, embed_dim=768,
                 depth=12, num_heads=12, mlp_ratio=4.0, qkv_bias=True, qk_scale=None, drop_rate=0.0,
                 attn_drop_rate=0.0, drop_path_rate=0.0, norm_layer=nn.LayerNorm, init_std=0.02, out_layers=None,
                 uniform_power=False, use_silu=False, wide_silu=True, use_sdpa=True,
                 use_activation_checkpointing=False, use_rope=False, handle_nonsquare_inputs=True, **kwargs):
        super().__init__()
        self.num_features = self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.out_layers = out_layers
        self.handle_nonsquare_inputs = handle_nonsquare_inputs
        if isinstance(img_size, int):
            img_size = (img_size, img_size)
        self.img_height, self.img_width = img_size
        self.patch_size = patch_size
        self.num_frames = num_frames
        self.tubelet_size = tubelet_size
        self.is_video = num_frames > 1
        if not self.is_video:
            raise NotImplementedError("image (2-D patch) encoders are outside the V-JEPA video train-step path")
        # Activations are kept (288 GB HBM); recompute would change no numerics, only cost time.
        self.use_activation_checkpointing = use_activation_checkpointing
        dpr = [v.item() for v in torch.linspace(0, drop_path_rate, depth)]
        self.patch_embed = PatchEmbed3D(patch_size=patch_size, tubelet_size=tubelet_size, in_chans=in_chans,
                                        embed_dim=embed_dim)
        self.num_patches = (num_frames // tubelet_size) * (img_size[0] // patch_size) * (img_size[1] // patch_size)
        self.uniform_power = uniform_power
        self.use_rope = use_rope
        self.pos_embed = None if use_rope else nn.Parameter(torch.zeros(1, self.num_patches, embed_dim),
                                                            requires_grad=False)
        self.blocks = nn.ModuleList([
            Block(use_rope=use_rope, grid_size=img_size[0] // patch_size, grid_depth=num_frames // tubelet_size,
                  dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, use_sdpa=use_sdpa, qkv_bias=qkv_bias,
                  qk_scale=qk_scale, drop=drop_rate, act_layer=nn.SiLU if use_silu else nn.GELU, wide_silu=wide_silu,
                  attn_drop=attn_drop_rate, drop_path=dpr[i], norm_layer=norm_layer) for i in range(depth)])
        self.norm = norm_layer(embed_dim)
        if self.pos_embed is not None:
            t = sincos_3d_table(embed_dim, self.img_height // patch_size, num_frames // tubelet_size, uniform_power)
            self.pos_embed.data.copy_(torch.from_numpy(t).float().unsqueeze(0))
        self.init_std = init_std
        self.apply(self._init_weights)
        rescale_blocks(self.blocks)

    def _init_weights(self, m):
        # vision_transformer.py:130-145
        if isinstance(m, (nn.Linear, nn.Conv2d, nn.Conv3d)):
            trunc_normal_(m.weight, std=self.init_std)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def get_num_layers(self):
        return len(self.blocks)

    def no_weight_decay(self):
        return {}

    # ---------------------------------------------------------------------------------------------
    def _geometry(self, x):
        if x.ndim != 5:
            raise ValueError(f"expected a video batch [B, C, T, H, W], got {tuple(x.shape)}")
        B, _, T, H, W = x.shape
        Tp, Hp, Wp = T // self.tubelet_size, H // self.patch_size, W // self.patch_size
        if self.handle_nonsquare_inputs:
            tpf, tpr = Hp * Wp, Wp
        else:
            g = self.img_height // self.patch_size
            tpf, tpr = g * g, g
        return B, Tp, Hp, Wp, tpf, tpr

    def interpolate_pos_encoding(self, x, pos_embed):
        """vision_transformer.py:215-272 (video branch)."""
        _, N, dim = pos_embed.shape
        _, _, T, H, W = x.shape
        if H == self.img_height and W == self.img_width and T == self.num_frames:
            return pos_embed
        if H == self.img_height and W == self.img_width and T < self.num_frames:
            return pos_embed[:, :int((T // self.tubelet_size) * (H // self.patch_size) * (W // self.patch_size))]
        Nt = self.num_frames // self.tubelet_size
        Nh, Nw = self.img_height // self.patch_size, self.img_width // self.patch_size
        sf = ((T // self.tubelet_size) / Nt, (H // self.patch_size) / Nh, (W // self.patch_size) / Nw)
        pe = nn.functional.interpolate(pos_embed.reshape(1, Nt, Nh, Nw, dim).permute(0, 4, 1, 2, 3),
                                       scale_factor=sf, mode="trilinear")
        return pe.permute(0, 2, 3, 4, 1).reshape(1, -1, dim)

    def tokens(self, x, masks=None, out_bf16=False):
        """Patch-embed the kept tubelets of every mask -> (f32, or bf16 with out_bf16 (RoPE models only),
        [sum_m B*K_m, D], TokenLayout)."""
        x = x.float().contiguous()
        B, Tp, Hp, Wp, tpf, tpr = self._geometry(x)
        N = Tp * Hp * Wp
        if masks is None:
            lay = fn.TokenLayout([(B, N)], ids=None, ids_mod=N, tpf=tpf, tpr=tpr)
        else:
            masks = [m.to(device=x.device, dtype=torch.int64).contiguous() for m in masks]
            lay = fn.TokenLayout([(B, m.shape[1]) for m in masks], ids=ops.ids_to_int32(masks), ids_mod=N,
                                 tpf=tpf, tpr=tpr)
        pos = None
        if self.pos_embed is not None:
            pos = self.interpolate_pos_encoding(x, self.pos_embed)[0].float().contiguous()
        _wait_ready(self.patch_embed)
        t = fn.run_patch_embed(x, self.patch_embed, masks, pos_table=pos, pos_ids=lay.ids, pos_mod=N,
                               out_bf16=out_bf16)
        return t, lay

    def bf16_residual_ok(self):
        """Whether the reference's bf16 autocast keeps this encoder's residual stream in bf16: the
        Conv3d tokens are bf16 and, with RoPE, no f32 pos-embed is added (vision_transformer.py:183-186
        would promote them to f32); and no active drop_path (not built on the bf16 training path)."""
        return self.pos_embed is None and not any(
            getattr(b.drop_path, "drop_prob", 0.0) and b.drop_path.training for b in self.blocks)

    def forward_ragged(self, x, masks, out_dtype=torch.bfloat16, final_norm=True, fp8=False, bf16_residual=False):
        """All masks in ONE pass. Returns (tokens [sum_m B*K_m, D], layout). fp8: QKV / fc1 GEMMs on
        the fp8 MFMA (forward-only, functions.block_forward_fp8). bf16_residual: the residual stream in
        bf16, as the reference's autocast keeps it (x = x + proj(...) in bf16); with gradients (the
        trained context encoder) only where bf16_residual_ok(), and the gradient stream is bf16 too."""
        direct = bf16_residual and self.pos_embed is None and not fp8
        if bf16_residual and not direct and torch.is_grad_enabled() and any(
                p.requires_grad for p in self.parameters()):
            raise NotImplementedError("bf16 residual training needs a RoPE encoder without pos-embed")
        t, lay = self.tokens(x, masks, out_bf16=direct)
        if bf16_residual and not direct:
            t = ops.cast_bf16(t)
        for blk in self.blocks:
            _wait_ready(blk)
            t = fn.run_block(t, blk, lay, fp8=fp8)
        if final_norm:
            _wait_ready(self.norm)
            t = fn.run_layernorm(t, self.norm, out_dtype=out_dtype)
        return t, lay

    @torch.no_grad()
    def forward_features(self, x, fp8=False, bf16_residual=False):
        """All tokens, no final norm (residual stream [B*N, D]: f32, or bf16 with bf16_residual); used
        by the target encoder, whose final norm is fused into the JEPA loss kernel."""
        t, _ = self.forward_ragged(x, None, final_norm=False, fp8=fp8, bf16_residual=bf16_residual and not fp8)
        return t

    def forward(self, x, masks=None):
        """vision_transformer.py:161-213."""
        if masks is not None and not isinstance(masks, list):
            masks = [masks]
        t, lay = self.tokens(x, masks)
        outs = []
        for i, blk in enumerate(self.blocks):
            t = fn.run_block(t, blk, lay)
            if self.out_layers is not None and i in self.out_layers:
                outs.append(self._reshape(fn.run_layernorm(t, self.norm), lay))
        if self.out_layers is not None:
            return outs
        if self.norm is not None:
            t = fn.run_layernorm(t, self.norm)
        return self._reshape(t, lay)

    @torch.no_grad()
    def forward_fp32(self, x, masks=None):
        """fp32-operand parity mode of forward(): f32 operands and intermediates throughout (f32 MFMA
        GEMMs, exact-softmax attention, the same LayerNorm / RoPE kernels). Not a training path: it
        isolates the bf16 path's operand rounding in the comparison with the fp32 reference."""
        if masks is not None and not isinstance(masks, list):
            masks = [masks]
        x = x.float().contiguous()
        B, Tp, Hp, Wp, tpf, tpr = self._geometry(x)
        N = Tp * Hp * Wp
        if masks is None:
            lay = fn.TokenLayout([(B, N)], ids=None, ids_mod=N, tpf=tpf, tpr=tpr)
        else:
            masks = [m.to(device=x.device, dtype=torch.int64).contiguous() for m in masks]
            lay = fn.TokenLayout([(B, m.shape[1]) for m in masks], ids=ops.ids_to_int32(masks), ids_mod=N,
                                 tpf=tpf, tpr=tpr)
        pos = None
        if self.pos_embed is not None:
            pos = self.interpolate_pos_encoding(x, self.pos_embed)[0].float().contiguous()
        t = fn.patch_embed_forward_f32(x, self.patch_embed, masks, pos_table=pos, pos_ids=lay.ids, pos_mod=N)
        for blk in self.blocks:
            t = fn.block_forward_f32(t, blk, lay)
        if self.norm is not None:
            t, _, _ = ops.layernorm_fwd(t, self.norm.weight, self.norm.bias, self.norm.eps, out_dtype=torch.float32,
                                        want_stats=False)
        return self._reshape(t, lay)

    @staticmethod
    def _reshape(t, lay):
        lens = {l for _, l in lay.groups}
        if len(lens) != 1:
            raise ValueError("masks of different lengths cannot be stacked into one batch (use forward_ragged)")
        return t.reshape(-1, lens.pop(), t.shape[-1])


# ------------------------------------------------------------------------------------------------
# Factories (vision_transformer.py:275-475): head dims 64 (large, giant_xformers), 80 (huge), 88 (giant).
def _ln():
    return partial(nn.LayerNorm, eps=1e-6)


def _vit(embed_dim, depth, num_heads, mlp_ratio, use_rope=False):
    def make(patch_size=16, **kwargs):
        if use_rope:
            kwargs["use_rope"] = True
        return VisionTransformer(patch_size=patch_size, embed_dim=embed_dim, depth=depth, num_heads=num_heads,
                                 mlp_ratio=mlp_ratio, qkv_bias=True, norm_layer=_ln(), **kwargs)

    return make


vit_tiny = _vit(192, 12, 3, 4)
vit_small = _vit(384, 12, 6, 4)
vit_base = _vit(768, 12, 12, 4)
vit_large = _vit(1024, 24, 16, 4)
vit_huge = _vit(1280, 32, 16, 4)
vit_giant = _vit(1408, 40, 16, 48 / 11)
vit_giant_xformers = _vit(1408, 40, 22, 48 / 11)
vit_large_rope = _vit(1024, 24, 16, 4, use_rope=True)
vit_huge_rope = _vit(1280, 32, 16, 4, use_rope=True)
vit_giant_rope = _vit(1408, 40, 16, 48 / 11, use_rope=True)
vit_giant_xformers_rope = _vit(1408, 40, 22, 48 / 11, use_rope=True)

VIT_EMBED_DIMS = {"vit_tiny": 192, "vit_small": 384, "vit_base": 768, "vit_large": 1024, "vit_huge": 1280,
                  "vit_giant": 1408}
