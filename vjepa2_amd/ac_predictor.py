"""V-JEPA 2-AC action-conditioned predictor (src/models/ac_predictor.py:17-200) on the HIP kernels:
same constructor signature, init RNG order and state_dict() keys as the reference.

The reference interleaves, per frame, the action / state (/ extrinsics) tokens in front of the frame's
H*W tokens (ac_predictor.py:161-172) and runs ACBlocks with a frame-causal attention mask
(build_action_block_causal_attention_mask, modules.py:12-23). Here:
 * the embeddings are HIP GEMMs (the 7-wide encoders' reduction dim zero-padded to 8);
 * the interleaved sequence is assembled by row scatters (vj_gather_rows, scatter mode) from the
   embedding outputs, and its backward is the matching gathers;
 * every block is the fused HIP block (functions.run_block) on a TokenLayout whose RoPE ids put each
   frame's conditioning tokens at (frame, 0, 0) (depth rotation only, ACRoPEAttention :184-200) and
   whose attention is frame-causal over blocks of cond + H*W tokens (vj_attn_fwd_fc / vj_attn_bwd_fc);
 * the frame tokens are gathered back out (ac_predictor.py:187-189) before predictor_norm / proj.
"""

import math
from functools import partial

import torch
import torch.nn as nn

from . import functions as fn
from . import ops
from .modules import ACBlock, ac_token_layout, build_action_block_causal_attention_mask, trunc_normal_


class _ScatterRowsFn(torch.autograd.Function):
    """seq[idx_i] = src_i for several sources (every row of seq written exactly once); backward gathers."""

    @staticmethod
    def forward(ctx, S, idxs, *srcs):
        D = srcs[0].shape[1]
        seq = torch.empty(S, D, dtype=torch.float32, device=srcs[0].device)
        for src, idx in zip(srcs, idxs):
            ops.scatter_rows(src.float().contiguous(), idx, seq)
        ctx.idxs = idxs
        return seq

    @staticmethod
    def backward(ctx, dseq):
        dseq = dseq.contiguous()
        return (None, None) + tuple(ops.gather_rows(dseq, idx) for idx in ctx.idxs)


class VisionTransformerPredictorAC(nn.Module):
    """ac_predictor.py:17-190."""

    def __init__(self, img_size=(224, 224), patch_size=16, num_frames=1, tubelet_size=2, embed_dim=768,
                 predictor_embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                 drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0, norm_layer=nn.LayerNorm, init_std=0.02,
                 uniform_power=True, use_silu=False, wide_silu=True, is_frame_causal=True,
                 use_activation_checkpointing=False, use_rope=True, action_embed_dim=7, use_extrinsics=False,
                 **kwargs):
        super().__init__()
        self.is_frame_causal = is_frame_causal
        self.use_extrinsics = use_extrinsics
        self.predictor_embed = nn.Linear(embed_dim, predictor_embed_dim, bias=True)
        self.action_encoder = nn.Linear(action_embed_dim, predictor_embed_dim, bias=True)
        self.state_encoder = nn.Linear(action_embed_dim, predictor_embed_dim, bias=True)
        self.extrinsics_encoder = nn.Linear(action_embed_dim - 1, predictor_embed_dim, bias=True)
        if type(img_size) is int:
            img_size = (img_size, img_size)
        self.img_height, self.img_width = img_size
        self.patch_size = patch_size
        self.num_frames = num_frames
        self.tubelet_size = tubelet_size
        self.is_video = num_frames > 1
        self.grid_height = img_size[0] // self.patch_size
        self.grid_width = img_size[1] // self.patch_size
        self.use_activation_checkpointing = use_activation_checkpointing
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, depth)]
        self.uniform_power = uniform_power
        self.use_rope = use_rope
        if not use_rope:
            raise NotImplementedError("the AC predictor without RoPE is not on the HIP path (configs use RoPE)")
        self.predictor_blocks = nn.ModuleList([
            ACBlock(use_rope=use_rope, grid_size=self.grid_height, dim=predictor_embed_dim, num_heads=num_heads,
                    mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=qk_scale, drop=drop_rate,
                    act_layer=nn.SiLU if use_silu else nn.GELU, wide_silu=wide_silu, attn_drop=attn_drop_rate,
                    drop_path=dpr[i], norm_layer=norm_layer) for i in range(depth)])
        self.predictor_norm = norm_layer(predictor_embed_dim)
        self.predictor_proj = nn.Linear(predictor_embed_dim, embed_dim, bias=True)
        self.init_std = init_std
        self.apply(self._init_weights)
        self._rescale_blocks()
        attn_mask = None
        if self.is_frame_causal:
            attn_mask = build_action_block_causal_attention_mask(self.num_frames // self.tubelet_size,
                                                                 self.grid_height, self.grid_width,
                                                                 add_tokens=3 if use_extrinsics else 2)
        self.attn_mask = attn_mask
        self._idx_cache = {}

    def _init_weights(self, m):
        """ac_predictor.py:124-131."""
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=self.init_std)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    def _rescale_blocks(self):
        """ac_predictor.py:133-139."""
        for layer_id, layer in enumerate(self.predictor_blocks):
            layer.attn.proj.weight.data.div_(math.sqrt(2.0 * (layer_id + 1)))
            layer.mlp.fc2.weight.data.div_(math.sqrt(2.0 * (layer_id + 1)))

    def _indices(self, B, T, cond, device):
        """Rows of the interleaved [B*T*(cond + H*W)] sequence taken by each source (int32, device)."""
        key = (B, T, cond, str(device))
        c = self._idx_cache.get(key)
        if c is None:
            hw = self.grid_height * self.grid_width
            n_t = cond + hw
            base = (torch.arange(B * T, device=device) * n_t)[:, None]
            conds = [(base + i).reshape(-1).to(torch.int32).contiguous() for i in range(cond)]
            frame = (base + cond + torch.arange(hw, device=device)[None, :]).reshape(-1).to(torch.int32).contiguous()
            c = (conds, frame)
            self._idx_cache[key] = c
        return c

    def forward(self, x, actions, states, extrinsics=None):
        """ac_predictor.py:141-190: x [B, T*H*W, embed_dim] context tokens, actions / states [B, T, 7]
        (extrinsics [B, T, 6]) -> [B, T*H*W, embed_dim] (f32)."""
        B, N_ctxt, C = x.shape
        hw = self.grid_height * self.grid_width
        T = N_ctxt // hw
        cond = 3 if self.use_extrinsics else 2
        e = fn.run_linear(x.reshape(B * N_ctxt, C), self.predictor_embed, out_dtype=torch.float32)
        a = fn.run_linear(actions.reshape(B * T, -1), self.action_encoder, out_dtype=torch.float32)
        s = fn.run_linear(states.reshape(B * T, -1), self.state_encoder, out_dtype=torch.float32)
        srcs = [a, s]
        if self.use_extrinsics:
            srcs.append(fn.run_linear(extrinsics.reshape(B * T, -1), self.extrinsics_encoder, out_dtype=torch.float32))
        conds, frame = self._indices(B, T, cond, x.device)
        S = B * T * (cond + hw)
        seq = _ScatterRowsFn.apply(S, conds + [frame], *srcs, e)
        if self.attn_mask is not None and T > self.num_frames // self.tubelet_size:
            raise ValueError("more frames than the frame-causal mask was built for (ac_predictor.py:174)")
        lay = ac_token_layout(B, T, self.grid_height, self.grid_width, cond, self.attn_mask is not None, x.device)
        for blk in self.predictor_blocks:
            seq = fn.run_block(seq, blk, lay)
        rows = fn.gather_rows(seq, frame)
        y = fn.run_layernorm(rows, self.predictor_norm, out_dtype=torch.bfloat16)
        out = fn.run_linear(y, self.predictor_proj, out_dtype=torch.float32)
        return out.reshape(B, T * hw, -1)


def vit_ac_predictor(**kwargs):
    """ac_predictor.py:193-200."""
    return VisionTransformerPredictorAC(mlp_ratio=4, qkv_bias=True, norm_layer=partial(nn.LayerNorm, eps=1e-6),
                                        **kwargs)
