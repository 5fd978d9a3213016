"""Transformer layers with the reference's constructor signatures and parameter names
(src/models/utils/modules.py): Block, RoPEAttention, Attention, MLP — so state_dict() keys and the
init-time RNG consumption match the reference exactly. Compute runs on the HIP kernels
(functions.block_forward / block_backward); these modules are parameter containers plus a
reference-compatible forward() for direct use.
"""

import math

import torch
import torch.nn as nn

from . import functions as fn
from . import ops


class MLP(nn.Module):
    """modules.py:67-83 (fc1 -> GELU(erf) -> dropout -> fc2 -> dropout; the two nn.Dropout run while
    training, on vj_dropout's element masks)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)
        if act_layer is not nn.GELU:
            raise NotImplementedError("MLP supports the exact-erf GELU (nn.GELU) on the HIP path")

    def forward(self, x):
        """modules.py:77-83: fc2(GELU(fc1(x))), fc1 + GELU fused in one GEMM epilogue."""
        shp = x.shape
        y = fn.run_sublayer(x.reshape(-1, shp[-1]), self)
        return y.reshape(*shp[:-1], y.shape[-1])


class SwiGLUFFN(nn.Module):
    """modules.py:86-106 (act_layer=nn.SiLU): fc1, fc2: in -> h (h = hidden rounded as 2/3 hidden up to a
    multiple of 8 when wide_silu), fc3: h -> out; fc3(silu(fc1 x) * fc2 x). `drop` is accepted and unused,
    as in the reference."""

    swiglu = True

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.SiLU, drop=0.0,
                 wide_silu=True):
        super().__init__()
        out_features = out_features or in_features
        hidden = hidden_features or in_features
        if wide_silu:
            hidden = (int(2 * hidden / 3) + 7) // 8 * 8
        self.fc1 = nn.Linear(in_features, hidden)
        self.fc2 = nn.Linear(in_features, hidden)
        self.act = act_layer()
        self.fc3 = nn.Linear(hidden, out_features)
        if act_layer is not nn.SiLU:
            raise NotImplementedError("SwiGLUFFN gates with SiLU (the reference builds it for act_layer=nn.SiLU)")
        if hidden % 8:
            raise NotImplementedError(f"SwiGLU hidden width {hidden} is not a multiple of 8 (16-B GEMM rows)")

    def forward(self, x):
        """fc1 / fc2 GEMMs side by side, vj_swiglu_fwd gate, fc3 (f32 out)."""
        shp = x.shape
        y = fn.run_sublayer(x.reshape(-1, shp[-1]), self)
        return y.reshape(*shp[:-1], y.shape[-1])


class DropPath(nn.Module):
    """modules.py:53-64: stochastic depth, timm's drop_path (timm 0.9.x, not in this image; restated):
    in training, a residual branch's output is multiplied per sample by Bernoulli(keep) / keep
    (keep = 1 - drop_prob), drawn as x.new_empty((B, 1, 1)).bernoulli_(keep).div_(keep) in the branch's
    dtype (bf16 under autocast). It runs fused in Block / ACBlock (functions.block_forward draws one
    factor per sequence and branch with sample(), the kernels scale the branch rows)."""

    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob

    def sample(self, n, device):
        """n per-sample factors (f32 holding the bf16 values the reference's random_tensor takes)."""
        keep = 1.0 - self.drop_prob
        rt = torch.empty(n, dtype=torch.bfloat16, device=device).bernoulli_(keep)
        if keep > 0.0:
            rt.div_(keep)
        return rt.float()

    def forward(self, x):
        if not self.drop_prob or not self.training:
            return x
        raise NotImplementedError("DropPath runs fused inside Block / ACBlock (functions.block_forward)")

    def extra_repr(self):
        return f"p={self.drop_prob}"


class RoPEAttention(nn.Module):
    """modules.py:261-382: fused QKV, 3-axis RoPE on the (frame, row, col) of each token id, SDPA."""

    use_rope = True

    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0.0, proj_drop=0.0, use_sdpa=True,
                 grid_size=14, is_causal=False):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = head_dim = dim // num_heads
        self.scale = qk_scale or head_dim**-0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop_prob = proj_drop
        self.proj_drop = nn.Dropout(proj_drop)
        self.use_sdpa = use_sdpa
        self.d_dim = self.h_dim = self.w_dim = int(2 * ((head_dim // 3) // 2))
        self.grid_size = grid_size
        self.is_causal = is_causal
        _check_attn(head_dim, attn_drop, proj_drop, is_causal)

    def forward(self, x, mask=None, attn_mask=None, T=None, H_patches=None, W_patches=None):
        """modules.py:326-382: QKV (+ 3-axis RoPE of q, k at the token positions: `mask` ids or
        0..N-1) -> SDPA -> proj, on the fused HIP kernels."""
        if attn_mask is not None:
            raise NotImplementedError("attn_mask is not supported on the HIP path")
        B, N, C = x.shape
        lay = token_layout(B, N, mask, self.grid_size, H_patches, W_patches, x.device)
        return fn.run_sublayer(x.reshape(B * N, C), self, lay).reshape(B, N, C)


class Attention(nn.Module):
    """modules.py:385-429 (no positional rotation)."""

    use_rope = False

    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0.0, proj_drop=0.0, use_sdpa=True,
                 is_causal=False):
        super().__init__()
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim**-0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop_prob = proj_drop
        self.proj_drop = nn.Dropout(proj_drop)
        self.use_sdpa = use_sdpa
        self.is_causal = is_causal
        _check_attn(head_dim, attn_drop, proj_drop, is_causal)

    def forward(self, x, mask=None, attn_mask=None):
        """modules.py:408-429: QKV -> SDPA -> proj on the HIP kernels (no positional rotation)."""
        if attn_mask is not None:
            raise NotImplementedError("attn_mask is not supported on the HIP path")
        B, N, C = x.shape
        lay = fn.TokenLayout([(B, N)], ids=None, ids_mod=N)
        return fn.run_sublayer(x.reshape(B * N, C), self, lay).reshape(B, N, C)


def _check_attn(head_dim, attn_drop, proj_drop, is_causal):
    """Dropout: proj_drop is also SDPA's dropout_p (modules.py:246 / 370 / 417, active in eval too, as
    there); attn_drop only acts without SDPA (use_sdpa=False, while training). Both run on the kernels'
    hash masks (vj_attn_fwd_ex, vj_dropout)."""
    if head_dim not in (32, 64, 80, 88):
        raise NotImplementedError(f"HIP attention supports head_dim 32, 64, 80, 88 (got {head_dim})")
    if not (0.0 <= attn_drop < 1.0 and 0.0 <= proj_drop < 1.0):
        raise ValueError(f"dropout probabilities must be in [0, 1) (attn_drop={attn_drop}, proj_drop={proj_drop})")
    if is_causal:
        raise NotImplementedError("causal attention is not on the V-JEPA pre-training path")


def _make_mlp(dim, hidden, act_layer, wide_silu, drop):
    """Block's MLP choice (modules.py:548-554): SwiGLUFFN for nn.SiLU, else the GELU MLP."""
    if act_layer is nn.SiLU:
        return SwiGLUFFN(in_features=dim, hidden_features=hidden, act_layer=act_layer, wide_silu=wide_silu, drop=drop)
    return MLP(in_features=dim, hidden_features=hidden, act_layer=act_layer, drop=drop)


class Block(nn.Module):
    """modules.py:500-563: x = x + drop_path(attn(norm1(x))); x = x + drop_path(mlp(norm2(x)))."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, qk_scale=None, drop=0.0, attn_drop=0.0,
                 drop_path=0.0, act_layer=nn.GELU, wide_silu=True, norm_layer=nn.LayerNorm, use_sdpa=True,
                 is_causal=False, grid_size=16, use_rope=False, **kwargs):
        super().__init__()
        self.norm1 = norm_layer(dim)
        if use_rope:
            self.attn = RoPEAttention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                      attn_drop=attn_drop, use_sdpa=use_sdpa, is_causal=is_causal,
                                      grid_size=grid_size, proj_drop=drop)
        else:
            self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                  attn_drop=attn_drop, use_sdpa=use_sdpa, is_causal=is_causal, proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = _make_mlp(dim, int(dim * mlp_ratio), act_layer, wide_silu, drop)

    def layout_for(self, B, N, mask, T, H_patches, W_patches, device):
        g = self.attn.grid_size if self.attn.use_rope else 1
        return token_layout(B, N, mask, g, H_patches, W_patches, device)

    def forward(self, x, mask=None, attn_mask=None, T=None, H_patches=None, W_patches=None):
        if attn_mask is not None:
            raise NotImplementedError("attn_mask is not supported on the HIP path")
        B, N, C = x.shape
        lay = self.layout_for(B, N, mask, T, H_patches, W_patches, x.device)
        y = fn.run_block(_residual_rows(x, self), self, lay)
        return y.reshape(B, N, C)


def _residual_rows(x, blk):
    """The block's residual stream in the input's dtype, as under the reference's autocast: a bf16 x
    stays bf16 (x + attn(norm1(x)) is a bf16 add, modules.py:561-562, and the block returns bf16), an
    f32 x stays f32. An active drop_path in training keeps f32 (not built on the bf16 stream)."""
    rows = x.reshape(-1, x.shape[-1]).contiguous()
    if rows.dtype == torch.bfloat16 and not (getattr(blk.drop_path, "drop_prob", 0.0) and blk.drop_path.training):
        return rows
    return rows.float()


def build_action_block_causal_attention_mask(T, H, W, add_tokens=1):
    """modules.py:12-23: [N, N] bool, token i attends to j iff frame(j) <= frame(i), frames of
    add_tokens + H*W tokens (local window = T: every earlier frame)."""
    n_t = add_tokens + H * W
    f = torch.arange(T * n_t) // n_t
    return f[None, :] <= f[:, None]


def ac_token_layout(B, T, H, W, cond, causal, device):
    """TokenLayout of the action-conditioned sequence [B, T*(cond + H*W)] (ACRoPEAttention.forward,
    modules.py:163-247): frame tokens keep their (frame, row, col) RoPE positions; each frame's cond
    (action / state / extrinsics) tokens get id frame*H*W, i.e. position (frame, 0, 0): the depth slice
    is rotated by the frame index and the row / column slices by angle 0 (= left unrotated, :190-193).
    causal: frame-causal attention over blocks of cond + H*W tokens (the attn_mask of
    build_action_block_causal_attention_mask)."""
    hw = H * W
    n_t = cond + hw
    t = torch.arange(T, device=device)[:, None]
    j = torch.arange(n_t, device=device)[None, :]
    ids = torch.where(j < cond, t * hw, t * hw + (j - cond))  # [T, n_t]
    ids = ids.reshape(1, -1).expand(B, -1).reshape(-1).to(torch.int32).contiguous()
    return fn.TokenLayout([(B, T * n_t)], ids=ids, ids_mod=T * hw, tpf=hw, tpr=W, fblk=n_t if causal else 0)


class ACRoPEAttention(RoPEAttention):
    """modules.py:109-258 (same parameters as RoPEAttention; action tokens handled by the layout)."""

    def forward(self, x, mask=None, attn_mask=None, T=None, H=None, W=None, action_tokens=0):
        if mask is not None:
            raise NotImplementedError("ACRoPEAttention with a token mask (the AC predictor passes None)")
        B, N, C = x.shape
        lay = _ac_layout_checked(B, N, attn_mask, T, H, W, action_tokens, self.grid_size, x.device)
        return fn.run_sublayer(x.reshape(B * N, C), self, lay).reshape(B, N, C)


def _ac_layout_checked(B, N, attn_mask, T, H, W, cond, grid_size, device):
    if H != W or grid_size != H:
        raise NotImplementedError("AC RoPE positions are snapped by grid_size / H, grid_size / W; only the "
                                  "identity snap (square grid, grid_size == H) is on the HIP path")
    n_t = cond + H * W
    if T is None or N != T * n_t:
        raise ValueError(f"AC sequence of {N} tokens is not T={T} frames of {n_t}")
    causal = False
    if attn_mask is not None:
        ref = build_action_block_causal_attention_mask(T, H, W, cond)[:N, :N]
        if not torch.equal(attn_mask.to(device="cpu", dtype=torch.bool), ref):
            raise NotImplementedError("only the frame-causal attn_mask of build_action_block_causal_attention_mask "
                                      "is supported on the HIP path")
        causal = True
    return ac_token_layout(B, T, H, W, cond, causal, device)


class ACBlock(nn.Module):
    """modules.py:432-497: the Block of the action-conditioned predictor (ACRoPEAttention or Attention)."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, qk_scale=None, drop=0.0, attn_drop=0.0,
                 drop_path=0.0, act_layer=nn.GELU, wide_silu=True, norm_layer=nn.LayerNorm, use_sdpa=True,
                 is_causal=False, grid_size=16, use_rope=False, **kwargs):
        super().__init__()
        self.norm1 = norm_layer(dim)
        if use_rope:
            self.attn = ACRoPEAttention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                        attn_drop=attn_drop, use_sdpa=use_sdpa, is_causal=is_causal,
                                        grid_size=grid_size, proj_drop=drop)
        else:
            self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                                  attn_drop=attn_drop, use_sdpa=use_sdpa, is_causal=is_causal, proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = _make_mlp(dim, int(dim * mlp_ratio), act_layer, wide_silu, drop)

    def forward(self, x, mask=None, attn_mask=None, T=None, H=None, W=None, action_tokens=0):
        if mask is not None:
            raise NotImplementedError("ACBlock with a token mask (the AC predictor passes None)")
        B, N, C = x.shape
        if isinstance(self.attn, ACRoPEAttention):
            lay = _ac_layout_checked(B, N, attn_mask, T, H, W, action_tokens, self.attn.grid_size, x.device)
        else:
            if attn_mask is not None:
                raise NotImplementedError("attn_mask without RoPE is not on the AC predictor path")
            lay = fn.TokenLayout([(B, N)], ids=None, ids_mod=N)
        return fn.run_block(_residual_rows(x, self), self, lay).reshape(B, N, C)


class CrossAttention(nn.Module):
    """modules.py:566-594: q / kv Linears and SDPA of the (few) queries over the tokens x; no output
    projection. q / kv projections on the HIP GEMMs (bf16 outputs), attention on vj_xattn."""

    def __init__(self, dim, num_heads=12, qkv_bias=False, use_sdpa=True):
        super().__init__()
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = head_dim**-0.5
        self.q = nn.Linear(dim, dim, bias=qkv_bias)
        self.kv = nn.Linear(dim, int(dim * 2), bias=qkv_bias)
        self.use_sdpa = use_sdpa
        if head_dim % 8 or head_dim > 128:
            raise NotImplementedError(f"HIP cross-attention supports head_dim % 8 == 0, <= 128 (got {head_dim})")

    def forward(self, q, x):
        """q [B, n, C], x [B, N, C] -> [B, n, C] (f32; SDPA's default scale = self.scale either branch)."""
        B, n, C = q.shape
        N = x.shape[1]
        H = self.num_heads
        qp = fn.run_linear(q.reshape(B * n, C), self.q, out_dtype=torch.bfloat16)
        kv = fn.run_linear(x.reshape(B * N, C), self.kv, out_dtype=torch.bfloat16)
        o = fn.cross_attention(qp, kv, B, n, N, H, C // H, self.scale)
        return o.float().reshape(B, n, C)


class CrossAttentionBlock(nn.Module):
    """modules.py:597-610: q + xattn(q, norm1(x)); then q + mlp(norm2(q)). norm1 normalises the
    TOKENS x (the keys / values), not the queries."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, act_layer=nn.GELU, norm_layer=nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.xattn = CrossAttention(dim, num_heads=num_heads, qkv_bias=qkv_bias)
        self.norm2 = norm_layer(dim)
        mlp_hidden_dim = int(dim * mlp_ratio)
        self.mlp = MLP(in_features=dim, hidden_features=mlp_hidden_dim, act_layer=act_layer)

    def forward(self, q, x):
        B, n, C = q.shape
        N = x.shape[1]
        xn = fn.run_layernorm(x.reshape(B * N, C).contiguous(), self.norm1, out_dtype=torch.bfloat16)
        q = q.float() + self.xattn(q, xn.reshape(B, N, C))
        y = fn.run_layernorm(q.reshape(B * n, C).contiguous(), self.norm2, out_dtype=torch.bfloat16)
        return q + fn.run_sublayer(y, self.mlp).reshape(B, n, C)


def token_layout(B, N, mask, grid_size, H_patches, W_patches, device):
    """RoPE token positions of a [B, N] batch (modules.py:293-341): ids from `mask` ([B, N] token ids)
    or 0..N-1, split into (frame, row, col) by H_patches / W_patches or the init-time grid size."""
    g = grid_size
    if H_patches is None or W_patches is None:
        tpf, tpr = g * g, g
    else:
        tpf, tpr = H_patches * W_patches, W_patches
    ids, nids = None, N
    if mask is not None:
        ids = ops.ids_to_int32([mask.to(device=device, dtype=torch.int64).contiguous()])
        nids = int(mask.max()) + 1  # bounds the RoPE positions (table rows)
    return fn.TokenLayout([(B, N)], ids=ids, ids_mod=nids, tpf=tpf, tpr=tpr)


def rescale_blocks(blocks):
    """vision_transformer.py:147-153 / predictor.py:158-164."""
    for layer_id, layer in enumerate(blocks):
        layer.attn.proj.weight.data.div_(math.sqrt(2.0 * (layer_id + 1)))
        layer.mlp.fc2.weight.data.div_(math.sqrt(2.0 * (layer_id + 1)))


def trunc_normal_(tensor, mean=0.0, std=1.0, a=-2.0, b=2.0):
    """src/utils/tensors.py:14-47 (same RNG consumption: uniform_ then erfinv_)."""

    def norm_cdf(x):
        return (1.0 + math.erf(x / math.sqrt(2.0))) / 2.0

    with torch.no_grad():
        lo = norm_cdf((a - mean) / std)
        hi = norm_cdf((b - mean) / std)
        tensor.uniform_(2 * lo - 1, 2 * hi - 1)
        tensor.erfinv_()
        tensor.mul_(std * math.sqrt(2.0))
        tensor.add_(mean)
        tensor.clamp_(min=a, max=b)
        return tensor
