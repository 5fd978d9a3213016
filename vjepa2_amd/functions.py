"""Fused forward/backward of the V-JEPA hot-path layers on the HIP kernels.

Token-major "ragged" execution: the tokens of every sequence of a pass (e.g. both JEPA mask passes
of a step) are concatenated into one [T, D] buffer; a TokenLayout says where the sequences are
(attention is the only op that needs it) and which token id each row is (RoPE positions).

The residual stream is f32, or bf16 where the reference's autocast keeps it in bf16 (the target
encoder, and the trained context encoder of a RoPE model under bf16 mixed precision: the Conv3d
output is bf16 and every x = x + branch(...) is a bf16 add; its gradient is then bf16 too); every
GEMM operand is bf16 with f32 accumulation. Parameter gradients are accumulated (+=) straight into
`param.grad` (f32, a view of the flat gradient arena when the trainer owns the parameters), so
autograd only carries activation gradients between layers.
"""

import os
import weakref

import torch

from . import ops
from .ops import BF16, EPI_BF16, EPI_BF16_RESID, EPI_F32, EPI_F32_RESID, EPI_GELU, F32

# ------------------------------------------------------------------------------------------------
# parameter views


def weight_bf16(p):
    """bf16 shadow of an f32 parameter: the arena-maintained copy when the trainer owns the
    parameter (refreshed by the fused AdamW / EMA kernels), else a cached cast keyed by version."""
    v = getattr(p, "_vj_bf16", None)
    if v is not None:
        return v
    key = (p.data_ptr(), p._version)
    c = getattr(p, "_vj_bf16_cache", None)
    if c is None or c[0] != key:
        c = (key, ops.cast_bf16(p.detach().contiguous()))
        p._vj_bf16_cache = c
    return c[1]


# Bumped whenever the arenas' bf16 shadows are rewritten (AdamW, EMA, sync): invalidates W^T copies.
SHADOW_EPOCH = [0]


def weight_bf16_t(p):
    """W^T [in, out] bf16 contiguous: the K-major B operand of the data-gradient GEMM dX = dY W
    (ops.linear_dgrad). Transposed by a HIP kernel once per weight update and cached; the copies of
    arena-owned weights are registered so refresh_weight_transposes() redoes them all in one launch
    right after the update."""
    src = weight_bf16(p)
    arena_owned = getattr(p, "_vj_bf16", None) is not None
    key = (src.data_ptr(), SHADOW_EPOCH[0] if arena_owned else p._version)
    c = getattr(p, "_vj_bf16_t", None)
    if c is None or c[0] != key:
        out = c[1] if c is not None and c[1].shape == (src.shape[1], src.shape[0]) else None
        c = (key, ops.transpose_bf16(src.reshape(src.shape[0], -1), out=out))
        p._vj_bf16_t = c
        if arena_owned:
            _WT_REG[id(p)] = p
    return c[1]


_WT_REG = weakref.WeakValueDictionary()  # id -> arena-owned parameter with a cached W^T copy
_WT_BATCH = [None]  # (the batch's (src, dst) pointer key, device descriptor table, tiles)


def refresh_weight_transposes():
    """Re-transpose every registered W^T copy whose bf16 shadow changed (after AdamW / a weight
    sync) with one vj_transpose_bf16_batch launch instead of one launch per weight in the backward."""
    stale = [p for p in _WT_REG.values() if p._vj_bf16_t[0][1] != SHADOW_EPOCH[0]]
    if not stale:
        return
    pairs = []
    for p in stale:
        src = weight_bf16(p)
        pairs.append((src.reshape(src.shape[0], -1), p._vj_bf16_t[1]))
    key = tuple((s.data_ptr(), d.data_ptr()) for s, d in pairs)
    if _WT_BATCH[0] is None or _WT_BATCH[0][0] != key:
        desc, tiles = ops.transpose_batch_desc(pairs)
        _WT_BATCH[0] = (key, desc, tiles)
    ops.transpose_bf16_batch(_WT_BATCH[0][1], len(pairs), _WT_BATCH[0][2])
    for p, (s, _) in zip(stale, pairs):
        p._vj_bf16_t = ((s.data_ptr(), SHADOW_EPOCH[0]), p._vj_bf16_t[1])


def weight_fp8(p):
    """Per-output-channel scaled e4m3 copy of a Linear weight [out, in] (the fp8 target encoder's B
    operands): (uint8 [out, in], int32 [out]), quantised from the fp32 master weight once per
    weight update and cached."""
    arena_owned = getattr(p, "_vj_bf16", None) is not None
    key = (p.data_ptr(), SHADOW_EPOCH[0] if arena_owned else p._version)
    c = getattr(p, "_vj_fp8", None)
    if c is None or c[0] != key:
        w = p.detach().reshape(p.shape[0], -1)
        if not w.is_contiguous():
            w = w.contiguous()
        out = c[1] if c is not None else (None, None)
        c = (key, ops.quant_rows_fp8(w, out=out[0], exps=out[1]))
        p._vj_fp8 = c
    return c[1]


def grad_buf(p):
    """p.grad for an accumulating (+=) write. Gradients in a lazily zeroed arena (FlatArena.zero_grad
    skips the weights the weight-gradient GEMMs overwrite) are zeroed here on their first touch of
    the step if that touch is not an overwrite."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    a = getattr(p, "_vj_arena", None)
    if a is not None and p._vj_gepoch != a.epoch:
        p.grad.zero_()
        p._vj_gepoch = a.epoch
    return p.grad


def wgrad_buf(p):
    """(p.grad, accumulate) for a weight-gradient GEMM: the first write of the step overwrites
    (EPI_F32: no zero fill of the gradient, no read of it in the epilogue), later writes add."""
    a = getattr(p, "_vj_arena", None)
    if a is None or p.grad is None:
        return grad_buf(p), True
    p._vj_ow = True
    if p._vj_gepoch != a.epoch:
        p._vj_gepoch = a.epoch
        return p.grad, False
    return p.grad, True


def wgrad(dy, x, w, shape=None, lin=None):
    """dW (+)= dY^T X into w's gradient (nn.Linear / Conv3d-as-GEMM weight gradient); with `lin` (the
    Linear owning w) its bias gradient dY.sum(0) too, summed inside the same GEMM."""
    buf, acc = wgrad_buf(w)
    db = _bias_buf(lin) if lin is not None else None
    ops.linear_wgrad(dy, x, buf if shape is None else buf.view(*shape), accumulate=acc, db=db)


_ROPE_TABLES = {}


def rope_tables(hd, device, npos):
    """cos/sin [npos, half] of the reference's per-axis angles (modules.py:30-39, fp32 op order)."""
    key = (hd, str(device), npos)
    t = _ROPE_TABLES.get(key)
    if t is None:
        sw = 2 * ((hd // 3) // 2)
        omega = torch.arange(sw // 2, dtype=torch.float32)
        omega /= sw / 2.0
        omega = 1.0 / 10000**omega
        freq = torch.arange(npos, dtype=torch.float32)[:, None] * omega[None, :]
        t = (freq.cos().contiguous().to(device), freq.sin().contiguous().to(device))
        if t[0].is_cuda:  # cached across streams (the target encoder runs on a side stream): make the
            torch.cuda.current_stream().synchronize()  # one-time H2D copy complete before any stream uses it
        _ROPE_TABLES[key] = t
    return t


class TokenLayout:
    """Ragged token batch: `groups` = [(nseq, seqlen), ...] in row order; RoPE ids per row
    (int32 device tensor) or None for `row % ids_mod`; tokens_per_frame / tokens_per_row."""

    def __init__(self, groups, ids=None, ids_mod=0, tpf=1, tpr=1, fblk=0):
        self.fblk = int(fblk)  # > 0: frame-causal attention over blocks of fblk tokens (AC predictor)
        self.groups = [(int(n), int(l)) for n, l in groups if n > 0]
        self.T = sum(n * l for n, l in self.groups)
        self.ids, self.ids_mod, self.tpf, self.tpr = ids, int(ids_mod), int(tpf), int(tpr)
        # positions per axis: frame < ceil(ids_mod / tpf), row < ceil(tpf / tpr), column < tpr
        self.npos = max(-(-self.ids_mod // self.tpf), -(-self.tpf // self.tpr), self.tpr, 1)


# ------------------------------------------------------------------------------------------------
# Transformer block (modules.py:500-563): x + attn(LN1 x); x + mlp(LN2 x)


def _attn_scale(attn, hd, lay=None):
    # F.scaled_dot_product_attention uses the default 1/sqrt(hd) (modules.py:367-372); the non-SDPA
    # branch uses attn.scale (= qk_scale or hd^-0.5). With the frame-causal attn_mask (lay.fblk > 0,
    # the AC predictor) ACRoPEAttention always takes the SDPA branch (modules.py:243-247), whatever
    # use_sdpa says, so the scale is SDPA's default there too.
    if attn.use_sdpa or (lay is not None and lay.fblk > 0):
        return hd**-0.5
    return attn.scale


def _resid_epi(x):
    # bf16 residual stream only on the no-grad target encoder (VisionTransformer.forward_features with
    # bf16_residual): the reference's own autocast precision, half the residual bytes
    return EPI_BF16_RESID if x.dtype == BF16 else EPI_F32_RESID


def block_forward_fp8(x, blk, lay):
    """Forward-only block with the QKV and fc1 GEMMs on the fp8 MFMA (opt-in for the no-grad target
    encoder, BASELINE configs[4]): LN1 / LN2 write per-row scaled e4m3, the weights are per-channel
    scaled e4m3; attention, proj and fc2 stay bf16 (their inputs come out of the attention / GELU
    kernels, whose rows span many tiles). f32 residual stream as in block_forward."""
    attn, mlp = blk.attn, blk.mlp
    if getattr(mlp, "swiglu", False) or _drop_scales(blk, lay, x.device) is not None or _has_dropout(blk):
        raise NotImplementedError("the fp8 block path covers the GELU MLP without drop_path / dropout")
    H = attn.num_heads
    hd = x.shape[1] // H
    ln1, e1 = ops.layernorm_fwd_fp8(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps)
    w8, ew = weight_fp8(attn.qkv.weight)
    if attn.use_rope:
        c, s = rope_tables(hd, x.device, lay.npos)
        qkv = ops.qkv_rope_fp8(ln1, e1, w8, ew, attn.qkv.bias, H, hd, lay.ids, lay.ids_mod, lay.tpf, lay.tpr, c, s)
    else:
        qkv = ops.linear_fwd_fp8(ln1, e1, w8, ew, attn.qkv.bias, EPI_BF16)
    o, _ = ops.attn_fwd(qkv, H, hd, lay.groups, _attn_scale(attn, hd, lay), fblk=lay.fblk)
    x_mid = ops.linear_fwd(o, weight_bf16(attn.proj.weight), attn.proj.bias, _resid_epi(x), resid=x)
    ln2, e2 = ops.layernorm_fwd_fp8(x_mid, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps)
    w18, ew1 = weight_fp8(mlp.fc1.weight)
    _, act = ops.linear_fwd_fp8(ln2, e2, w18, ew1, mlp.fc1.bias, EPI_GELU)
    return ops.linear_fwd(act, weight_bf16(mlp.fc2.weight), mlp.fc2.bias, _resid_epi(x), resid=x_mid)


def _drop_scales(blk, lay, device):
    """Stochastic depth (Block.forward, modules.py:561-562: timm drop_path(x, drop_prob, training)):
    per-row factors (attention branch, MLP branch) — each sequence's draw repeated over its tokens —
    or None when the block has no active DropPath. Draw order per block as in the reference: the
    attention branch's, then the MLP branch's."""
    dp = blk.drop_path
    if not getattr(dp, "drop_prob", None) or not dp.training:
        return None
    lens = getattr(lay, "_vj_seq_lens", None)  # built once per layout (one H2D copy, not one per block)
    if lens is None or lens.device != torch.device(device):
        lens = lay._vj_seq_lens = torch.tensor([ln for n, ln in lay.groups for _ in range(n)], device=device)
    # One draw per sequence for all packed mask groups at once (the reference's MultiSeqWrapper runs one
    # forward per mask and draws per mask): the same distribution, another RNG stream order, so a
    # multi-mask drop_path run is not replayable from the reference's seed (single-group fixtures are).
    return tuple(dp.sample(lens.numel(), device).repeat_interleave(lens, output_size=lay.T) for _ in range(2))


class DropCfg:
    """Dropout of one block call (modules.py): the attention probabilities' (SDPA dropout_p =
    proj_drop_prob, applied whether or not the module trains, :246 / 370 / 417; without SDPA, attn_drop
    while training, :252 / 376 / 423), the projection's proj_drop (:257 / 381) and the MLP's two
    nn.Dropout (after the activation and after fc2, :75-82) while training. Each active one gets its own
    seed for vj_common.h's mask hash, kept for the backward. SwiGLUFFN takes no dropout (its `drop` is
    unused in the reference too)."""

    def __init__(self, attn=None, mlp=None):
        self.pa, self.pp = _attn_drop_probs(attn) if attn is not None else (0.0, 0.0)
        self.pm = _mlp_drop_prob(mlp) if mlp is not None else 0.0
        self.sa, self.sp, self.sm1, self.sm2 = (_drop_seed() if p > 0 else 0 for p in (self.pa, self.pp, self.pm,
                                                                                        self.pm))

    @property
    def branches(self):  # proj / MLP dropout: the residual adds leave the GEMM epilogues
        return self.pp > 0 or self.pm > 0


def _attn_drop_probs(attn):
    """(attention-probability dropout, proj_drop) in effect for a call of `attn` (see DropCfg)."""
    if getattr(attn, "use_sdpa", True):
        pa = float(getattr(attn, "proj_drop_prob", 0.0) or 0.0)
    else:
        pa = float(attn.attn_drop.p) if attn.attn_drop.training else 0.0
    pp = float(attn.proj_drop.p) if attn.proj_drop.training else 0.0
    return pa, pp


def _mlp_drop_prob(mlp):
    drop = None if getattr(mlp, "swiglu", False) else getattr(mlp, "drop", None)
    return float(drop.p) if drop is not None and drop.training else 0.0


def _has_dropout(blk):
    return any(_attn_drop_probs(blk.attn)) or _mlp_drop_prob(blk.mlp) > 0


def _drop_seed():
    """A 32-bit mask seed from torch's default CPU generator, so torch.manual_seed replays a run. Only
    blocks with an active dropout draw (the shipped configs never do); the reference's dropout draws
    from the CUDA generator instead, so with dropout on, later CPU draws of this process (e.g. masks
    made in the main process) follow another sequence than the reference's."""
    return int(torch.randint(0, 2**32, (1,), dtype=torch.int64))


def _drop_cfg(blk):
    return DropCfg(blk.attn, blk.mlp) if _has_dropout(blk) else None


def _branch_out(inp, lin, resid, scale, p=0.0, seed=0):
    """resid + lin(inp): the residual add of a branch, fused into the output GEMM's epilogue; with a
    drop_path factor the GEMM writes the branch and vj_rowscale_add scales and adds it; with dropout
    (p > 0) vj_dropout drops the branch (then drop_path, if any) and adds it."""
    if scale is None and p == 0:
        return ops.linear_fwd(inp, weight_bf16(lin.weight), lin.bias, _resid_epi(resid), resid=resid)
    y = ops.linear_fwd(inp, weight_bf16(lin.weight), lin.bias, EPI_F32)
    if p == 0:
        return ops.rowscale_add(y, scale, resid)
    if scale is None:
        return ops.dropout(y, p, seed, resid=resid)
    return ops.rowscale_add(ops.dropout(y, p, seed).float(), scale, resid)


def _branch_grad(dxo, scale, p, seed):
    """bf16 gradient of a branch's output projection from the residual stream's gradient: drop_path's
    factor, then dropout's mask (the forward applied them in the other order)."""
    g = ops.rowscale_bf16(dxo, scale) if scale is not None else dxo
    if p > 0:
        return ops.dropout(g, p, seed)
    return g if g.dtype == BF16 else ops.cast_bf16(g)


def _mlp_forward(ln2, mlp, save, p=0.0, seed=0):
    """The MLP up to its output projection: (that projection's input, the output Linear, saved).
    GELU MLP (modules.py:77-83): fc1 + GELU in one GEMM epilogue, which also saves GELU'(pre-activation)
    for the backward (bf16, the bytes the pre-activation took), then the activation's dropout (p > 0).
    SwiGLUFFN (modules.py:102-106): fc1 and fc2 write x1 | x2 side by side, vj_swiglu_fwd makes
    silu(x1) * x2."""
    T = ln2.shape[0]
    if getattr(mlp, "swiglu", False):
        h = mlp.fc1.weight.shape[0]
        x12 = torch.empty(T, 2 * h, dtype=BF16, device=ln2.device)
        ops.linear_fwd(ln2, weight_bf16(mlp.fc1.weight), mlp.fc1.bias, EPI_BF16, out=x12[:, :h])
        ops.linear_fwd(ln2, weight_bf16(mlp.fc2.weight), mlp.fc2.bias, EPI_BF16, out=x12[:, h:])
        hidden = ops.swiglu_fwd(x12)
        return hidden, mlp.fc3, ((x12, hidden) if save else None)
    dgelu = torch.empty(T, mlp.fc1.weight.shape[0], dtype=BF16, device=ln2.device) if save else None
    _, act = ops.linear_fwd(ln2, weight_bf16(mlp.fc1.weight), mlp.fc1.bias, EPI_GELU, out=dgelu)
    if p > 0:
        act = ops.dropout(act, p, seed)
    return act, mlp.fc2, ((dgelu, act) if save else None)


def block_forward(x, blk, lay, save):
    """x f32, or bf16 (the residual stream in the reference's own autocast precision: the no-grad
    target encoder, and the trained context encoder of a RoPE model under bf16 mixed precision, where
    x = x + attn(norm1(x)) is a bf16 add, modules.py:561-562). The residual adds are fused into the
    proj / fc2 GEMM epilogues in x's dtype."""
    T, D = x.shape
    attn, mlp = blk.attn, blk.mlp
    H = attn.num_heads
    hd = D // H
    scales = _drop_scales(blk, lay, x.device)
    if save and scales is not None and x.dtype == BF16:
        raise NotImplementedError("drop_path on the trained bf16 residual stream (the trainer keeps f32 there)")
    dc = _drop_cfg(blk)
    pa, sa = (dc.pa, dc.sa) if dc is not None else (0.0, 0)
    ln1, m1, r1 = ops.layernorm_fwd(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, want_stats=save)
    if attn.use_rope:  # QKV GEMM with RoPE of q, k fused into its epilogue
        c, s = rope_tables(hd, x.device, lay.npos)
        qkv = ops.qkv_rope(ln1, weight_bf16(attn.qkv.weight), attn.qkv.bias, H, hd, lay.ids, lay.ids_mod, lay.tpf,
                           lay.tpr, c, s)
    else:
        qkv = ops.linear_fwd(ln1, weight_bf16(attn.qkv.weight), attn.qkv.bias, EPI_BF16)
    o, stats = ops.attn_fwd(qkv, H, hd, lay.groups, _attn_scale(attn, hd, lay), fblk=lay.fblk, dropout_p=pa, seed=sa)
    x_mid = _branch_out(o, attn.proj, x, scales and scales[0], *((dc.pp, dc.sp) if dc else ()))
    ln2, m2, r2 = ops.layernorm_fwd(x_mid, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps, want_stats=save)
    hidden, out_lin, msaved = _mlp_forward(ln2, mlp, save, *((dc.pm, dc.sm1) if dc else ()))
    x_out = _branch_out(hidden, out_lin, x_mid, scales and scales[1], *((dc.pm, dc.sm2) if dc else ()))
    saved = (x, ln1, m1, r1, qkv, o, stats, x_mid, ln2, m2, r2, msaved, scales, dc) if save else None
    return x_out, saved


def block_forward_f32(x, blk, lay):
    """fp32-operand parity mode of block_forward: the same LayerNorm / RoPE kernels, f32 MFMA GEMMs
    (vj_gemm_f32) and exact-softmax attention (vj_attn_fwd_f32); every intermediate stays f32."""
    if lay.fblk:
        raise NotImplementedError("the fp32-operand parity mode has no frame-causal attention")
    if getattr(blk.mlp, "swiglu", False) or _drop_scales(blk, lay, x.device) is not None or _has_dropout(blk):
        raise NotImplementedError("the fp32-operand parity mode covers the GELU MLP without drop_path / dropout")
    attn, mlp = blk.attn, blk.mlp
    H = attn.num_heads
    hd = x.shape[1] // H
    ln1, _, _ = ops.layernorm_fwd(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, out_dtype=F32, want_stats=False)
    qkv = ops.linear_fwd_f32(ln1, attn.qkv.weight.detach().float(), attn.qkv.bias, EPI_F32)
    if attn.use_rope:
        c, s = rope_tables(hd, x.device, lay.npos)
        ops.rope_f32_(qkv, H, hd, lay.ids, lay.ids_mod, lay.tpf, lay.tpr, c, s)
    o, _ = ops.attn_fwd_f32(qkv, H, hd, lay.groups, _attn_scale(attn, hd))
    x_mid = ops.linear_fwd_f32(o, attn.proj.weight.detach().float(), attn.proj.bias, EPI_F32_RESID, resid=x)
    ln2, _, _ = ops.layernorm_fwd(x_mid, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps, out_dtype=F32,
                                  want_stats=False)
    _, act = ops.linear_fwd_f32(ln2, mlp.fc1.weight.detach().float(), mlp.fc1.bias, EPI_GELU)
    return ops.linear_fwd_f32(act, mlp.fc2.weight.detach().float(), mlp.fc2.bias, EPI_F32_RESID, resid=x_mid)


def patch_embed_forward_f32(clip, pe, masks, pos_table=None, pos_ids=None, pos_mod=0):
    """fp32-operand parity mode of patch_embed_forward."""
    proj = pe.proj
    D = proj.weight.shape[0]
    p, tub = pe.patch_size, pe.tubelet_size
    cols = ops.im2col_f32(clip, p, tub) if masks is None else torch.cat(
        [ops.im2col_f32(clip, p, tub, idx=m.contiguous()) for m in masks], 0)
    x = ops.linear_fwd_f32(cols, proj.weight.detach().float().reshape(D, -1).contiguous(), proj.bias, EPI_F32)
    if pos_table is not None:
        ops.add_rows(x, pos_table, idx=pos_ids, idx_mod=pos_mod)
    return x


# ------------------------------------------------------------------------------------------------
# Weight-gradient stream. In a block's backward the weight-gradient GEMMs (with their split-K
# reduction) and the fc1 / qkv bias column sums feed nothing but the gradient arena, while the data
# gradients form the critical path (dgrad -> LayerNorm backward -> dgrad -> attention backward -> ...).
# With VJ_WGRAD_STREAM=1 they are issued on a second HIP stream (after everything the current stream
# has issued so far, their operands' memory held for it with record_stream), so they fill the CUs the
# critical path leaves idle. Whoever reads the gradients after the backward waits for that stream:
# the first use queues an autograd end-of-backward callback that makes the current stream wait, and
# the gradient all-reduce issues its buckets from the wgrad stream (distributed.GradReducer).
# On by default: +2.0 % clips/s (207.2 / 206.8 -> 211.5 / 210.6, bench.py A/B in one call,
# profiles/r04_wgrad_stream_step_ab.txt); VJ_WGRAD_STREAM=0 keeps everything on one stream.

_WG_STREAMS = {}


def wgrad_stream():
    """The per-device weight-gradient stream, or None when disabled (VJ_WGRAD_STREAM=0)."""
    if os.environ.get("VJ_WGRAD_STREAM", "1") != "1" or not torch.cuda.is_available():
        return None
    dev = torch.cuda.current_device()
    s = _WG_STREAMS.get(dev)
    if s is None:
        s = _WG_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return s


def join_wgrad_stream():
    """Make the current stream wait for every weight-gradient launch issued so far."""
    s = _WG_STREAMS.get(torch.cuda.current_device()) if torch.cuda.is_available() else None
    if s is not None:
        torch.cuda.current_stream().wait_stream(s)


_WG_JOIN_TASK = [None]  # autograd graph task whose end-of-backward join is queued


class JoinQueue(list):
    """Work to issue on the weight-gradient stream right after its next join with the current stream
    (distributed.GradReducer: a bucket's all-reduce also needs the LayerNorm / bias gradients written on
    the current stream; riding on the join every block's weight gradients take anyway saves a join of
    its own per bucket). One queue per owner, so two armed reducers in one process (a trainer and an
    eval probe, two frames-per-clip groups) never issue each other's collectives; at a join the queues
    are drained in the order their owners were created, which is the same host program order on every
    rank, whatever the interleaving of the owners' backward hooks."""


_JOIN_QUEUES = []  # weakrefs to the live JoinQueues, creation order


def join_queue():
    q = JoinQueue()
    _JOIN_QUEUES.append(weakref.ref(q))
    return q


def _drain_join_queues():
    """Issue every queued item (called on the weight-gradient stream, right after a join)."""
    live = []
    for r in _JOIN_QUEUES:
        q = r()
        if q is None:
            continue
        live.append(r)
        while q:
            q.pop(0)()
    _JOIN_QUEUES[:] = live


def drain_join_queue(q):
    """Issue q's items now: after one join of the weight-gradient stream with the current stream, on
    it; directly when that stream is off (VJ_WGRAD_STREAM=0 set since the items were queued)."""
    if not q:
        return
    side = wgrad_stream()
    if side is None:
        while q:
            q.pop(0)()
        return
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        while q:
            q.pop(0)()


def _join_at_backward_end():
    _WG_JOIN_TASK[0] = None
    join_wgrad_stream()


class _OnWgradStream:
    """`with _OnWgradStream(*tensors):` the enclosed launches go to the weight-gradient stream (when
    enabled), ordered after everything issued so far on the current stream."""

    def __init__(self, *tensors):
        self.tensors = tensors
        self.side = wgrad_stream()
        self.ctx = None

    def __enter__(self):
        if self.side is None:
            return self
        self.side.wait_stream(torch.cuda.current_stream())
        for t in self.tensors:
            t.record_stream(self.side)
        task = torch._C._current_graph_task_id()
        self.join_on_exit = task == -1  # called outside an autograd backward: join right away
        if task != -1 and _WG_JOIN_TASK[0] != task:
            # inside an autograd backward: join once, when the whole pass ends
            torch.autograd.Variable._execution_engine.queue_callback(_join_at_backward_end)
            _WG_JOIN_TASK[0] = task
        self.ctx = torch.cuda.stream(self.side)
        self.ctx.__enter__()
        _drain_join_queues()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
            if self.join_on_exit:
                join_wgrad_stream()
        return False


def _bias_buf(lin):
    return grad_buf(lin.bias) if lin.bias is not None and lin.bias.requires_grad else None


def _bias_grad(lin, dy):
    if lin.bias is not None and lin.bias.requires_grad:
        ops.colsum(dy, grad_buf(lin.bias))


def _ln_grads(ln):
    if ln.weight is None:
        return None, None
    return grad_buf(ln.weight), grad_buf(ln.bias)


def _mlp_backward(dy_b, mlp, ln2, saved, p=0.0, seed=0):
    """bf16 gradient of the MLP output -> bf16 gradient of its input ln2; weight and hidden-bias
    gradients accumulated (the output Linear's bias gradient is the caller's). Each weight gradient is
    issued before the data gradient that shares its dY, so on the weight-gradient stream the two overlap.
    SwiGLU: d(ln2) = dx1 W1 + dx2 W2, the second dgrad GEMM adding the first's output in its epilogue
    (autograd sums the two Linears' input gradients)."""
    if getattr(mlp, "swiglu", False):
        x12, hidden = saved
        h = hidden.shape[1]
        with _OnWgradStream(dy_b, hidden):
            wgrad(dy_b, hidden, mlp.fc3.weight)
        dh = ops.linear_dgrad(dy_b, weight_bf16(mlp.fc3.weight), wt=weight_bf16_t(mlp.fc3.weight))
        dx12 = ops.swiglu_bwd(dh, x12)
        dx1, dx2 = dx12[:, :h], dx12[:, h:]
        with _OnWgradStream(dx12, ln2):
            wgrad(dx1, ln2, mlp.fc1.weight, lin=mlp.fc1)
            wgrad(dx2, ln2, mlp.fc2.weight, lin=mlp.fc2)
        dl = ops.linear_dgrad(dx1, weight_bf16(mlp.fc1.weight), wt=weight_bf16_t(mlp.fc1.weight))
        return ops.linear_dgrad(dx2, weight_bf16(mlp.fc2.weight), wt=weight_bf16_t(mlp.fc2.weight), resid=dl)
    dgelu, act = saved
    with _OnWgradStream(dy_b, act):
        wgrad(dy_b, act, mlp.fc2.weight)
    if p > 0:  # the activation's dropout between the fc2 data gradient and GELU's backward
        dh = ops.linear_dgrad(dy_b, weight_bf16(mlp.fc2.weight), wt=weight_bf16_t(mlp.fc2.weight))
        dpre = ops.dropout(dh, p, seed, aux=dgelu)
    else:
        dpre = ops.linear_dgrad(dy_b, weight_bf16(mlp.fc2.weight), gelu_grad=dgelu, wt=weight_bf16_t(mlp.fc2.weight))
    with _OnWgradStream(dpre, ln2):
        wgrad(dpre, ln2, mlp.fc1.weight, lin=mlp.fc1)
    return ops.linear_dgrad(dpre, weight_bf16(mlp.fc1.weight), wt=weight_bf16_t(mlp.fc1.weight))


def block_backward(dxo, blk, lay, saved):
    x, ln1, m1, r1, qkv, o, stats, x_mid, ln2, m2, r2, msaved, scales, dc = saved
    branch_drop = dc is not None and dc.branches
    attn, mlp = blk.attn, blk.mlp
    out_lin = mlp.fc3 if getattr(mlp, "swiglu", False) else mlp.fc2
    T, D = x.shape
    H = attn.num_heads
    hd = D // H
    if branch_drop:  # dropout (and drop_path) of the MLP branch: the bias gradient from its dY, not from dxo
        dy_mlp = _branch_grad(dxo, scales and scales[1], dc.pm, dc.sm2)
        _bias_grad(out_lin, dy_mlp)
    elif dxo.dtype == BF16:  # bf16 residual stream: its gradient is bf16 too (as under the reference's autocast)
        dy_mlp = dxo
    elif scales is None:
        twin = getattr(dxo, "_vj_grad_bf16", None)  # bf16 twin written by the next block's LN1 backward,
        dy_mlp = twin[0] if twin is not None and twin[1] == dxo._version else ops.cast_bf16(dxo)  # unless changed
    else:  # drop_path: the MLP branch's dY = its factor x dxo (bias gradient from it, not from dxo)
        dy_mlp = ops.rowscale_bf16(dxo, scales[1])
        _bias_grad(out_lin, dy_mlp)
    dln2 = _mlp_backward(dy_mlp, mlp, ln2, msaved, *((dc.pm, dc.sm1) if dc else ()))
    gw, gb = _ln_grads(blk.norm2)
    # without drop_path / dropout the output-projection / proj bias gradients are the column sums of
    # dxo / dxm, fused into the LayerNorm backward
    fused = scales is None and not branch_drop
    dxm, dxm_b = ops.layernorm_bwd(dln2, x_mid, m2, r2, blk.norm2.weight, dres_in=dxo, dweight=gw, dbias=gb,
                                   want_bf16=fused, sum_in=_bias_buf(out_lin) if fused else None,
                                   sum_out=_bias_buf(attn.proj) if fused else None)
    if not fused:
        dxm_b = _branch_grad(dxm, scales and scales[0], dc.pp if dc else 0.0, dc.sp if dc else 0)
        _bias_grad(attn.proj, dxm_b)
    # attention
    with _OnWgradStream(dxm_b, o):
        wgrad(dxm_b, o, attn.proj.weight)
    do = ops.linear_dgrad(dxm_b, weight_bf16(attn.proj.weight), wt=weight_bf16_t(attn.proj.weight))
    rope = None
    if attn.use_rope:  # inverse RoPE fused into the dq / dk stores of the attention backward
        c, s = rope_tables(hd, x.device, lay.npos)
        rope = (lay.ids, lay.ids_mod, lay.tpf, lay.tpr, c, s)
    dqkv = ops.attn_bwd(qkv, o, do, stats, H, hd, lay.groups, _attn_scale(attn, hd, lay), rope=rope, fblk=lay.fblk,
                        dropout_p=dc.pa if dc else 0.0, seed=dc.sa if dc else 0)
    with _OnWgradStream(dqkv, ln1):
        wgrad(dqkv, ln1, attn.qkv.weight, lin=attn.qkv)
    dln1 = ops.linear_dgrad(dqkv, weight_bf16(attn.qkv.weight), wt=weight_bf16_t(attn.qkv.weight))
    gw, gb = _ln_grads(blk.norm1)
    dxi, dxi_b = ops.layernorm_bwd(dln1, x, m1, r1, blk.norm1.weight, dres_in=dxm, dweight=gw, dbias=gb,
                                   want_bf16=True)
    if dxi.dtype == F32:
        dxi._vj_grad_bf16 = (dxi_b, dxi._version)  # the previous block's fc2 dgrad / wgrad operand (saves a cast)
    return dxi


def _fire_hook(mod):
    hook = getattr(mod, "_vj_grad_ready", None)
    if hook is not None:
        hook(mod)


class _BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, blk, lay):
        y, saved = block_forward(x, blk, lay, save=True)
        ctx.blk, ctx.lay, ctx.saved = blk, lay, saved
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = block_backward(dy.contiguous(), ctx.blk, ctx.lay, ctx.saved)
        ctx.saved = None
        _fire_hook(ctx.blk)
        return dx, None, None, None


def _needs_grad(x, mod):
    return torch.is_grad_enabled() and (
        (x is not None and x.requires_grad) or any(p.requires_grad for p in mod.parameters()))


def run_block(x, blk, lay, fp8=False):
    if _needs_grad(x, blk):
        if fp8:
            raise NotImplementedError("the fp8 block path is forward-only (the no-grad target encoder)")
        return _BlockFn.apply(x, blk.norm1.weight, blk, lay)
    if fp8:
        return block_forward_fp8(x, blk, lay)
    return block_forward(x, blk, lay, save=False)[0]


# ------------------------------------------------------------------------------------------------
# Standalone RoPEAttention / Attention (modules.py:326-382, 408-429) and MLP (modules.py:77-83)
# forward()s on the same kernels as the fused block: bf16 operands, f32 outputs.


def attn_module_forward(x, attn, lay):
    """x bf16 [T, C] -> (proj(attention(x)) f32 [T, C], saved for backward)."""
    H = attn.num_heads
    hd = x.shape[1] // H
    if attn.use_rope:
        c, s = rope_tables(hd, x.device, lay.npos)
        qkv = ops.qkv_rope(x, weight_bf16(attn.qkv.weight), attn.qkv.bias, H, hd, lay.ids, lay.ids_mod, lay.tpf,
                           lay.tpr, c, s)
    else:
        qkv = ops.linear_fwd(x, weight_bf16(attn.qkv.weight), attn.qkv.bias, EPI_BF16)
    dc = DropCfg(attn=attn) if any(_attn_drop_probs(attn)) else None
    o, stats = ops.attn_fwd(qkv, H, hd, lay.groups, _attn_scale(attn, hd, lay), fblk=lay.fblk,
                            dropout_p=dc.pa if dc else 0.0, seed=dc.sa if dc else 0)
    y = ops.linear_fwd(o, weight_bf16(attn.proj.weight), attn.proj.bias, EPI_F32)
    if dc is not None and dc.pp > 0:  # proj_drop (modules.py:257 / 381): the module's output in bf16
        y = ops.dropout(y, dc.pp, dc.sp).float()
    return y, (x, qkv, o, stats, dc)


def attn_module_backward(dy, attn, lay, saved):
    x, qkv, o, stats, dc = saved
    H = attn.num_heads
    hd = x.shape[1] // H
    if dc is not None and dc.pp > 0:
        dy = ops.dropout(dy, dc.pp, dc.sp).float()
    dy_b = ops.cast_bf16(dy)
    do = ops.linear_dgrad(dy_b, weight_bf16(attn.proj.weight), wt=weight_bf16_t(attn.proj.weight))
    wgrad(dy_b, o, attn.proj.weight)
    _bias_grad(attn.proj, dy)
    rope = None
    if attn.use_rope:
        c, s = rope_tables(hd, x.device, lay.npos)
        rope = (lay.ids, lay.ids_mod, lay.tpf, lay.tpr, c, s)
    dqkv = ops.attn_bwd(qkv, o, do, stats, H, hd, lay.groups, _attn_scale(attn, hd, lay), rope=rope, fblk=lay.fblk,
                        dropout_p=dc.pa if dc else 0.0, seed=dc.sa if dc else 0)
    dx = ops.linear_dgrad(dqkv, weight_bf16(attn.qkv.weight), wt=weight_bf16_t(attn.qkv.weight))
    wgrad(dqkv, x, attn.qkv.weight, lin=attn.qkv)
    return dx


def mlp_module_forward(x, mlp):
    """x bf16 [T, C] -> (fc2(GELU(fc1 x)) or SwiGLU's fc3(silu(fc1 x) * fc2 x), f32; saved)."""
    dc = DropCfg(mlp=mlp) if _mlp_drop_prob(mlp) > 0 else None
    hidden, out_lin, msaved = _mlp_forward(x, mlp, True, *((dc.pm, dc.sm1) if dc else ()))
    y = ops.linear_fwd(hidden, weight_bf16(out_lin.weight), out_lin.bias, EPI_F32)
    if dc is not None:  # the output dropout (modules.py:82)
        y = ops.dropout(y, dc.pm, dc.sm2).float()
    return y, (x, msaved, dc)


def mlp_module_backward(dy, mlp, saved):
    x, msaved, dc = saved
    if dc is not None:
        dy = ops.dropout(dy, dc.pm, dc.sm2).float()
    dx = _mlp_backward(ops.cast_bf16(dy), mlp, x, msaved, *((dc.pm, dc.sm1) if dc else ()))
    _bias_grad(mlp.fc3 if getattr(mlp, "swiglu", False) else mlp.fc2, dy)
    return dx


class _SubLayerFn(torch.autograd.Function):
    """Autograd node of a standalone attention or MLP module (parameter grads go straight into
    param.grad, as for the fused block)."""

    @staticmethod
    def forward(ctx, x, anchor, mod, lay):
        xb = ops.cast_bf16(x.contiguous()) if x.dtype != BF16 else x.contiguous()
        if lay is None:
            y, saved = mlp_module_forward(xb, mod)
        else:
            y, saved = attn_module_forward(xb, mod, lay)
        ctx.mod, ctx.lay, ctx.saved, ctx.in_dtype = mod, lay, saved, x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous().float()
        if ctx.lay is None:
            dx = mlp_module_backward(dy, ctx.mod, ctx.saved)
        else:
            dx = attn_module_backward(dy, ctx.mod, ctx.lay, ctx.saved)
        ctx.saved = None
        _fire_hook(ctx.mod)
        return dx.to(ctx.in_dtype), None, None, None


def run_sublayer(x, mod, lay=None):
    """x [T, C] (f32 or bf16) through an attention module (lay = its TokenLayout) or an MLP (lay None)."""
    if _needs_grad(x, mod):
        return _SubLayerFn.apply(x, next(mod.parameters()), mod, lay)
    xb = ops.cast_bf16(x.contiguous()) if x.dtype != BF16 else x.contiguous()
    return (mlp_module_forward(xb, mod) if lay is None else attn_module_forward(xb, mod, lay))[0]


# ------------------------------------------------------------------------------------------------
# Patch embedding: Conv3d(k=s=(tub,p,p)) over the kept tubelets only (patch_embed.py:42-52 +
# apply_masks vision_transformer.py:188-192), optional sincos pos-embed add (:183-186).


def patch_embed_forward(clip, pe, masks, pos_table=None, pos_ids=None, pos_mod=0, save=False, out_bf16=False):
    """out_bf16: the tokens in bf16 (the Conv3d's autocast output dtype, patch_embed.py:42-52), for a
    bf16 residual stream; only without a pos-embed add (RoPE models: bf16 + an f32 table would promote
    to f32 in the reference)."""
    proj = pe.proj
    D = proj.weight.shape[0]
    kdim = proj.weight[0].numel()
    p, tub = pe.patch_size, pe.tubelet_size
    if masks is None:
        cols = ops.im2col(clip, p, tub)
    else:
        B = clip.shape[0]
        R = sum(B * m.shape[1] for m in masks)
        cols = torch.empty(R, kdim, dtype=BF16, device=clip.device)
        r0 = 0
        for m in masks:
            n = B * m.shape[1]
            ops.im2col(clip, p, tub, idx=m.contiguous(), out=cols[r0:r0 + n])
            r0 += n
    assert not (out_bf16 and pos_table is not None), "bf16 tokens: no pos-embed add (RoPE models)"
    x = ops.linear_fwd(cols, weight_bf16(proj.weight).view(D, kdim), proj.bias, EPI_BF16 if out_bf16 else EPI_F32)
    if pos_table is not None:
        ops.add_rows(x, pos_table, idx=pos_ids, idx_mod=pos_mod)
    return x, (cols if save else None)


class _PatchEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, clip, anchor, pe, masks, pos_table, pos_ids, pos_mod, out_bf16):
        x, cols = patch_embed_forward(clip, pe, masks, pos_table, pos_ids, pos_mod, save=True, out_bf16=out_bf16)
        ctx.pe, ctx.cols = pe, cols
        return x

    @staticmethod
    def backward(ctx, dx):
        proj = ctx.pe.proj
        D = proj.weight.shape[0]
        dx = dx.contiguous()
        wgrad(dx if dx.dtype == BF16 else ops.cast_bf16(dx), ctx.cols, proj.weight, (D, -1))
        _bias_grad(proj, dx)
        ctx.cols = None
        _fire_hook(ctx.pe)
        return None, None, None, None, None, None, None, None


def run_patch_embed(clip, pe, masks, pos_table=None, pos_ids=None, pos_mod=0, out_bf16=False):
    if _needs_grad(None, pe):
        return _PatchEmbedFn.apply(clip, pe.proj.weight, pe, masks, pos_table, pos_ids, pos_mod, out_bf16)
    return patch_embed_forward(clip, pe, masks, pos_table, pos_ids, pos_mod, out_bf16=out_bf16)[0]


# ------------------------------------------------------------------------------------------------
# LayerNorm (affine) as its own op (encoder / predictor final norms)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, ln, out_dtype):
        y, m, r = ops.layernorm_fwd(x, ln.weight, ln.bias, ln.eps, out_dtype=out_dtype)
        ctx.ln, ctx.x, ctx.m, ctx.r = ln, x, m, r
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dy_b = dy if dy.dtype == BF16 else ops.cast_bf16(dy)
        gw, gb = _ln_grads(ctx.ln)
        dx, _ = ops.layernorm_bwd(dy_b, ctx.x, ctx.m, ctx.r, ctx.ln.weight, dweight=gw, dbias=gb)
        ctx.x = ctx.m = ctx.r = None
        _fire_hook(ctx.ln)
        return dx, None, None, None


def run_layernorm(x, ln, out_dtype=F32):
    if _needs_grad(x, ln):
        return _LayerNormFn.apply(x, ln.weight, ln, out_dtype)
    return ops.layernorm_fwd(x, ln.weight, ln.bias, ln.eps, out_dtype=out_dtype, want_stats=False)[0]


# ------------------------------------------------------------------------------------------------
# Linear (predictor_embed / predictor_proj, predictor.py:182, 244)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, lin, out_dtype):
        xb = x.contiguous() if x.dtype == BF16 else ops.cast_bf16(x.contiguous())
        y = ops.linear_fwd(xb, weight_bf16(lin.weight), lin.bias, EPI_BF16 if out_dtype == BF16 else EPI_F32)
        ctx.lin, ctx.x, ctx.in_dtype = lin, xb, x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dy_b = dy if dy.dtype == BF16 else ops.cast_bf16(dy)
        lin = ctx.lin
        w = lin.weight
        wt = weight_bf16_t(w) if w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0 else None  # else padded in linear_dgrad
        dx = ops.linear_dgrad(dy_b, weight_bf16(lin.weight), wt=wt)
        wgrad(dy_b, ctx.x, lin.weight)
        _bias_grad(lin, dy)
        ctx.x = None
        _fire_hook(lin)
        return dx.to(ctx.in_dtype), None, None, None


def run_linear(x, lin, out_dtype=F32):
    """x [M, K] (bf16, or f32: cast on the device; the gradient comes back in x's dtype) -> y [M, N]."""
    if _needs_grad(x, lin):
        return _LinearFn.apply(x, lin.weight, lin, out_dtype)
    if x.dtype != BF16:
        x = ops.cast_bf16(x.contiguous())
    return ops.linear_fwd(x, weight_bf16(lin.weight), lin.bias, EPI_BF16 if out_dtype == BF16 else EPI_F32)


# ------------------------------------------------------------------------------------------------
# Predictor token assembly (predictor.py:192-217): context rows scattered to their sorted slots,
# mask token broadcast into the target slots, optional sincos pos-embed of every slot.


class _AssembleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, e, token, ctx_dst, tgt_rows, S, pos_table, pos_ids, owner):
        Dp = e.shape[1]
        seq = torch.empty(S, Dp, dtype=F32, device=e.device)
        ops.scatter_rows(e, ctx_dst, seq)
        ops.fill_rows(seq, tgt_rows, token.detach().reshape(-1).contiguous())
        if pos_table is not None:
            ops.add_rows(seq, pos_table, idx=pos_ids)
        ctx.ctx_dst, ctx.tgt_rows, ctx.token, ctx.owner = ctx_dst, tgt_rows, token, owner
        return seq

    @staticmethod
    def backward(ctx, dseq):
        dseq = dseq.contiguous()
        de = ops.gather_rows(dseq, ctx.ctx_dst)
        if ctx.token.requires_grad:
            rows = ops.gather_rows(dseq, ctx.tgt_rows)
            ops.colsum(rows, grad_buf(ctx.token).view(-1))
        _fire_hook(ctx.owner)
        return de, None, None, None, None, None, None, None


class _GatherRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx):
        ctx.S, ctx.idx = x.shape[0], idx
        return ops.gather_rows(x, idx)

    @staticmethod
    def backward(ctx, dy):
        dx = torch.zeros(ctx.S, dy.shape[1], dtype=dy.dtype, device=dy.device)
        ops.scatter_rows(dy.contiguous(), ctx.idx, dx)
        return dx, None


def gather_rows(x, idx):
    if torch.is_grad_enabled() and x.requires_grad:
        return _GatherRowsFn.apply(x, idx)
    return ops.gather_rows(x, idx)


# ------------------------------------------------------------------------------------------------
# Cross-attention of learned queries over encoder tokens (modules.py:577-594 SDPA part)


class _XAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, kv, B, nq, N, H, hd, scale):
        o, lse2 = ops.xattn_fwd(q, kv, B, nq, N, H, hd, scale)
        ctx.save_for_backward(q, kv, o, lse2)
        ctx.dims = (B, nq, N, H, hd, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, kv, o, lse2 = ctx.saved_tensors
        do = do.contiguous()
        do_b = do if do.dtype == BF16 else ops.cast_bf16(do.float())
        dq, dkv = ops.xattn_bwd(q, kv, o, do_b, lse2, *ctx.dims)
        return dq, dkv, None, None, None, None, None, None


def cross_attention(q, kv, B, nq, N, H, hd, scale):
    """q bf16 [B*nq, H*hd], kv bf16 [B*N, 2*H*hd] -> O bf16 [B*nq, H*hd] (SDPA, non-causal)."""
    if torch.is_grad_enabled() and (q.requires_grad or kv.requires_grad):
        return _XAttnFn.apply(q, kv, B, nq, N, H, hd, scale)
    return ops.xattn_fwd(q, kv, B, nq, N, H, hd, scale)[0]
