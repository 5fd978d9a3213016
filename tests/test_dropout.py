"""Dropout (nn.Dropout in MLP / the attention projection, SDPA's attention dropout_p; modules.py:75-82,
246, 257, 370, 381, 417): the kernels' counter-based keep masks restated in numpy
(vj_dropout_mask_ref), checked bit-exactly against vj_dropout and through fp32 references that use the
same masks for the attention kernels and the Block.

The reference draws its masks from torch's Philox stream, which no restatement can replay; what is
pinned here is the op each mask feeds (scaling, rounding points, forward/backward consistency, the
attention dropout's place between softmax and PV) and the mask's statistics. Parity unpinned for
the individual mask bits.
"""

import numpy as np
import pytest
import torch

M32 = 0xFFFFFFFF


def _mix(x):
    x = x.astype(np.uint64)
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def drop_thresh(p):
    t = p * 4294967296.0
    return 0 if t <= 0 else (M32 if t >= M32 else int(t + 0.5))


def vj_dropout_mask_ref(seed, rows, cols, p):
    """keep[r, c] of vj_common.h: drop_u(drop_row(seed, r), c) >= round(p * 2^32), uint32 arithmetic.
    rows / cols: 1-D integer arrays (the row / column ids)."""
    r = np.asarray(rows, dtype=np.uint64)[:, None]
    c = np.asarray(cols, dtype=np.uint64)[None, :]
    rk = _mix(np.uint64(seed) ^ ((r * 0x9E3779B1) & M32))
    u = _mix((rk + c * 0x85EBCA77) & M32)
    return u >= drop_thresh(p)


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_mask_statistics(p):
    """Keep fraction within 5 sigma of 1 - p; rows and seeds give different masks."""
    keep = vj_dropout_mask_ref(1234, np.arange(512), np.arange(1024), p)
    n = keep.size
    frac = keep.mean()
    assert abs(frac - (1 - p)) < 5 * np.sqrt(p * (1 - p) / n), frac
    assert (keep[0] != keep[1]).mean() > 0.5 * 2 * p * (1 - p)
    other = vj_dropout_mask_ref(1235, np.arange(512), np.arange(1024), p)
    assert (keep != other).mean() > 0.5 * 2 * p * (1 - p)
    assert vj_dropout_mask_ref(7, np.arange(4), np.arange(8), 0.0).all()


# ------------------------------------------------------------------------------------------------
DEV = "cuda"


def _bf(x):
    return x.bfloat16().float()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["plain", "resid_f32", "resid_bf16", "aux"])
@pytest.mark.parametrize("x_f32", [True, False])
def test_dropout_kernel_bit_exact(mode, x_f32):
    """vj_dropout vs torch on the restated mask: y = bf16(bf16(x) * z), + resid / * aux as documented."""
    from vjepa2_amd import ops

    g = torch.Generator().manual_seed(3)
    M, N, p, seed = 300, 520, 0.3, 987654321
    x = torch.randn(M, N, generator=g) * 3
    x = x if x_f32 else x.bfloat16()
    z = torch.from_numpy(vj_dropout_mask_ref(seed, np.arange(M), np.arange(N), p)).float() / (1 - p)
    y = _bf(_bf(x.float()) * z)
    kw = {}
    if mode == "resid_f32":
        r = torch.randn(M, N, generator=g)
        kw["resid"], exp = r.to(DEV), r + y
    elif mode == "resid_bf16":
        r = torch.randn(M, N, generator=g).bfloat16()
        kw["resid"], exp = r.to(DEV), _bf(r.float() + y)
    elif mode == "aux":
        a = torch.randn(M, N, generator=g).bfloat16()
        kw["aux"], exp = a.to(DEV), _bf(y * a.float())
    else:
        exp = y
    out = ops.dropout(x.to(DEV), p, seed, **kw)
    torch.cuda.synchronize()
    assert torch.equal(out.float().cpu(), exp), (out.float().cpu() - exp).abs().max()


def _attn_drop_ref(q, k, v, groups, scale, H, p, seed, fblk=0):
    """fp32 attention with the kernels' dropout mask: O = (softmax(S) * Z) V, Z[t, h, j] = keep / (1 - p)
    for query token t, head h, key j of its sequence (mask row t * H + h, column j); fblk > 0 adds the
    frame-causal mask (key j visible to query i iff j // fblk <= i // fblk, modules.py:12-23)."""
    outs, t0 = [], 0
    for ns, ln in groups:
        for _ in range(ns):
            qq, kk, vv = (x[t0:t0 + ln].transpose(0, 1) for x in (q, k, v))
            s = (qq @ kk.transpose(-1, -2)) * scale
            if fblk:
                f = torch.arange(ln) // fblk
                s = s.masked_fill(f[None, :] > f[:, None], float("-inf"))
            rows = (np.arange(t0, t0 + ln)[None, :] * H + np.arange(H)[:, None]).reshape(-1)
            z = torch.from_numpy(vj_dropout_mask_ref(seed, rows, np.arange(ln), p)).float().reshape(H, ln, ln)
            outs.append(((torch.softmax(s, -1) * z / (1 - p)) @ vv).transpose(0, 1))
            t0 += ln
    return torch.cat(outs, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("hd,H,groups,fblk", [(64, 2, [(3, 70), (2, 130)], 0), (32, 3, [(2, 257), (1, 5)], 0),
                                              (32, 2, [(1, 1504)], 0), (88, 2, [(1, 200), (3, 31)], 0),
                                              # frame-causal (the action-conditioned predictor), partial last frame
                                              (64, 2, [(1, 500), (2, 70)], 130)])
def test_attention_dropout_fwd_bwd(hd, H, groups, fblk):
    """Attention dropout (vj_attn_fwd_ex / vj_attn_bwd_ex) vs fp32 autograd on the same mask; the
    statistics (lse) are those of the undropped scores; deterministic for a seed."""
    from vjepa2_amd import ops

    T = sum(n * l for n, l in groups)
    D = H * hd
    p, seed = 0.2, 4242
    g = torch.Generator().manual_seed(hd + T)
    qkv = torch.randn(T, 3 * D, generator=g).to(DEV).bfloat16()
    scale = hd ** -0.5
    o, stats = ops.attn_fwd(qkv, H, hd, groups, scale, dropout_p=p, seed=seed, fblk=fblk)
    o0, stats0 = ops.attn_fwd(qkv, H, hd, groups, scale, fblk=fblk)
    q, k, v = (qkv[:, i * D:(i + 1) * D].float().cpu().reshape(T, H, hd).requires_grad_(True) for i in range(3))
    o_ref = _attn_drop_ref(q, k, v, groups, scale, H, p, seed, fblk)
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.float().cpu() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    assert rel(o.reshape(T, H, hd), o_ref.detach()) < 1e-2
    assert torch.equal(stats[0], stats0[0])  # log-sum-exp of the undropped scores
    do = torch.randn(T, D, generator=g).bfloat16()
    o_ref.backward(do.float().reshape(T, H, hd))
    dqkv = ops.attn_bwd(qkv, o, do.to(DEV), stats, H, hd, groups, scale, dropout_p=p, seed=seed, fblk=fblk)
    torch.cuda.synchronize()
    for i, (name, t) in enumerate((("dq", q), ("dk", k), ("dv", v))):
        r = rel(dqkv[:, i * D:(i + 1) * D].reshape(T, H, hd), t.grad)
        assert r < 2e-2, (name, r)
    assert torch.equal(dqkv, ops.attn_bwd(qkv, o, do.to(DEV), stats, H, hd, groups, scale, dropout_p=p, seed=seed,
                                          fblk=fblk))


@pytest.mark.gpu
@pytest.mark.parametrize("sdpa", [True, False])
def test_block_dropout_vs_fp32_reference(sdpa, monkeypatch):
    """Block(drop=0.15, attn_drop=0.1) in training (modules.py:500-563): attention dropout (proj_drop_prob
    under SDPA, attn_drop without), proj_drop and the MLP's two dropouts, forward and backward, vs an
    fp32 autograd Block using the masks of the seeds the HIP path drew."""
    import torch.nn as tnn

    from vjepa2_amd import functions as fn
    from vjepa2_amd.modules import Block

    seeds = iter([11, 22, 33, 44, 55])
    drawn = []

    def fake_seed():
        s = next(seeds)
        drawn.append(s)
        return s

    monkeypatch.setattr(fn, "_drop_seed", fake_seed)
    torch.manual_seed(0)
    D, H, hd, B, N = 128, 2, 64, 2, 96
    pd, pa = 0.15, 0.1
    blk = Block(D, H, qkv_bias=True, drop=pd, attn_drop=pa, use_sdpa=sdpa).to(DEV)
    blk.train()
    x = torch.randn(B, N, D, device=DEV, requires_grad=True)
    y = blk(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    torch.cuda.synchronize()
    p_attn = pd if sdpa else pa
    sa, sp, sm1, sm2 = drawn

    # fp32 reference with the same masks
    ps = {n: t.detach().float().cpu().clone().requires_grad_(True) for n, t in blk.named_parameters()}
    xr = x.detach().float().cpu().requires_grad_(True)
    T = B * N

    def z(seed, p, rows, cols):
        return torch.from_numpy(vj_dropout_mask_ref(seed, np.arange(rows), np.arange(cols), p)).float() / (1 - p)

    def ln(t, w, b):
        return tnn.functional.layer_norm(t, (D,), w, b, blk.norm1.eps)

    t = xr.reshape(T, D)
    h1 = ln(t, ps["norm1.weight"], ps["norm1.bias"])
    qkv = h1 @ ps["attn.qkv.weight"].t() + ps["attn.qkv.bias"]
    q, k, v = (qkv[:, i * D:(i + 1) * D].reshape(T, H, hd) for i in range(3))
    o = _attn_drop_ref(q, k, v, [(B, N)], hd ** -0.5, H, p_attn, sa).reshape(T, D)
    xm = t + (o @ ps["attn.proj.weight"].t() + ps["attn.proj.bias"]) * z(sp, pd, T, D)
    h2 = ln(xm, ps["norm2.weight"], ps["norm2.bias"])
    act = tnn.functional.gelu(h2 @ ps["mlp.fc1.weight"].t() + ps["mlp.fc1.bias"]) * z(sm1, pd, T, 4 * D)
    yr = xm + (act @ ps["mlp.fc2.weight"].t() + ps["mlp.fc2.bias"]) * z(sm2, pd, T, D)
    yr.backward(dy.float().cpu().reshape(T, D))

    rel = lambda a, b: ((a.float().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y.reshape(T, D), yr.detach()) < 1e-2
    assert rel(x.grad, xr.grad) < 2e-2
    for n, prm in blk.named_parameters():
        assert rel(prm.grad, ps[n].grad) < 3e-2, (n, rel(prm.grad, ps[n].grad))
