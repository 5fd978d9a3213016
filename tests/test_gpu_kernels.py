"""GPU parity tests of every HIP kernel against a plain-PyTorch fp32 reference (or the oracle).

Tolerances: bf16 operands with fp32 accumulation are compared to fp32 math on the SAME bf16-rounded
operands, so only accumulation order and the bf16 rounding of outputs differ:
  - f32 outputs:  |err| <= 1e-4 * sqrt(K) * scale     - bf16 outputs: 1 bf16 ulp (rtol 2^-7)
Index/byte kernels (gather/scatter/fill/index build) must be bit-exact.
"""

import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vjepa_oracle as orc  # noqa: E402

DEV = "cuda"


def _close(got, exp, atol, rtol, what):
    got = got.detach().float().cpu()
    exp = exp.detach().float().cpu()
    err = (got - exp).abs()
    bad = err > atol + rtol * exp.abs()
    assert not bool(bad.any()), (
        f"{what}: max abs err {err.max().item():.3e} (atol {atol}, rtol {rtol}), "
        f"{int(bad.sum())}/{bad.numel()} bad")


# ------------------------------------------------------------------------------------------------
GEMM_SHAPES = [(128, 128, 64), (300, 136, 72), (264, 200, 1000), (1, 8, 8), (520, 384, 1536),
               # M >= 1024 -> 256-row tile kernel (vj_gemm256.hip): BN=128 ragged, BN=256, K tail, N tail
               (1100, 384, 1536), (2048, 1024, 200), (1500, 640, 264), (1030, 1160, 128)]


@pytest.mark.parametrize("a_kmajor", [True, False])
@pytest.mark.parametrize("b_kmajor", [True, False])
@pytest.mark.parametrize("shape", GEMM_SHAPES)
def test_gemm_layouts(a_kmajor, b_kmajor, shape):
    from vjepa2_amd import ops

    M, N, K = shape
    if not a_kmajor and M % 8:
        M += 8 - M % 8
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    B = torch.randn(N, K, generator=g).to(DEV).bfloat16()
    bias = torch.randn(N, generator=g).to(DEV)
    exp = A.float() @ B.float().t() + bias
    a_store = A.contiguous() if a_kmajor else A.t().contiguous()
    b_store = B.contiguous() if b_kmajor else B.t().contiguous()
    out = torch.empty(M, N, device=DEV)
    ops.gemm(M, N, K, a_store, a_store.stride(0), a_kmajor, b_store, b_store.stride(0), b_kmajor, ops.EPI_F32,
             out=out, ldc=N, bias=bias)
    torch.cuda.synchronize()
    _close(out, exp, 1e-4 * math.sqrt(K) * 4, 1e-4, f"gemm {shape} ak={a_kmajor} bk={b_kmajor}")


@pytest.mark.parametrize("MNK", [(200, 136, 3000), (520, 392, 3000), (512, 256, 4100), (600, 1408, 2000)])
@pytest.mark.parametrize("epi", [1, 2, 0])
def test_gemm_splitk(epi, MNK):
    """Deterministic split-K (weight-gradient shape: small M x N, K = tokens). M >= 256 and N >= 128
    take the 256-row-tile partial kernel (BN 128 / 256; N = 1408: 256-wide tiles with a half-empty
    last one, ViT-g's width), the first shape the 128-tile one."""
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(epi)
    M, N, K = MNK
    dY = torch.randn(K, M, generator=g).to(DEV).bfloat16()  # A MN-major: A(m,k) = dY[k][m]
    X = torch.randn(K, N, generator=g).to(DEV).bfloat16()   # B MN-major
    bias = torch.randn(N, generator=g).to(DEV)
    resid = torch.randn(M, N, generator=g).to(DEV)
    exp = dY.float().t() @ X.float() + bias
    if epi == ops.EPI_F32_RESID:
        exp = exp + resid
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16 if epi == ops.EPI_BF16 else torch.float32)
    runs = []
    for _ in range(2):
        ops.gemm(M, N, K, dY, M, False, X, N, False, epi, out=out, ldc=N, bias=bias,
                 aux=resid if epi == ops.EPI_F32_RESID else None, ldaux=N, splitk=5)
        runs.append(out.clone())
    first = runs[0]
    torch.cuda.synchronize()
    _close(out, exp, 2e-3 if epi == 0 else 2e-4 * math.sqrt(K), 8e-3 if epi == 0 else 1e-5, f"splitk epi={epi}")
    assert torch.equal(out, first), "split-K must be deterministic"


@pytest.mark.parametrize("NKM", [(1024, 1024, 11712), (4096, 1024, 5000), (1152, 384, 3000), (1032, 1408, 2000),
                                 (384, 1152, 71232), (200, 136, 3000), (1024, 1024, 700), (12, 64, 999)])
@pytest.mark.parametrize("acc", [False, True])
def test_wgrad_fused_bias(NKM, acc):
    """vj_gemm_bf16_wgrad: dW (+)= dY^T X and db (+)= dY.sum(0) in one call (nn.Linear's weight and bias
    gradients). Split-K shapes with M >= 256 sum the bias inside the 256-row partial kernel (column tile
    0's A fragments; ragged M = 1032 / 1152, BN = 128 for N = 384, 256-wide N = 1408); the rest (128-tile
    kernel, no split, a 12-wide output) take the column-sum pass. Against float64 sums of the same bf16
    values; deterministic."""
    from vjepa2_amd import ops

    N, K, M = NKM
    g = torch.Generator(device="cpu").manual_seed(N + K + M)
    dY = torch.randn(M, N, generator=g).to(DEV).bfloat16()
    X = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    dw0, db0 = torch.randn(N, K, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    exp_w = dY.double().t() @ X.double() + (dw0.double() if acc else 0)
    exp_b = dY.double().sum(0) + db0.double()  # db always accumulates (grad_buf semantics)
    outs = []
    for _ in range(2):
        dw, db = dw0.clone(), db0.clone()
        ops.linear_wgrad(dY, X, dw, accumulate=acc, db=db)
        outs.append((dw, db))
    torch.cuda.synchronize()
    _close(outs[0][0], exp_w, 2e-4 * math.sqrt(M), 1e-5, f"wgrad dW {NKM}")
    _close(outs[0][1], exp_b, 2e-5 * math.sqrt(M), 1e-5, f"wgrad db {NKM}")
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), "must be deterministic"


@pytest.mark.parametrize("N", [256, 384, 200, 1152])
@pytest.mark.parametrize("M", [333, 1333])
def test_gemm_epilogues(M, N):
    """Every epilogue; M >= 1024 runs the 256-row kernel (N = 256: 256-wide tiles, 384 / 200: 128-wide,
    200 ragged, 1152: 256-wide with a half-empty last column tile), whose K-major-B forms store straight
    from registers (permuted B staging)."""
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(0)
    K = 192
    X = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    W = (0.1 * torch.randn(N, K, generator=g)).to(DEV).bfloat16()
    b = torch.randn(N, generator=g).to(DEV)
    ref = X.float() @ W.float().t() + b
    y = ops.linear_fwd(X, W, b, ops.EPI_BF16)
    _close(y, ref, 1e-3, 8e-3, "EPI_BF16")
    resid = torch.randn(M, N, generator=g).to(DEV)
    y = ops.linear_fwd(X, W, b, ops.EPI_F32_RESID, resid=resid)
    _close(y, ref + resid, 2e-4, 1e-5, "EPI_F32_RESID")
    rb = resid.bfloat16()  # bf16 residual stream (no-grad target encoder): one rounding of acc + b + r
    y = ops.linear_fwd(X, W, b, ops.EPI_BF16_RESID, resid=rb)
    assert y.dtype == torch.bfloat16
    _close(y, ref + rb.float(), 1e-3, 8e-3, "EPI_BF16_RESID")
    pre = ops.linear_fwd(X, W, b, ops.EPI_BF16)  # the same bf16 pre-activation the GELU epilogue rounds
    dgelu, act = ops.linear_fwd(X, W, b, ops.EPI_GELU, out=torch.empty(M, N, device=DEV, dtype=torch.bfloat16))
    _, act2 = ops.linear_fwd(X, W, b, ops.EPI_GELU)  # no derivative requested (no-grad target path)
    assert torch.equal(act, act2)
    xp = pre.float().requires_grad_(True)
    yp = torch.nn.functional.gelu(xp)
    yp.backward(torch.ones_like(yp))
    _close(act, yp.detach(), 1e-3, 8e-3, "EPI_GELU act")
    _close(dgelu, xp.grad, 1e-3, 8e-3, "EPI_GELU saved derivative")
    # GELU of the bf16 pre-activation, rounded once (erf polynomial, |err| <= 1.5e-7): 1-ulp ties only
    assert float((act == yp.detach().bfloat16()).float().mean()) > 0.995
    assert float((dgelu == xp.grad.bfloat16()).float().mean()) > 0.995
    # GELU backward epilogue: out = (dY W) * saved derivative
    dY = torch.randn(M, N, generator=g).to(DEV).bfloat16()
    W2 = (0.1 * torch.randn(N, K, generator=g)).to(DEV).bfloat16()
    pre2 = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    x = pre2.float().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(dY.float() @ W2.float())
    xd = pre2.float().requires_grad_(True)
    torch.nn.functional.gelu(xd).sum().backward()
    dg2 = xd.grad.bfloat16()  # what the forward epilogue saves
    got = ops.linear_dgrad(dY, W2, gelu_grad=dg2)
    _close(got, x.grad, 2e-3, 1.5e-2, "EPI_GELU_BWD")
    # the same with B K-major (direct-store epilogue) and the plain f32 epilogue
    W2t = W2.t().contiguous()  # [K, N]: B(n=k_out, k=n_in) K-major
    got2 = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    ops.gemm(M, K, N, dY, N, True, W2t, N, True, ops.EPI_GELU_BWD, out=got2, ldc=K, aux=dg2, ldaux=K)
    _close(got2, x.grad, 2e-3, 1.5e-2, "EPI_GELU_BWD (B K-major)")
    got3 = ops.linear_dgrad(dY, W2, gelu_grad=dg2, wt=ops.transpose_bf16(W2))
    _close(got3, x.grad, 2e-3, 1.5e-2, "EPI_GELU_BWD (linear_dgrad on W^T)")
    f32 = torch.empty(M, K, device=DEV)
    ops.gemm(M, K, N, dY, N, True, W2t, N, True, ops.EPI_F32, out=f32, ldc=K)
    _close(f32, dY.float() @ W2.float(), 2e-4 * math.sqrt(N), 1e-5, "EPI_F32 (B K-major)")
    # wgrad accumulate
    dw = torch.randn(N, K, generator=g).to(DEV)
    exp = dw + dY.float().t() @ pre2.float()
    ops.linear_wgrad(dY, pre2, dw)
    _close(dw, exp, 2e-4 * math.sqrt(M), 1e-5, "wgrad accumulate")


@pytest.mark.parametrize("two_wg", ["0", "1"])
def test_gemm_bf16_resid_tile_paths(two_wg, monkeypatch):
    """EPI_BF16_RESID through the LDS-staged epilogue (8-wave, 128-wide tiles: VJ_GEMM_2W=0) and the
    two-workgroup direct-store kernel (VJ_GEMM_2W=1), N = 384 (not a multiple of 256)."""
    from vjepa2_amd import ops

    monkeypatch.setenv("VJ_GEMM_2W", two_wg)
    g = torch.Generator(device="cpu").manual_seed(5)
    M, N, K = 1333, 384, 320
    X = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    W = (0.1 * torch.randn(N, K, generator=g)).to(DEV).bfloat16()
    b = torch.randn(N, generator=g).to(DEV)
    r = torch.randn(M, N, generator=g).to(DEV).bfloat16()
    y = ops.linear_fwd(X, W, b, ops.EPI_BF16_RESID, resid=r)
    _close(y, X.float() @ W.float().t() + b + r.float(), 1e-3, 8e-3, f"EPI_BF16_RESID (2W={two_wg})")


@pytest.mark.parametrize("knobs", [dict(VJ_GEMM_PXCD="1"), dict(VJ_GEMM_PXCD="3", VJ_GEMM_GROUP="3")])
def test_gemm_persistent_walk(knobs, monkeypatch):
    """The 256-row kernel is persistent: with few blocks per XCD every block walks many tiles, which
    exercises the next-tile DMA hand-off (slot parity for odd K-tile counts, K <= 64 single-tile,
    ragged tails) for every layout and epilogue, plus the grouped tile order."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    for shape in [(2100, 768, 320), (1500, 384, 64), (1030, 1160, 128), (2048, 1024, 200)]:
        for ak in (True, False):
            for bk in (True, False):
                test_gemm_layouts(ak, bk, shape)
    for M, N in [(1333, 256), (1333, 384), (1333, 200)]:
        test_gemm_epilogues(M, N)
    test_gemm_splitk(2, (520, 392, 3000))
    test_gemm_splitk(0, (512, 256, 4100))
    test_fused_rope_paths(1500, 64, 2, monkeypatch)


# ------------------------------------------------------------------------------------------------
def _attn_ref(q, k, v, groups, scale):
    """q,k,v f32 [T, H, hd] (concatenated sequences) -> O [T,H,hd], lse [H,T]"""
    outs, lses = [], []
    t0 = 0
    for ns, ln in groups:
        for _ in range(ns):
            qq, kk, vv = (x[t0:t0 + ln].transpose(0, 1) for x in (q, k, v))
            s = (qq @ kk.transpose(-1, -2)) * scale
            lses.append(torch.logsumexp(s, -1))
            outs.append((torch.softmax(s, -1) @ vv).transpose(0, 1))
            t0 += ln
    return torch.cat(outs, 0), torch.cat(lses, 1)


@pytest.mark.parametrize("hd,H,groups", [(64, 2, [(3, 70), (2, 130)]), (32, 3, [(2, 257), (1, 5)]),
                                         (64, 1, [(1, 128)]), (32, 2, [(4, 33)]),
                                         # vit_huge / vit_giant head dims (padded to 96 inside)
                                         (80, 2, [(2, 150), (1, 33)]), (88, 2, [(1, 200), (3, 31)]),
                                         # long sequences: ViT-L 16x256^2 (2048), ViT-g 16x384^2 (4608)
                                         (64, 2, [(1, 2048), (1, 4608)]), (32, 2, [(1, 4608), (1, 1504)]),
                                         # ViT-g 64x256^2: predictor n = 6013 (hd 32), context K = 2398
                                         # and the full 8192-token target sequence (hd 64)
                                         (32, 2, [(1, 6013)]), (64, 2, [(1, 2398), (1, 8192)])])
def test_attention_fwd_bwd(hd, H, groups, monkeypatch):
    """Forward / backward vs fp32 autograd: the two sweeps (the dQ sweep, which recomputes S, P, dP,
    computes delta itself and runs first; then the dK/dV sweep); bitwise deterministic."""
    from vjepa2_amd import ops

    T = sum(n * l for n, l in groups)
    D = H * hd
    g = torch.Generator(device="cpu").manual_seed(hd + T)
    qkv = torch.randn(T, 3 * D, generator=g).to(DEV).bfloat16()
    scale = hd ** -0.5
    o, stats = ops.attn_fwd(qkv, H, hd, groups, scale)
    q, k, v = (qkv[:, i * D:(i + 1) * D].float().reshape(T, H, hd).requires_grad_(True) for i in range(3))
    o_ref, lse_ref = _attn_ref(q, k, v, groups, scale)
    torch.cuda.synchronize()
    _close(o.reshape(T, H, hd), o_ref, 1e-2, 2e-2, f"attn fwd hd={hd}")
    _close(stats[0] * math.log(2.0), lse_ref, 2e-3, 1e-4, f"attn lse hd={hd}")  # stats hold log2 units
    do = torch.randn(T, D, generator=g).to(DEV).bfloat16()
    o_ref.backward(do.float().reshape(T, H, hd))
    dqkv = ops.attn_bwd(qkv, o, do, stats, H, hd, groups, scale)
    torch.cuda.synchronize()
    for i, (name, t) in enumerate((("dq", q), ("dk", k), ("dv", v))):
        _close(dqkv[:, i * D:(i + 1) * D].reshape(T, H, hd), t.grad, 2e-2, 3e-2, f"attn {name} hd={hd}")
    # determinism
    dqkv2 = ops.attn_bwd(qkv, o, do, stats, H, hd, groups, scale)
    assert torch.equal(dqkv, dqkv2)


@pytest.mark.parametrize("M,N,K,epi", [(300, 520, 1024, 1), (1100, 384, 200, 2), (64, 4096, 1024, 3), (5, 8, 3, 1)])
def test_gemm_f32_parity_mode(M, N, K, epi):
    """fp32-operand parity mode GEMM (v_mfma_f32_32x32x2_f32) vs fp64 math: f32 accumulation only."""
    from vjepa2_amd import ops

    g = torch.Generator().manual_seed(M + N + K)
    a, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5, torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g)
    exp = a.double() @ w.double().t() + b.double()
    bound = 4 * K * 2.0 ** -24 * (a.double().abs() @ w.double().abs().t() + b.double().abs())
    out = ops.linear_fwd_f32(a.to(DEV), w.to(DEV), b.to(DEV), epi, resid=r.to(DEV) if epi == 2 else None)
    torch.cuda.synchronize()
    if epi == 2:
        exp = exp + r.double()
        bound = bound + 2.0 ** -23 * exp.abs()
    if epi == 3:
        pre, act = out
        assert ((pre.cpu().double() - exp).abs() <= bound).all()
        ga = torch.nn.functional.gelu(pre.cpu().double())
        assert (act.cpu().double() - ga).abs().max().item() <= 1e-6 * max(1.0, ga.abs().max().item())
    else:
        assert ((out.cpu().double() - exp).abs() <= bound).all()


@pytest.mark.parametrize("hd,H,groups", [(64, 2, [(2, 300), (1, 77)]), (32, 3, [(1, 1504)]), (88, 1, [(2, 130)])])
def test_attention_f32_parity_mode(hd, H, groups):
    """fp32-operand parity mode attention vs fp32 torch softmax attention (ulp-level)."""
    from vjepa2_amd import ops

    T = sum(n * l for n, l in groups)
    D = H * hd
    qkv = torch.randn(T, 3 * D, generator=torch.Generator().manual_seed(hd + T))
    o, lse = ops.attn_fwd_f32(qkv.to(DEV), H, hd, groups, hd ** -0.5)
    q, k, v = (qkv[:, i * D:(i + 1) * D].double().reshape(T, H, hd) for i in range(3))
    o_ref, lse_ref = _attn_ref(q, k, v, groups, hd ** -0.5)
    torch.cuda.synchronize()
    _close(o.reshape(T, H, hd), o_ref, 2e-6, 2e-5, f"attn f32 hd={hd}")
    _close(lse, lse_ref, 2e-6, 2e-6, f"attn f32 lse hd={hd}")


SPIKE_BWD_REL = 1.0e-2


@pytest.mark.parametrize("hd", [64, 32, 80])
def test_attention_rescale_spikes(hd):
    """Score maxima that grow tile after tile (every step takes the lazy-rescale branch) and one
    isolated spike key per sequence: exercises the O/l rescale of the pipelined forward."""
    from vjepa2_amd import ops

    H, groups = 2, [(2, 300), (1, 77)]
    T = sum(n * l for n, l in groups)
    D = H * hd
    g = torch.Generator(device="cpu").manual_seed(7 * hd)
    qkv = torch.randn(T, 3 * D, generator=g)
    t0 = 0
    for ns, ln in groups:
        for _ in range(ns):
            ramp = torch.linspace(0.5, 6.0, ln).unsqueeze(1)
            qkv[t0:t0 + ln, D:2 * D] *= ramp  # keys grow with position -> max rises every tile
            qkv[t0 + ln // 2, D:2 * D] = qkv[t0, :D] * 8.0  # spike aligned with the first query
            t0 += ln
    qkv = qkv.to(DEV).bfloat16()
    scale = hd ** -0.5
    o, stats = ops.attn_fwd(qkv, H, hd, groups, scale)
    q, k, v = (qkv[:, i * D:(i + 1) * D].float().reshape(T, H, hd).requires_grad_(True) for i in range(3))
    o_ref, lse_ref = _attn_ref(q, k, v, groups, scale)
    torch.cuda.synchronize()
    _close(o.reshape(T, H, hd), o_ref, 1e-2, 2e-2, f"attn spikes fwd hd={hd}")
    _close(stats[0] * math.log(2.0), lse_ref, 2e-3, 1e-4, f"attn spikes lse hd={hd}")
    # the backward on the same large, growing logits (the spike key's score is ~8 |q|^2)
    do = torch.randn(T, D, generator=g).to(DEV).bfloat16()
    o_ref.backward(do.float().reshape(T, H, hd))
    dqkv = ops.attn_bwd(qkv, o, do, stats, H, hd, groups, scale)
    torch.cuda.synchronize()
    # elementwise bounds do not fit here (dq of the spike rows is large; P and dS are bf16 MFMA
    # operands), so the bound is on the relative L2 error of each gradient
    for i, (name, t) in enumerate((("dq", q), ("dk", k), ("dv", v))):
        got = dqkv[:, i * D:(i + 1) * D].reshape(T, H, hd).float().cpu()
        exp = t.grad.float().cpu()
        rel = ((got - exp).norm() / exp.norm()).item()
        print(f"attn spikes {name} hd={hd}: relative L2 error {rel:.3e}")
        assert rel < SPIKE_BWD_REL, (name, hd, rel)


# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("fwd", ["default", "1"])
@pytest.mark.parametrize("D", [64, 384, 1024, 1408])
def test_layernorm(D, fwd, monkeypatch):
    """LayerNorm forward (k_ln_fwd3: all rows of a wave in flight; VJ_LN_FWD=1 and f32 rows wider
    than 1024: k_ln_fwd) and backward vs torch, f32 / bf16 inputs and outputs."""
    from vjepa2_amd import ops

    if fwd != "default":
        monkeypatch.setenv("VJ_LN_FWD", fwd)

    g = torch.Generator(device="cpu").manual_seed(D)
    M = 301
    x = (3 * torch.randn(M, D, generator=g) + 1).to(DEV)
    w = torch.randn(D, generator=g).to(DEV)
    b = torch.randn(D, generator=g).to(DEV)
    y, mean, rstd = ops.layernorm_fwd(x, w, b, 1e-6, out_dtype=torch.float32)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-6)
    _close(y, yr, 1e-4, 1e-4, "ln fwd")
    yb, _, _ = ops.layernorm_fwd(x, w, b, 1e-6)
    _close(yb, yr, 1e-3, 8e-3, "ln fwd bf16")
    # bf16 input rows (the no-grad target encoder's bf16 residual stream), f32 and bf16 outputs
    xb = x.bfloat16()
    ref_b = torch.nn.functional.layer_norm(xb.float(), (D,), w, b, 1e-6)
    y32b, mb, rb = ops.layernorm_fwd(xb, w, b, 1e-6, out_dtype=torch.float32)
    _close(y32b, ref_b, 1e-4, 1e-4, "ln fwd (bf16 x)")
    _close(mb, xb.float().mean(1), 1e-5, 1e-5, "ln fwd mean (bf16 x)")
    y16b, _, _ = ops.layernorm_fwd(xb, w, b, 1e-6)
    _close(y16b, ref_b, 1e-3, 8e-3, "ln fwd bf16 (bf16 x)")
    dy = torch.randn(M, D, generator=g).to(DEV).bfloat16()
    yr.backward(dy.float())
    dres_in = torch.randn(M, D, generator=g).to(DEV)
    dw = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    dres, dres_bf = ops.layernorm_bwd(dy, x, mean, rstd, w, dres_in=dres_in, dweight=dw, dbias=db, want_bf16=True)
    torch.cuda.synchronize()
    _close(dres, xr.grad + dres_in, 1e-4, 1e-4, "ln bwd dx")
    _close(dres_bf, xr.grad + dres_in, 1e-3, 8e-3, "ln bwd dx bf16")
    _close(dw, wr.grad, 1e-3, 1e-4, "ln bwd dgamma")
    _close(db, br.grad, 1e-3, 1e-4, "ln bwd dbeta")
    # fused bias gradients: column sums of dres_in and of dres, accumulated
    dw2, db2 = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    s_in, s_out = torch.ones(D, device=DEV), torch.ones(D, device=DEV)
    dres2, _ = ops.layernorm_bwd(dy, x, mean, rstd, w, dres_in=dres_in, dweight=dw2, dbias=db2, sum_in=s_in,
                                 sum_out=s_out)
    torch.cuda.synchronize()
    assert torch.equal(dres2, dres) and torch.equal(dw2, dw) and torch.equal(db2, db)
    _close(s_in, 1 + dres_in.sum(0), 1e-3, 1e-4, "ln bwd sum(dres_in)")
    _close(s_out, 1 + (xr.grad + dres_in).sum(0), 1e-3, 1e-4, "ln bwd sum(dres)")
    if D % 8:
        return
    # bf16 residual stream (the trained context encoder under bf16 autocast): x, dres_in bf16; dres bf16
    # = bf16(dres_in + dLN/dx) from the f32 sum; the same column partials
    xbr = xb.float().requires_grad_(True)
    torch.nn.functional.layer_norm(xbr, (D,), w, b, 1e-6).backward(dy.float())
    dres_in_b = dres_in.bfloat16()
    exact = xbr.grad + dres_in_b.float()
    dw3, db3 = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    s_in3, s_out3 = torch.ones(D, device=DEV), torch.ones(D, device=DEV)
    dres3, same = ops.layernorm_bwd(dy, xb, mb, rb, w, dres_in=dres_in_b, dweight=dw3, dbias=db3, sum_in=s_in3,
                                    sum_out=s_out3)
    torch.cuda.synchronize()
    assert dres3.dtype == torch.bfloat16 and same is dres3
    # one bf16 rounding of an f32 value within 1e-4 relative of the exact sum: at most 1 ulp off
    ulp = torch.clamp(exact.abs(), min=1e-30) * 2.0 ** -7
    assert ((dres3.float() - exact).abs() <= ulp + 1e-5).all(), "ln bwd bf16 stream: more than 1 ulp off"
    _close(dw3, (dy.float() * ((xb.float() - mb[:, None]) * rb[:, None])).sum(0), 1e-3, 1e-4, "ln bwd dgamma (bf16 x)")
    _close(db3, dy.float().sum(0), 1e-3, 1e-4, "ln bwd dbeta (bf16 x)")
    _close(s_in3, 1 + dres_in_b.float().sum(0), 1e-3, 1e-4, "ln bwd sum(dres_in) (bf16)")
    _close(s_out3, 1 + exact.sum(0), 1e-3, 1e-4, "ln bwd sum(dres) (bf16)")
    dres4, _ = ops.layernorm_bwd(dy, xb, mb, rb, w)  # no residual input, no column sums
    torch.cuda.synchronize()
    assert ((dres4.float() - xbr.grad).abs() <= torch.clamp(xbr.grad.abs(), min=1e-30) * 2.0 ** -7 + 1e-5).all()


def test_colsum():
    from vjepa2_amd import ops

    x = torch.randn(70000, 96, device=DEV).bfloat16()
    out = torch.ones(96, device=DEV)
    ops.colsum(x, out, accumulate=True)
    _close(out, 1 + x.float().sum(0), 5e-3, 1e-4, "colsum")


# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("hd,H", [(64, 2), (32, 3), (80, 2), (88, 2)])
def test_rope_fwd_bwd(hd, H):
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(hd)
    T, D = 200, H * hd
    tpf, tpr = 16, 4  # 4x4 grid, up to 12 frames
    ids = torch.randint(0, 12 * 16, (T,), generator=g)
    qkv = torch.randn(T, 3 * D, generator=g).bfloat16()
    cos_t, sin_t = orc.rope_tables(hd, 16)
    qkv_d = qkv.to(DEV)
    ops.rope_(qkv_d, H, hd, 0, D, ids.to(DEV).int(), 0, tpf, tpr, cos_t.to(DEV), sin_t.to(DEV))
    q = qkv[:, :D].float().reshape(T, H, hd).transpose(0, 1)[None].requires_grad_(True)
    k = qkv[:, D:2 * D].float().reshape(T, H, hd).transpose(0, 1)[None]
    qr, kr = orc.apply_rope_qk(q, k, ids[None], tpf, tpr)
    torch.cuda.synchronize()
    got = qkv_d.cpu().float()
    _close(got[:, :D], qr[0].transpose(0, 1).reshape(T, D), 1e-5, 8e-3, "rope q")
    _close(got[:, D:2 * D], kr[0].transpose(0, 1).reshape(T, D), 1e-5, 8e-3, "rope k")
    assert torch.equal(got[:, 2 * D:], qkv[:, 2 * D:].float()), "rope touched v"
    # inverse == transpose (autograd of the oracle map)
    gq = torch.randn(T, D, generator=g).bfloat16()
    qr.backward(gq.float().reshape(T, H, hd).transpose(0, 1)[None])
    buf = torch.zeros(T, 3 * D).bfloat16()
    buf[:, :D] = gq
    buf_d = buf.to(DEV)
    ops.rope_(buf_d, H, hd, 0, D, ids.to(DEV).int(), 0, tpf, tpr, cos_t.to(DEV), sin_t.to(DEV), inverse=True)
    torch.cuda.synchronize()
    _close(buf_d.cpu()[:, :D], q.grad[0].transpose(0, 1).reshape(T, D), 1e-5, 8e-3, "rope inverse")


@pytest.mark.parametrize("M", [300, 1500])
@pytest.mark.parametrize("hd,H", [(64, 2), (32, 3), (80, 2), (88, 1), (32, 12)])
def test_fused_rope_paths(M, hd, H, monkeypatch):
    """QKV GEMM with RoPE fused into the epilogue vs fp32 GEMM + oracle RoPE (M >= 1024: one bf16
    rounding of the fp32 result, <= 1 ulp; M < 1024 takes GEMM -> bf16 -> rope -> bf16, two
    roundings, so the bound is 1 ulp of the rotated inputs). Attention backward with the inverse
    RoPE fused into the dq/dk stores vs fp32 autograd of softmax attention and of the oracle RoPE."""
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(M + hd)
    D, K = H * hd, 128
    tpf, tpr = 16, 4
    ids = torch.randint(0, 8 * 16, (M,), generator=g).to(DEV).int()
    cos_t, sin_t = (t.to(DEV) for t in orc.rope_tables(hd, 16))
    x = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    w = (0.1 * torch.randn(3 * D, K, generator=g)).to(DEV).bfloat16()
    b = torch.randn(3 * D, generator=g).to(DEV)
    fused = ops.qkv_rope(x, w, b, H, hd, ids, 0, tpf, tpr, cos_t, sin_t)
    if M >= 1024:
        # 192-row tiles (where N takes 256-wide ones), the one-tile and the staggered main loop: the
        # same MFMAs in the same K order, bitwise equal
        for bm, stg in (("1", "0"), ("0", "0"), ("0", "1")):
            monkeypatch.setenv("VJ_GEMM_BM192", bm)
            monkeypatch.setenv("VJ_GEMM_STG", stg)
            other = ops.qkv_rope(x, w, b, H, hd, ids, 0, tpf, tpr, cos_t, sin_t)
            assert torch.equal(fused, other), f"qkv_rope: VJ_GEMM_BM192={bm} VJ_GEMM_STG={stg} differs"
        monkeypatch.delenv("VJ_GEMM_BM192")
        monkeypatch.delenv("VJ_GEMM_STG")
    # expected: our own f32 GEMM (same accumulation), RoPE in fp32 by the oracle
    y32 = ops.linear_fwd(x, w, b, ops.EPI_F32).cpu()
    idl = ids.cpu().long()[None]
    q = y32[:, :D].reshape(M, H, hd).transpose(0, 1)[None]
    k = y32[:, D:2 * D].reshape(M, H, hd).transpose(0, 1)[None]
    qr, kr = orc.apply_rope_qk(q, k, idl, tpf, tpr)
    exp = torch.cat([qr[0].transpose(0, 1).reshape(M, D), kr[0].transpose(0, 1).reshape(M, D), y32[:, 2 * D:]], 1)
    torch.cuda.synchronize()
    if M >= 1024:
        _close(fused, exp, 1e-5, 8e-3, "qkv_rope (fused epilogue)")
    else:
        _close(fused, exp, 8e-3 * float(y32.abs().max()), 8e-3, "qkv_rope (GEMM + rope kernel)")
    assert torch.equal(fused[:, 2 * D:].cpu(), y32[:, 2 * D:].bfloat16()), "v part != bf16(f32 GEMM)"
    # backward with fused inverse rope vs fp32 autograd through attention and the oracle RoPE
    groups = [(M // 100, 100)] if M % 100 == 0 else [(1, M)]
    scale = hd ** -0.5
    o, stats = ops.attn_fwd(fused, H, hd, groups, scale)
    do = torch.randn(M, D, generator=g).to(DEV).bfloat16()
    got = ops.attn_bwd(fused, o, do, stats, H, hd, groups, scale, rope=(ids, 0, tpf, tpr, cos_t, sin_t))
    fc = fused.cpu().float()
    u_q = fc[:, :D].reshape(M, H, hd).transpose(0, 1)[None]  # stands in for the un-rotated q, k:
    u_k = fc[:, D:2 * D].reshape(M, H, hd).transpose(0, 1)[None]  # only the map's transpose matters
    qn = fc[:, :D].reshape(M, H, hd).requires_grad_(True)
    kn = fc[:, D:2 * D].reshape(M, H, hd).requires_grad_(True)
    vn = fc[:, 2 * D:].reshape(M, H, hd).requires_grad_(True)
    o_ref, _ = _attn_ref(qn, kn, vn, groups, scale)
    o_ref.backward(do.cpu().float().reshape(M, H, hd))
    uq = u_q.clone().requires_grad_(True)
    uk = u_k.clone().requires_grad_(True)
    rq, rk = orc.apply_rope_qk(uq, uk, idl, tpf, tpr)
    (rq * qn.grad.transpose(0, 1)[None]).sum().add((rk * kn.grad.transpose(0, 1)[None]).sum()).backward()
    torch.cuda.synchronize()
    gc = got.cpu()
    # bf16 P / dS operands: error scales with the gradient magnitude (q, k here are ~1.5x the
    # unit-variance inputs of test_attention_fwd_bwd, so the softmax is sharper)
    for j, (name, ref) in enumerate((("dq", uq.grad[0].transpose(0, 1)), ("dk", uk.grad[0].transpose(0, 1)),
                                     ("dv", vn.grad))):
        _close(gc[:, j * D:(j + 1) * D].reshape(M, H, hd), ref, 1.5e-2 * float(ref.abs().max()), 3e-2,
               f"attn_bwd fused inverse rope: {name}")


# ------------------------------------------------------------------------------------------------
def test_im2col_patch_embed():
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(5)
    B, C, Tf, Hf, Wf, p, tub, D = 2, 3, 4, 32, 48, 16, 2, 64
    clip = torch.randn(B, C, Tf, Hf, Wf, generator=g)
    w = 0.05 * torch.randn(D, C, tub, p, p, generator=g)
    b = torch.randn(D, generator=g)
    N = (Tf // tub) * (Hf // p) * (Wf // p)
    mask = torch.stack([torch.randperm(N, generator=g)[:5].sort().values for _ in range(B)])
    clip_d = clip.to(DEV)
    cols = ops.im2col(clip_d, p, tub, idx=mask.to(DEV))
    y = ops.linear_fwd(cols, w.reshape(D, -1).to(DEV).bfloat16(), b.to(DEV), ops.EPI_F32)
    ref = torch.nn.functional.conv3d(clip.bfloat16().float(), w.bfloat16().float(), b, stride=(tub, p, p))
    ref = orc.apply_masks(ref.flatten(2).transpose(1, 2), [mask]).reshape(B * 5, D)
    torch.cuda.synchronize()
    _close(y.cpu(), ref, 1e-3, 1e-4, "patch embed (masked)")
    cols_all = ops.im2col(clip_d, p, tub)
    assert cols_all.shape == (B * N, C * tub * p * p)


@pytest.mark.parametrize("shape", [(1024, 4096), (1408, 6144), (384, 1152), (72, 200)])
def test_transpose_bf16(shape):
    from vjepa2_amd import ops

    x = torch.randn(*shape).to(DEV).bfloat16()
    assert torch.equal(ops.transpose_bf16(x), x.t().contiguous())


def test_row_ops_bit_exact():
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(9)
    src = torch.randn(100, 96, generator=g).to(DEV)
    idx = torch.randint(0, 100, (37,), generator=g).to(DEV).int()
    got = ops.gather_rows(src, idx)
    assert torch.equal(got, src[idx.long()])
    srcb = src.bfloat16()
    assert torch.equal(ops.gather_rows(srcb, idx), srcb[idx.long()])
    perm = torch.randperm(100, generator=g).to(DEV).int()
    out = torch.zeros_like(src)
    ops.scatter_rows(src, perm, out)
    exp = torch.zeros_like(src)
    exp[perm.long()] = src
    assert torch.equal(out, exp)
    vec = torch.randn(96, generator=g).to(DEV)
    ops.fill_rows(out, perm[:10], vec)
    exp[perm[:10].long()] = vec
    assert torch.equal(out, exp)


@pytest.mark.parametrize("case", ["sorted", "unsorted", "dups", "edge"])
def test_pred_index_matches_argsort(case):
    """Merge-path ranks (sorted masks, the collator's output) and the counting fallback (unsorted
    rows, ids repeated across masks_x / masks_y) both equal the reference's stable torch.argsort
    (predictor.py:210-217, 240-242)."""
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(3)
    B, N, K, Kp = 4, 2048, 513, 966
    if case == "edge":
        K, Kp = 1, 2047
    perms = [torch.randperm(N, generator=g) for _ in range(B)]
    mx = torch.stack([p[:K].sort().values for p in perms])
    my = torch.stack([p[K:K + Kp].sort().values for p in perms])
    if case == "unsorted":
        mx[1] = mx[1][torch.randperm(K, generator=g)]
        my[2] = my[2][torch.randperm(Kp, generator=g)]
    elif case == "dups":  # masks_y repeats some masks_x ids (still sorted): stability decides the order
        my = torch.stack([torch.cat([mx[b][:100], my[b][100:]]).sort().values for b in range(B)])
    n = K + Kp
    row0 = 17
    pos = torch.full((row0 + B * n,), -1, dtype=torch.int32, device=DEV)
    ctx = torch.empty(B * K, dtype=torch.int32, device=DEV)
    tgt = torch.empty(B * Kp, dtype=torch.int32, device=DEV)
    lrows = torch.empty(B * Kp, dtype=torch.int32, device=DEV)
    ops.pred_index(mx.to(DEV), my.to(DEV), row0, N, pos, ctx, tgt, lrows)
    m = torch.cat([mx, my], 1)
    order = torch.argsort(m, dim=1, stable=True)
    sorted_ids = torch.gather(m, 1, order)
    rev = torch.argsort(order, dim=1)
    base = (row0 + torch.arange(B) * n)[:, None]
    torch.cuda.synchronize()
    assert torch.equal(pos[row0:].cpu().long().reshape(B, n), sorted_ids)
    assert torch.equal(ctx.cpu().long().reshape(B, K), base + rev[:, :K])
    assert torch.equal(tgt.cpu().long().reshape(B, Kp), base + rev[:, K:])
    assert torch.equal(lrows.cpu().long().reshape(B, Kp), torch.arange(B)[:, None] * N + my)


# ------------------------------------------------------------------------------------------------
def test_jepa_loss():
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(4)
    B, N, D = 3, 40, 128
    h_res = torch.randn(B * N, D, generator=g)
    gamma = 1 + 0.1 * torch.randn(D, generator=g)
    beta = 0.1 * torch.randn(D, generator=g)
    masks = [torch.stack([torch.randperm(N, generator=g)[:k].sort().values for _ in range(B)]) for k in (7, 11)]
    rows = torch.cat([(torch.arange(B)[:, None] * N + m).reshape(-1) for m in masks]).int()
    z = torch.randn(rows.numel(), D, generator=g)
    loss, dz, _ = ops.jepa_loss(z.to(DEV), h_res.to(DEV), rows.to(DEV), gamma.to(DEV), beta.to(DEV),
                                [B * 7, B * 11])
    h = torch.nn.functional.layer_norm(h_res, (D,), gamma, beta, 1e-6)
    h = torch.nn.functional.layer_norm(h, (D,)).reshape(B, N, D)
    zr = z.clone().requires_grad_(True)
    zl = [zr[:B * 7].reshape(B, 7, D), zr[B * 7:].reshape(B, 11, D)]
    ref = orc.jepa_loss(zl, h, masks)
    ref.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, ref.item())
    _close(dz, zr.grad, 1e-9, 8e-3, "loss dz")


def test_adamw_ema_match_oracle():
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(6)
    n = 4096
    p = torch.randn(n, generator=g)
    gr = torch.randn(n, generator=g)
    m = 0.1 * torch.randn(n, generator=g)
    v = torch.rand(n, generator=g)
    pd, gd, md, vd = (t.clone().to(DEV) for t in (p, gr, m, v))
    pbf = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    for step in (1, 2, 3):
        ops.adamw(pd, gd, md, vd, pbf, 5e-4, 0.9, 0.999, 1e-8, 0.04, step)
        orc.adamw_step(p, gr, m, v, step, 5e-4, 0.04)
    torch.cuda.synchronize()
    # fp32 elementwise math; the device may contract a*b+c into one fma (1-2 ulp)
    _close(pd, p, 1e-7, 2e-6, "adamw p")
    _close(md, m, 1e-7, 2e-6, "adamw m")
    _close(vd, v, 1e-7, 4e-6, "adamw v")
    assert torch.equal(pbf, pd.bfloat16())
    # found_inf skip
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    gd[5] = float("inf")
    ops.check_finite(gd, flag)
    before = pd.clone()
    ops.adamw(pd, gd, md, vd, pbf, 5e-4, 0.9, 0.999, 1e-8, 0.04, 4, found_inf=flag)
    torch.cuda.synchronize()
    assert flag.item() == 1 and torch.equal(pd, before)
    t = torch.randn(n, generator=g)
    e = torch.randn(n, generator=g)
    td = t.to(DEV)
    tbf = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    ops.ema(td, e.to(DEV), 0.99925, tbf)
    orc.ema_update(t, e, 0.99925)
    torch.cuda.synchronize()
    _close(td, t, 1e-7, 1e-6, "ema")
    assert torch.equal(tbf, td.bfloat16())


@pytest.mark.parametrize("skip", [False, True])
def test_adamw_ema_fused_equals_separate(skip):
    """vj_adamw_ema (the EMA fused into the encoder arena's AdamW pass) == vj_adamw then vj_ema,
    bitwise, including a step skipped by found_inf (parameters unchanged, the EMA still applied)."""
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(16)
    n = 8192
    base = [torch.randn(n, generator=g), torch.randn(n, generator=g), 0.1 * torch.randn(n, generator=g),
            torch.rand(n, generator=g), torch.randn(n, generator=g)]
    flag = torch.tensor([1 if skip else 0], dtype=torch.int32, device=DEV)
    outs = []
    for fused in (True, False):
        p, gr, m, v, t = (x.clone().to(DEV) for x in base)
        pbf = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        tbf = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        if fused:
            ops.adamw_ema(p, gr, m, v, pbf, 5e-4, 0.9, 0.999, 1e-8, 0.04, 3, t, tbf, 0.99925, grad_scale=0.5,
                          found_inf=flag)
        else:
            ops.adamw(p, gr, m, v, pbf, 5e-4, 0.9, 0.999, 1e-8, 0.04, 3, grad_scale=0.5, found_inf=flag)
            ops.ema(t, p, 0.99925, tbf)
        torch.cuda.synchronize()
        outs.append((p, m, v, t, tbf))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    if skip:
        assert torch.equal(outs[0][0].cpu(), base[0])


@pytest.mark.parametrize("K", [64, 192, 256, 1024])
@pytest.mark.parametrize("pxcd", [None, "1", "3"])
def test_gemm_256_tiles_vs_fp32(K, pxcd, monkeypatch):
    """The 256 x 256-tile kernel (one-tile main loop: VJ_GEMM_STG=0, 256-row tiles) on every epilogue
    against fp32 math: K = 64 / 192 / 256 make 1 / 3 / 4 K-tiles (tail paths), VJ_GEMM_PXCD = 1 / 3
    many tiles per block (the next tile's stages DMA'd under the epilogue), M = 2100 / 1333 ragged
    last row tiles and N = 1000 a ragged last column tile."""
    from vjepa2_amd import ops

    if pxcd:
        monkeypatch.setenv("VJ_GEMM_PXCD", pxcd)
    monkeypatch.setenv("VJ_GEMM_BM192", "0")
    monkeypatch.setenv("VJ_GEMM_STG", "0")
    g = torch.Generator(device="cpu").manual_seed(K)
    for M, N in [(2100, 512), (1333, 1000)]:
        X = torch.randn(M, K, generator=g).to(DEV).bfloat16()
        W = (0.1 * torch.randn(N, K, generator=g)).to(DEV).bfloat16()
        b = torch.randn(N, generator=g).to(DEV)
        resid = torch.randn(M, N, generator=g).to(DEV)
        dgs = torch.randn(M, N, generator=g).to(DEV).bfloat16()
        ref = X.float() @ W.float().t() + b
        outs = {"bf16": ops.linear_fwd(X, W, b, ops.EPI_BF16),
                "f32": ops.linear_fwd(X, W, b, ops.EPI_F32),
                "f32_resid": ops.linear_fwd(X, W, b, ops.EPI_F32_RESID, resid=resid)}
        gb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.gemm(M, N, K, X, K, True, W, K, True, ops.EPI_GELU_BWD, out=gb, ldc=N, aux=dgs, ldaux=N)
        d, a = ops.linear_fwd(X, W, b, ops.EPI_GELU, out=torch.empty(M, N, device=DEV, dtype=torch.bfloat16))
        nosave = ops.linear_fwd(X, W, b, ops.EPI_GELU)[1]
        torch.cuda.synchronize()
        assert torch.equal(a, nosave)
        _close(outs["f32"], ref, 1e-4 * math.sqrt(K) * 4, 1e-4, "EPI_F32 vs fp32")
        _close(outs["f32_resid"], ref + resid, 1e-4 * math.sqrt(K) * 4, 1e-4, "EPI_F32_RESID vs fp32")
        _close(outs["bf16"], ref, 1e-3, 8e-3, "EPI_BF16 vs fp32")
        _close(gb, (X.float() @ W.float().t()) * dgs.float(), 2e-3, 1.5e-2, "EPI_GELU_BWD")
        pre = outs["bf16"].float()
        _close(a, torch.nn.functional.gelu(pre), 2e-3, 1.5e-2, "EPI_GELU vs gelu(bf16 pre-activation)")


@pytest.mark.parametrize("K", [32, 64, 96, 128, 192, 384, 1024])
@pytest.mark.parametrize("pxcd", [None, "1", "3"])
@pytest.mark.parametrize("form", ["1", "2"])
def test_gemm_staggered_matches_one_tile(K, pxcd, form, monkeypatch):
    """The staggered main loops (VJ_GEMM_STG=1) run the same MFMAs on every accumulator in the same K
    order as the one-tile kernel, so every epilogue's output is bitwise equal. Form 1 (VJ_GEMM_STG64=0):
    32-deep K units in a 4/5-slot LDS ring, one stream of units across the block's tiles, waves 4-7 one
    barrier behind waves 0-3; K = 32 / 64 / 96 make 1 / 2 / 3 units per tile (the DMA stream runs 2-3
    units, i.e. up to 3 tiles, ahead). Form 2 (S64, VJ_GEMM_STG64=1, K % 64 == 0; form 1 otherwise):
    64-deep steps of 128-row granules, A and B streamed by the two wave halves 3 granules ahead; K = 64 /
    128 / 192 make 1 / 2 / 3 steps per tile (the streams run up to 3 tiles ahead, where a wave half's
    stream crosses tiles at a different point than the other's). VJ_GEMM_PXCD = 1 / 3 give many tiles
    per block (epilogue / tile hand-over paths of both wave halves), M = 2100 / 1333 ragged last row
    tiles (S64: a tile whose A1 granule is empty), N = 1000 a ragged last column tile; plus the fused
    QKV + RoPE epilogue."""
    from vjepa2_amd import ops

    if pxcd:
        monkeypatch.setenv("VJ_GEMM_PXCD", pxcd)
    monkeypatch.setenv("VJ_GEMM_BM192", "0")  # 256-row tiles for both
    monkeypatch.setenv("VJ_GEMM_STG64", "1" if form == "2" else "0")
    g = torch.Generator(device="cpu").manual_seed(K + 7)
    for M, N in [(2100, 512), (1333, 1000)]:
        X = torch.randn(M, K, generator=g).to(DEV).bfloat16()
        W = (0.1 * torch.randn(N, K, generator=g)).to(DEV).bfloat16()
        b = torch.randn(N, generator=g).to(DEV)
        resid = torch.randn(M, N, generator=g).to(DEV)
        dgs = torch.randn(M, N, generator=g).to(DEV).bfloat16()

        def run():
            outs = {"bf16": ops.linear_fwd(X, W, b, ops.EPI_BF16),
                    "f32": ops.linear_fwd(X, W, b, ops.EPI_F32),
                    "f32_resid": ops.linear_fwd(X, W, b, ops.EPI_F32_RESID, resid=resid),
                    "bf16_resid": ops.linear_fwd(X, W, b, ops.EPI_BF16_RESID, resid=resid.bfloat16())}
            d, a = ops.linear_fwd(X, W, b, ops.EPI_GELU, out=torch.empty(M, N, device=DEV, dtype=torch.bfloat16))
            outs["gelu_d"], outs["gelu_a"] = d, a
            outs["gelu_nosave"] = ops.linear_fwd(X, W, b, ops.EPI_GELU)[1]
            gb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(M, N, K, X, K, True, W, K, True, ops.EPI_GELU_BWD, out=gb, ldc=N, aux=dgs, ldaux=N)
            outs["gelu_bwd"] = gb
            torch.cuda.synchronize()
            return {k: v.detach().clone() for k, v in outs.items()}

        monkeypatch.setenv("VJ_GEMM_STG", "0")
        one = run()
        monkeypatch.setenv("VJ_GEMM_STG", "1")
        stg = run()
        for k in one:
            assert torch.equal(stg[k], one[k]), f"staggered {k} != one-tile kernel (M={M} N={N} K={K} pxcd={pxcd})"
    # QKV GEMM with the fused RoPE epilogue (N = 3 * 4 * 64 = 768: 256-wide tiles)
    H, hd, M = 4, 64, 2100
    ids = torch.randint(0, 8 * 16, (M,), generator=g).to(DEV).int()
    cos_t, sin_t = (t.to(DEV) for t in orc.rope_tables(hd, 16))
    x = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    w = (0.1 * torch.randn(3 * H * hd, K, generator=g)).to(DEV).bfloat16()
    bq = torch.randn(3 * H * hd, generator=g).to(DEV)
    res = []
    for stg in ("0", "1"):
        monkeypatch.setenv("VJ_GEMM_STG", stg)
        res.append(ops.qkv_rope(x, w, bq, H, hd, ids, 0, 16, 4, cos_t, sin_t).clone())
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]), f"staggered qkv_rope != one-tile kernel (K={K} pxcd={pxcd})"


@pytest.mark.parametrize("stg", ["1", "0", "2"])
def test_gelu_epilogues_bitwise_all_bf16(stg, monkeypatch):
    """The fc1 GEMM's GELU epilogues against the exact evaluation (vj_gelu_eval: gelu_fwd_grad on the
    bf16 input) on EVERY bf16 pre-activation: X = 0 and the bias holds the 65536 bf16 values, so
    pre = bf16(0 + bias[n]) runs through the whole bit space. VJ_GEMM_STG=1: the staggered kernel's
    LDS-table epilogue (GELU and GELU' looked up by the 16 input bits); 0: the one-tile kernel's direct
    evaluation. Bitwise on every non-NaN input (the -0 pattern enters as +0: 0 + -0 = +0), NaN -> NaN."""
    from vjepa2_amd import ops

    monkeypatch.setenv("VJ_GEMM_STG", "1" if stg == "2" else stg)  # "2": the S64 form (K = 64)
    monkeypatch.setenv("VJ_GEMM_STG64", "1" if stg == "2" else "0")
    monkeypatch.setenv("VJ_GEMM_BM192", "0")
    n = 65536
    bits = torch.arange(n, dtype=torch.int32)
    bits = torch.where(bits >= 32768, bits - 65536, bits).to(torch.int16)
    xb = bits.view(torch.bfloat16)
    bias = xb.float().to(DEV)
    pre = bits.clone()
    pre[pre == -32768] = 0  # 0 + (-0) = +0
    y_ref, dy_ref = ops.gelu_eval(pre.view(torch.bfloat16).to(DEV).contiguous())
    M, K = 1024, (64 if stg == "2" else 32)
    X = torch.zeros(M, K, device=DEV, dtype=torch.bfloat16)
    W = torch.zeros(n, K, device=DEV, dtype=torch.bfloat16)
    d, a = ops.linear_fwd(X, W, bias, ops.EPI_GELU, out=torch.empty(M, n, device=DEV, dtype=torch.bfloat16))
    a_ns = ops.linear_fwd(X, W, bias, ops.EPI_GELU)[1]
    torch.cuda.synchronize()
    nan = torch.isnan(xb.float()).to(DEV)
    for name, got, ref in (("GELU", a, y_ref), ("GELU'", d, dy_ref), ("GELU (no save)", a_ns, y_ref)):
        gi = got.view(torch.int16)
        ri = ref.view(torch.int16)[None, :].expand(M, n)
        bad = (gi != ri) & ~nan[None, :]
        assert not bool(bad.any()), (
            f"{name} (STG={stg}): {int(bad.sum())} mismatches, e.g. input bits "
            f"{[hex(int(v) & 0xffff) for v in bits[bad[0].cpu()][:8]]}")
        assert bool(torch.isnan(got.float()[:, nan]).all()), f"{name}: NaN input must give NaN"


@pytest.mark.parametrize("K", [64, 128, 1024])
@pytest.mark.parametrize("pxcd", [None, "1"])
def test_gemm_192_row_tiles_match_256(K, pxcd, monkeypatch):
    """192-row tiles (k_gemm256<..., 192>: 3 m-tiles per wave M-half, chosen by the host cost model
    for context-sized M) against the 256-row kernel on every direct-store epilogue: each output's K
    order is the same sequence of MFMAs, so the outputs are BITWISE equal. M = 2100 / 1333 leave a
    ragged last 192-row tile (and 256-row tile), K = 64 / 128 one / two K-tiles per tile,
    VJ_GEMM_PXCD = 1 many tiles per block (the next tile's stages DMA'd under the epilogue)."""
    from vjepa2_amd import ops

    if pxcd:
        monkeypatch.setenv("VJ_GEMM_PXCD", pxcd)
    g = torch.Generator(device="cpu").manual_seed(K + 192)
    for M, N in [(2100, 512), (1333, 1024)]:
        X = torch.randn(M, K, generator=g).to(DEV).bfloat16()
        W = (0.1 * torch.randn(N, K, generator=g)).to(DEV).bfloat16()
        b = torch.randn(N, generator=g).to(DEV)
        resid = torch.randn(M, N, generator=g).to(DEV)
        dgs = torch.randn(M, N, generator=g).to(DEV).bfloat16()

        def run():
            outs = {"bf16": ops.linear_fwd(X, W, b, ops.EPI_BF16),
                    "f32": ops.linear_fwd(X, W, b, ops.EPI_F32),
                    "f32_resid": ops.linear_fwd(X, W, b, ops.EPI_F32_RESID, resid=resid),
                    "bf16_resid": ops.linear_fwd(X, W, b, ops.EPI_BF16_RESID, resid=resid.bfloat16())}
            d, a = ops.linear_fwd(X, W, b, ops.EPI_GELU, out=torch.empty(M, N, device=DEV, dtype=torch.bfloat16))
            outs["gelu_d"], outs["gelu_a"] = d, a
            outs["gelu_nosave"] = ops.linear_fwd(X, W, b, ops.EPI_GELU)[1]
            gb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(M, N, K, X, K, True, W, K, True, ops.EPI_GELU_BWD, out=gb, ldc=N, aux=dgs, ldaux=N)
            outs["gelu_bwd"] = gb
            torch.cuda.synchronize()
            return {k: v.detach().clone() for k, v in outs.items()}

        monkeypatch.setenv("VJ_GEMM_BM192", "1")
        t192 = run()
        monkeypatch.setenv("VJ_GEMM_BM192", "0")
        t256 = run()
        monkeypatch.delenv("VJ_GEMM_BM192")
        for k in t192:
            assert torch.equal(t192[k], t256[k]), f"192-row != 256-row tiles: {k} M={M} N={N} K={K} pxcd={pxcd}"
        ref = X.float() @ W.float().t() + b
        _close(t192["f32"], ref, 1e-4 * math.sqrt(K) * 4, 1e-4, "192-row EPI_F32")
        assert torch.equal(t192["gelu_a"], t192["gelu_nosave"])


@pytest.mark.parametrize("K", [32, 96, 384])
def test_gemm_2w_192x128_tiles_match_256x128(K, monkeypatch):
    """The two-workgroup kernel on 192 x 128 tiles 64 deep (VJ_GEMM_2W192=1: whole 128-B rows per
    DMA piece) against its 256 x 128, 32-deep form on the 128-wide shapes it serves (N = 384 / 640):
    each output's k-steps run in the same order, so every epilogue is BITWISE equal. K = 32 / 96 end
    in a half-empty 64-deep K-tile (zero-filled), M = 2100 / 1333 in ragged row tiles."""
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(K + 2)
    for M, N in [(2100, 384), (1333, 640)]:
        X = torch.randn(M, K, generator=g).to(DEV).bfloat16()
        W = (0.1 * torch.randn(N, K, generator=g)).to(DEV).bfloat16()
        b = torch.randn(N, generator=g).to(DEV)
        resid = torch.randn(M, N, generator=g).to(DEV)
        dgs = torch.randn(M, N, generator=g).to(DEV).bfloat16()

        def run():
            outs = {"bf16": ops.linear_fwd(X, W, b, ops.EPI_BF16),
                    "f32": ops.linear_fwd(X, W, b, ops.EPI_F32),
                    "f32_resid": ops.linear_fwd(X, W, b, ops.EPI_F32_RESID, resid=resid),
                    "bf16_resid": ops.linear_fwd(X, W, b, ops.EPI_BF16_RESID, resid=resid.bfloat16())}
            d, a = ops.linear_fwd(X, W, b, ops.EPI_GELU, out=torch.empty(M, N, device=DEV, dtype=torch.bfloat16))
            outs["gelu_d"], outs["gelu_a"] = d, a
            gb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(M, N, K, X, K, True, W, K, True, ops.EPI_GELU_BWD, out=gb, ldc=N, aux=dgs, ldaux=N)
            outs["gelu_bwd"] = gb
            torch.cuda.synchronize()
            return {k: v.detach().clone() for k, v in outs.items()}

        monkeypatch.setenv("VJ_GEMM_2W192", "1")
        t192 = run()
        monkeypatch.setenv("VJ_GEMM_2W192", "0")
        t256 = run()
        monkeypatch.delenv("VJ_GEMM_2W192")
        for k in t192:
            assert torch.equal(t192[k], t256[k]), f"2W 192x128 != 256x128: {k} M={M} N={N} K={K}"
        ref = X.float() @ W.float().t() + b
        _close(t192["f32"], ref, 1e-4 * math.sqrt(K) * 4, 1e-4, "2W 192x128 EPI_F32")


def test_transpose_bf16_single_and_batched():
    """Register-tile transpose (8 x 8 blocks per lane, one 64 x 64 tile per wave) and its batched
    form (one launch over a descriptor table, as refresh_weight_transposes uses): bitwise x.t(), on
    shapes with ragged 64-tiles, row-strided sources and the ViT-L / predictor weight shapes."""
    from vjepa2_amd import ops

    g = torch.Generator(device="cpu").manual_seed(7)
    shapes = [(8, 8), (72, 136), (3072, 1024), (1024, 4096), (384, 1536), (1152, 384), (200, 64)]
    srcs = [torch.randn(r, c, generator=g).to(DEV).bfloat16() for r, c in shapes]
    big = torch.randn(96, 200, generator=g).to(DEV).bfloat16()
    srcs.append(big[:, 8:136])  # row stride 200 > cols
    for x in srcs:
        assert torch.equal(ops.transpose_bf16(x), x.t().contiguous()), tuple(x.shape)
    outs = [torch.full((x.shape[1], x.shape[0]), 7.0, device=DEV, dtype=torch.bfloat16) for x in srcs]
    desc, tiles = ops.transpose_batch_desc(list(zip(srcs, outs)))
    ops.transpose_bf16_batch(desc, len(srcs), tiles)
    torch.cuda.synchronize()
    for x, o in zip(srcs, outs):
        assert torch.equal(o, x.t().contiguous()), tuple(x.shape)


def test_refresh_weight_transposes_matches_lazy_copies():
    """After an arena update the batched refresh leaves every registered W^T equal to the transpose
    of the new bf16 shadow, and weight_bf16_t then returns it without a new launch."""
    from vjepa2_amd import functions as F

    lin = torch.nn.Linear(256, 384).to(DEV)
    w = lin.weight
    w._vj_bf16 = w.detach().bfloat16()
    first = F.weight_bf16_t(w)
    assert torch.equal(first, w._vj_bf16.t().contiguous())
    w._vj_bf16.copy_((w.detach() * 2).bfloat16())  # an "AdamW" update of the shadow
    F.SHADOW_EPOCH[0] += 1
    F.refresh_weight_transposes()
    torch.cuda.synchronize()
    assert w._vj_bf16_t[0][1] == F.SHADOW_EPOCH[0]
    assert torch.equal(w._vj_bf16_t[1], w._vj_bf16.t().contiguous())
    assert F.weight_bf16_t(w) is w._vj_bf16_t[1]


# ------------------------------------------------------------------------------------------------
# Block variants (vj_variants.hip): SwiGLU gate, drop_path row scaling. Expected values are the
# reference's own bf16 autocast ops (torch elementwise kernels on the same bf16 inputs).
@pytest.mark.parametrize("M,h", [(1, 8), (37, 344), (1000, 1368)])
def test_swiglu_gate_vs_torch_bf16(M, h):
    from vjepa2_amd import ops

    torch.manual_seed(M + h)
    x12 = (2.5 * torch.randn(M, 2 * h, device=DEV)).bfloat16()
    x1 = x12[:, :h].clone().requires_grad_(True)
    x2 = x12[:, h:].clone().requires_grad_(True)
    ref = torch.nn.functional.silu(x1) * x2  # SwiGLUFFN.forward, modules.py:103-105, bf16 tensors
    got = ops.swiglu_fwd(x12)
    # silu in f32 then bf16: the device expf may differ from torch's by an f32 ulp -> at most 1 bf16 ulp
    _close(got, ref, 0.0, 2.0**-7, "swiglu fwd")
    assert (got.float() == ref.detach().float()).float().mean().item() > 0.99
    dh = torch.randn(M, h, device=DEV).bfloat16()
    ref.backward(dh)
    dx12 = ops.swiglu_bwd(dh, x12)
    _close(dx12[:, :h], x1.grad, 1e-30, 2.0**-6, "swiglu dx1")
    _close(dx12[:, h:], x2.grad, 1e-30, 2.0**-7, "swiglu dx2")


@pytest.mark.parametrize("bf16_resid", [False, True])
def test_rowscale_kernels_exact(bf16_resid):
    """vj_rowscale_add / vj_rowscale_bf16 against the same bf16-rounded arithmetic in torch: bit-exact."""
    from vjepa2_amd import ops

    torch.manual_seed(3)
    M, N = 777, 136
    y = torch.randn(M, N, device=DEV)
    keep = 0.6
    s = (torch.rand(M, device=DEV) < keep).bfloat16().div_(keep).float()
    resid = torch.randn(M, N, device=DEV)
    resid = resid.bfloat16() if bf16_resid else resid
    got = ops.rowscale_add(y, s, resid)
    branch = (y.bfloat16() * s.bfloat16()[:, None]).float()  # bf16 * bf16 -> bf16 (f32 math, one rounding)
    exp = resid.float() + branch
    exp = exp.bfloat16() if bf16_resid else exp
    assert got.dtype == resid.dtype and torch.equal(got, exp)
    dx = torch.randn(M, N, device=DEV)
    assert torch.equal(ops.rowscale_bf16(dx, s), dx.bfloat16() * s.bfloat16()[:, None])


def test_drop_path_sample_distribution():
    """DropPath.sample: the reference's random_tensor values (0 or bf16(1 / keep)) at rate ~keep."""
    from vjepa2_amd.modules import DropPath

    torch.manual_seed(0)
    dp = DropPath(0.3)
    r = dp.sample(200000, DEV)
    vals = set(r.unique().tolist())
    assert vals == {0.0, torch.tensor(1 / 0.7).bfloat16().item()} or vals == {0.0, (torch.tensor(1.0).bfloat16() / 0.7).item()}
    assert abs((r > 0).float().mean().item() - 0.7) < 0.005
