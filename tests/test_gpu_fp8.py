"""GPU: the opt-in fp8 target-encoder path (BASELINE configs[4]: ViT-g/16 64x256^2 "fp8 MFMA path").
The reference has no fp8, so this path is judged by its error envelope:

 * the per-row scaled e4m3 quantiser and the fp8 LayerNorm produce exactly torch's e4m3 rounding of
   x * 2^-e, with e the least exponent that fits max|x| into +-448;
 * the fp8 GEMMs (v_mfma_scale_f32_16x16x128_f8f6f4 with the per-row exponents as E8M0 operands)
   equal fp32 math on the DEQUANTISED operands up to accumulation order, for every epilogue;
 * a 2-block ViT-g-width target encoder at 64x256^2 (N = 8192 tokens) on the fp8 path vs the fp32
   oracle stays inside the stated envelope (rel L1 < 5e-2; measured values are printed).
"""

import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vjepa_oracle as orc  # noqa: E402

DEV = "cuda"


def _ref_quant(x):
    """torch e4m3fn rounding of x * 2^-e per row, e = least exponent with amax * 2^-e <= 448."""
    x = x.float()
    am = x.abs().amax(1)
    e = torch.zeros_like(am, dtype=torch.int32)
    nz = am > 0
    e[nz] = torch.ceil(torch.log2(am[nz] / 448.0)).int()
    e = torch.where(nz & (torch.ldexp(am, -e) > 448.0), e + 1, e)
    e = torch.where(nz & (torch.ldexp(am, -(e - 1)) <= 448.0), e - 1, e)
    q = torch.ldexp(x, -e[:, None].float()).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), e


def _deq(q8, e):
    return torch.ldexp(q8.cpu().view(torch.float8_e4m3fn).float(), e.cpu()[:, None].float())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_quant_rows_fp8_exact(dtype):
    from vjepa2_amd import ops

    g = torch.Generator().manual_seed(1)
    x = torch.randn(67, 1408, generator=g)
    x[3] *= 1e-3
    x[5] *= 1e3
    x[7] = 0.0
    x[9, 17] = 448.0 * 4  # an exact power-of-two boundary
    x = x.to(dtype)
    q, e = ops.quant_rows_fp8(x.to(DEV))
    qr, er = _ref_quant(x)
    torch.cuda.synchronize()
    assert torch.equal(e.cpu(), er), (e.cpu()[:12], er[:12])
    assert torch.equal(q.cpu(), qr)


@pytest.mark.parametrize("D", [384, 1408])
def test_layernorm_fwd_fp8(D):
    from vjepa2_amd import ops

    g = torch.Generator().manual_seed(D)
    x = (2 * torch.randn(301, D, generator=g) + 0.5)
    w = 1 + 0.1 * torch.randn(D, generator=g)
    b = 0.1 * torch.randn(D, generator=g)
    q, e = ops.layernorm_fwd_fp8(x.to(DEV), w.to(DEV), b.to(DEV), 1e-6)
    y = torch.nn.functional.layer_norm(x, (D,), w, b, 1e-6)
    qr, er = _ref_quant(y)
    torch.cuda.synchronize()
    assert torch.equal(e.cpu(), er)
    diff = (q.cpu().int() - qr.int()).abs()
    # LayerNorm in a different fp32 op order: an element may land on the other side of a rounding tie
    assert int(diff.max()) <= 1 and float((diff > 0).float().mean()) < 1e-3


@pytest.mark.parametrize("M,N,K", [(1100, 384, 1408), (2048, 1152, 208), (300, 520, 1024)])
def test_fp8_gemm_matches_dequantized(M, N, K):
    from vjepa2_amd import ops

    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g) * torch.exp(torch.randn(M, 1, generator=g))  # per-row magnitudes
    w = 0.05 * torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    a8, ea = ops.quant_rows_fp8(a.to(DEV))
    w8, ew = ops.quant_rows_fp8(w.to(DEV))
    ad, wd = _deq(a8, ea).double(), _deq(w8, ew).double()
    exp = (ad @ wd.t() + bias.double()).float()
    # products of e4m3 values are exact in fp32; only the summation differs. The scaled MFMA sums its
    # 128 products per lane-block in hardware order (not IEEE sequential: measured up to ~1.5e-5 of
    # sum|a w| at K = 208, above gamma_K there), so the bound is 2^-14 * sum_k |a_k w_k| -- ten bits
    # below the e4m3 input rounding (2^-4) that the envelope test prices.
    REL = 2.0 ** -14
    bound = REL * ((ad.abs() @ wd.abs().t()).float() + bias.abs())
    y = ops.linear_fwd_fp8(a8, ea, w8, ew, bias.to(DEV), ops.EPI_F32)
    torch.cuda.synchronize()
    err = (y.cpu() - exp).abs()
    print(f"fp8 GEMM {M}x{N}x{K}: max |err| / sum|a w| = {(err / (bound / REL)).max().item():.2e}")
    assert (err <= bound).all(), (err.max().item(), bound.min().item())
    resid = torch.randn(M, N, generator=g)
    y = ops.linear_fwd_fp8(a8, ea, w8, ew, bias.to(DEV), ops.EPI_F32_RESID, resid=resid.to(DEV))
    assert ((y.cpu() - (exp + resid)).abs() <= bound + 2.0 ** -23 * (exp.abs() + resid.abs())).all()
    yb = ops.linear_fwd_fp8(a8, ea, w8, ew, bias.to(DEV), ops.EPI_BF16)
    assert (yb.cpu().float() - exp).abs().max().item() <= 2 ** -7 * exp.abs().max().item()
    pre = ops.linear_fwd_fp8(a8, ea, w8, ew, bias.to(DEV), ops.EPI_BF16)  # the bf16 pre-activation
    dg = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    _, act = ops.linear_fwd_fp8(a8, ea, w8, ew, bias.to(DEV), ops.EPI_GELU, out=dg)
    torch.cuda.synchronize()
    xp = pre.cpu().float().requires_grad_(True)
    ga = torch.nn.functional.gelu(xp)
    ga.sum().backward()
    assert (act.cpu().float() - ga.detach()).abs().max().item() <= 2 ** -7 * ga.abs().max().item() + 1e-3
    assert (dg.cpu().float() - xp.grad).abs().max().item() <= 2 ** -7 * 1.2 + 1e-3


def test_fp8_qkv_rope_matches_dequantized():
    from vjepa2_amd import ops

    g = torch.Generator().manual_seed(5)
    M, H, hd, K = 1500, 2, 64, 256
    D = H * hd
    tpf, tpr = 16, 4
    ids = torch.randint(0, 8 * 16, (M,), generator=g)
    cos_t, sin_t = orc.rope_tables(hd, 16)
    a8, ea = ops.quant_rows_fp8(torch.randn(M, K, generator=g).to(DEV))
    w8, ew = ops.quant_rows_fp8((0.1 * torch.randn(3 * D, K, generator=g)).to(DEV))
    b = torch.randn(3 * D, generator=g)
    got = ops.qkv_rope_fp8(a8, ea, w8, ew, b.to(DEV), H, hd, ids.to(DEV).int(), 0, tpf, tpr, cos_t.to(DEV),
                           sin_t.to(DEV))
    y = (_deq(a8, ea).double() @ _deq(w8, ew).double().t() + b.double()).float()
    q = y[:, :D].reshape(M, H, hd).transpose(0, 1)[None]
    k = y[:, D:2 * D].reshape(M, H, hd).transpose(0, 1)[None]
    qr, kr = orc.apply_rope_qk(q, k, ids[None], tpf, tpr)
    exp = torch.cat([qr[0].transpose(0, 1).reshape(M, D), kr[0].transpose(0, 1).reshape(M, D), y[:, 2 * D:]], 1)
    torch.cuda.synchronize()
    err = (got.cpu().float() - exp).abs()
    assert (err <= 2 ** -7 * exp.abs() + 1e-3).all(), err.max()


def _rel_l1(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().mean() / b.abs().mean()).item()


def test_vitg_fp8_target_envelope():
    """ViT-g/16 width (vit_giant_xformers: D 1408, 22 heads, MLP 6144), 2 blocks, the 64x256^2 clip of
    configs/train/vitg16/cooldown-256px-64f.yaml as the TARGET encoder sees it (all 8192 tokens, no
    grad): fp8 forward_features vs the fp32 oracle, next to the bf16 path's error."""
    from vjepa2_amd.vision_transformer import VisionTransformer, _ln

    torch.manual_seed(13)
    enc = VisionTransformer(img_size=256, num_frames=64, tubelet_size=2, patch_size=16, embed_dim=1408, depth=2,
                            num_heads=22, mlp_ratio=48 / 11, qkv_bias=True, norm_layer=_ln(), use_rope=True,
                            uniform_power=True)
    sd = {k: v.detach().clone() for k, v in enc.state_dict().items()}
    enc = enc.to(DEV)
    x = torch.randn(1, 3, 64, 256, 256)
    with torch.no_grad():
        h8 = enc.forward_features(x.to(DEV), fp8=True).cpu()
        hb = enc.forward_features(x.to(DEV), fp8=False).cpu()
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    with torch.no_grad():
        ref = orc.encoder_forward(x, sd, dict(patch_size=16, tubelet_size=2, num_heads=22, depth=2, use_rope=True),
                                  final_norm=False).reshape(-1, 1408)
    e8, eb = _rel_l1(h8, ref), _rel_l1(hb, ref)
    print(f"ViT-g 64x256^2 target forward (2 blocks): rel_l1 fp8 {e8:.3e}, bf16 {eb:.3e}")
    assert torch.isfinite(h8).all()
    assert e8 < 5e-2 and eb < 1e-2
