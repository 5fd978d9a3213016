"""GPU parity of the frozen-encoder probe: the cross-attention kernel (vj_xattn)
against fp32 SDPA autograd on the same bf16 operands, and AttentiveClassifier / AttentivePooler
(src/models/attentive_pooler.py, modules.py:566-610) against the REFERENCE's outputs and gradients
(tests/golden/pooler.pt, written by tests/golden/make_golden.py running the reference on CPU, fp32).

Tolerances: the kernel keeps every product and sum in fp32 and rounds only O / dQ / dK / dV to bf16,
so its outputs are within bf16 rounding (2^-8 relative) of fp32 math on the same operands; the module
tests compare a bf16-operand path with the fp32 reference (relative L1, bounds per tensor below).
"""

import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def rel_l1(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().mean() / b.abs().mean().clamp_min(1e-12)).item()


def _sdpa_ref(q, kv, B, nq, N, H, hd):
    """fp32 SDPA on the bf16 operands (modules.py:579-594 layout)."""
    qh = q.float().reshape(B, nq, H, hd).permute(0, 2, 1, 3)
    kvh = kv.float().reshape(B, N, 2, H, hd).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(qh, kvh[0], kvh[1])
    return o.transpose(1, 2).reshape(B * nq, H * hd)


@pytest.mark.parametrize("B,nq,N,H,hd", [(3, 1, 2048, 16, 64), (2, 3, 1000, 16, 88), (2, 16, 77, 12, 32),
                                         (2, 20, 300, 4, 64), (1, 1, 8192, 16, 64), (2, 2, 129, 2, 128),
                                         (1, 16, 300, 2, 128), (1, 40, 130, 2, 120)])  # > 64 KB of LDS
def test_xattn_fwd_vs_fp32(B, nq, N, H, hd):
    from vjepa2_amd import ops

    g = torch.Generator(device=DEV).manual_seed(B * 1000 + N)
    D = H * hd
    q = torch.randn(B * nq, D, device=DEV, generator=g).to(torch.bfloat16)
    kv = (2 * torch.randn(B * N, 2 * D, device=DEV, generator=g)).to(torch.bfloat16)
    o, lse2 = ops.xattn_fwd(q, kv, B, nq, N, H, hd, hd**-0.5)
    ref = _sdpa_ref(q, kv, B, nq, N, H, hd)
    err = (o.float() - ref).abs().max().item()
    assert err <= 2**-8 * ref.abs().max().item() + 1e-4, err
    # lse2: log2-domain log-sum-exp of the scaled scores
    s = torch.einsum("bqhd,bkhd->bhqk", q.float().reshape(B, nq, H, hd), kv.float().reshape(B, N, 2, H, hd)[:, :, 0])
    lse_ref = torch.logsumexp(s * hd**-0.5, -1).reshape(B * H, nq) / torch.log(torch.tensor(2.0))
    assert (lse2 - lse_ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("B,nq,N,H,hd", [(3, 1, 2048, 16, 64), (2, 3, 1000, 16, 88), (2, 16, 77, 12, 32),
                                         (2, 3, 4600, 16, 80), (2, 37, 300, 4, 64), (1, 16, 300, 2, 128),
                                         (1, 40, 130, 2, 120)])
def test_xattn_bwd_vs_fp32(B, nq, N, H, hd):
    from vjepa2_amd import ops

    g = torch.Generator(device=DEV).manual_seed(7 * N + nq)
    D = H * hd
    q = torch.randn(B * nq, D, device=DEV, generator=g).to(torch.bfloat16)
    kv = (2 * torch.randn(B * N, 2 * D, device=DEV, generator=g)).to(torch.bfloat16)
    do = torch.randn(B * nq, D, device=DEV, generator=g).to(torch.bfloat16)
    o, lse2 = ops.xattn_fwd(q, kv, B, nq, N, H, hd, hd**-0.5)
    dq, dkv = ops.xattn_bwd(q, kv, o, do, lse2, B, nq, N, H, hd, hd**-0.5)
    qf = q.float().requires_grad_(True)
    kvf = kv.float().requires_grad_(True)
    _sdpa_ref(qf, kvf, B, nq, N, H, hd).backward(do.float())
    for name, got, exp in (("dq", dq, qf.grad), ("dk", dkv[:, :D], kvf.grad[:, :D]), ("dv", dkv[:, D:], kvf.grad[:, D:])):
        e = rel_l1(got, exp)
        assert e < 1e-2, f"{name}: rel_l1 {e:.2e}"
    # deterministic: a second run is bitwise identical
    dq2, dkv2 = ops.xattn_bwd(q, kv, o, do, lse2, B, nq, N, H, hd, hd**-0.5)
    assert torch.equal(dq, dq2) and torch.equal(dkv, dkv2)


@pytest.mark.parametrize("which", ["clf", "pool3"])
def test_pooler_matches_reference(which):
    """attentive_pooler.py:91-137 on the HIP path vs the reference's fp32 outputs and every gradient."""
    from vjepa2_amd.attentive_pooler import AttentiveClassifier, AttentivePooler

    g = torch.load(os.path.join(GOLD, "pooler.pt"), weights_only=True)[which]
    m = (AttentiveClassifier if which == "clf" else AttentivePooler)(**g["cfg"]).to(DEV)
    m.load_state_dict(g["state"])
    x = g["x"].to(DEV).requires_grad_(True)
    y = m(x)
    assert y.shape == g["y"].shape and y.dtype == torch.float32
    y.backward(g["gy"].to(DEV))
    rep = [f"y: {rel_l1(y, g['y']):.2e}", f"dx: {rel_l1(x.grad, g['gx']):.2e}"]
    assert rel_l1(y, g["y"]) < 1e-2, rep
    assert rel_l1(x.grad, g["gx"]) < 3e-2, rep
    for n, p in m.named_parameters():
        e = rel_l1(p.grad, g["gparams"][n])
        rep.append(f"d{n}: {e:.2e}")
        assert e < 4e-2, "\n".join(rep)
    print("\n".join(rep))


def test_pooler_vitl_width_vs_oracle():
    """ViT-L width probe as the evals configure it (configs/eval/vitl/*.yaml: 16 heads, 4 probe blocks)
    over one 16x256^2 clip's 2048 tokens, B=4, forward vs the CPU oracle."""
    from oracle import vjepa_oracle as orc
    from vjepa2_amd.attentive_pooler import AttentiveClassifier

    torch.manual_seed(0)
    m = AttentiveClassifier(embed_dim=1024, num_heads=16, depth=4, num_classes=174)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(4, 2048, 1024)
    with torch.no_grad():
        ref = orc.attentive_classifier(x, sd, 16, 4)
        got = m.to(DEV)(x.to(DEV))
    e = rel_l1(got, ref)
    assert e < 2e-2, e


def test_multiclip_matches_reference():
    """ClipAggregation (vit_encoder_multiclip.py:87-162) around the HIP encoder vs the reference's
    outputs (tests/golden/multiclip.pt); the temporal table equals the reference's bit for bit."""
    import torch.nn as nn

    from vjepa2_amd import vision_transformer as vit
    from vjepa2_amd.multiclip import ClipAggregation

    g = torch.load(os.path.join(GOLD, "multiclip.pt"), weights_only=True)
    enc = vit.VisionTransformer(img_size=32, patch_size=16, num_frames=4, tubelet_size=2, embed_dim=64, depth=2,
                                num_heads=1, mlp_ratio=4, qkv_bias=True, use_rope=True, uniform_power=True,
                                norm_layer=lambda d: nn.LayerNorm(d, eps=1e-6))
    enc.load_state_dict(g["state"])
    agg = ClipAggregation(enc.to(DEV), tubelet_size=2, max_frames=16, use_pos_embed=True).to(DEV)
    assert torch.equal(agg.pos_embed.cpu(), g["pos_embed"])
    x = [[v.to(DEV) for v in views] for views in g["x"]]
    with torch.no_grad():
        outs = agg(x, clip_indices=[c.to(DEV) for c in g["clip_indices"]])
    assert len(outs) == len(g["outs"])
    for o, e in zip(outs, g["outs"]):
        assert o.shape == e.shape
        assert rel_l1(o, e) < 1e-2, rel_l1(o, e)
