"""GPU parity of the V-JEPA 2-AC action-conditioned predictor: the frame-causal
attention kernels (vj_attn_fwd_fc / vj_attn_bwd_fc) against fp32 SDPA with the reference's
block-causal attn_mask on the same bf16 operands, and VisionTransformerPredictorAC against the
REFERENCE's outputs and gradients (tests/golden/ac_predictor.pt, make_golden.py) and the CPU oracle at
the 256^2 frame geometry (16x16 patches + 2 action / state tokens per frame).
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


def _ref_attn(qkv, H, hd, groups, fblk):
    """fp32 SDPA per sequence with the frame-causal mask (modules.py:12-23 structure)."""
    D = H * hd
    outs, t0 = [], 0
    for n, L in groups:
        x = qkv[t0:t0 + n * L].float().reshape(n, L, 3, H, hd).permute(2, 0, 3, 1, 4)
        f = torch.arange(L, device=qkv.device) // fblk
        mask = f[None, :] <= f[:, None]
        o = F.scaled_dot_product_attention(x[0], x[1], x[2], attn_mask=mask)
        outs.append(o.transpose(1, 2).reshape(n * L, D))
        t0 += n * L
    return torch.cat(outs, 0)


@pytest.mark.parametrize("hd,H,groups,fblk", [(64, 16, [(2, 1032)], 258), (64, 16, [(1, 2064)], 258),
                                              (32, 4, [(3, 18), (2, 30)], 6), (64, 2, [(2, 300)], 100),
                                              (88, 2, [(1, 777)], 259), (32, 3, [(2, 129)], 43),
                                              (64, 2, [(1, 500), (2, 70)], 130)])  # partial last frame
def test_frame_causal_attention_vs_fp32(hd, H, groups, fblk):
    from vjepa2_amd import ops

    g = torch.Generator(device=DEV).manual_seed(hd * 1000 + fblk)
    T = sum(n * L for n, L in groups)
    D = H * hd
    qkv = torch.randn(T, 3 * D, device=DEV, generator=g).to(torch.bfloat16)
    do = torch.randn(T, D, device=DEV, generator=g).to(torch.bfloat16)
    o, stats = ops.attn_fwd(qkv, H, hd, groups, hd**-0.5, fblk=fblk)
    ref = _ref_attn(qkv, H, hd, groups, fblk)
    err = (o.float() - ref).abs().max().item()
    assert err <= 2**-7 * ref.abs().max().item() + 1e-3, err
    dqkv = ops.attn_bwd(qkv, o, do, stats, H, hd, groups, hd**-0.5, fblk=fblk)
    x = qkv.float().requires_grad_(True)
    _ref_attn(x, H, hd, groups, fblk).backward(do.float())
    for name, sl in (("dq", slice(0, D)), ("dk", slice(D, 2 * D)), ("dv", slice(2 * D, 3 * D))):
        e = rel_l1(dqkv[:, sl], x.grad[:, sl])
        assert e < 1e-2, f"{name}: rel_l1 {e:.2e}"
    # non-causal call of the same kernels is unchanged: fblk = 0 attends to everything
    o0, _ = ops.attn_fwd(qkv, H, hd, groups, hd**-0.5)
    assert not torch.equal(o0, o)


@pytest.mark.parametrize("which", ["causal", "causal_ext", "causal_silu_dp"])
def test_ac_predictor_matches_reference(which):
    """causal_silu_dp: SwiGLU MLPs and drop_path (block 1 at rate 0.5) in training mode, the reference's
    per-sample draws replayed through DropPath.sample in its call order."""
    from vjepa2_amd.ac_predictor import vit_ac_predictor

    g = torch.load(os.path.join(GOLD, "ac_predictor.pt"), weights_only=True)[which]
    m = vit_ac_predictor(**g["cfg"]).to(DEV)
    m.load_state_dict(g["state"])
    draws = list(g.get("draws") or [])
    for blk in m.predictor_blocks:
        if getattr(blk.drop_path, "drop_prob", 0):
            mine = [draws.pop(0), draws.pop(0)]
            blk.drop_path.sample = lambda n, device, mine=mine: mine.pop(0).to(device)
    assert not draws
    ins = {k: g[k].to(DEV).requires_grad_(True) for k in ("x", "actions", "states", "ext")}
    y = m(ins["x"], ins["actions"], ins["states"], ins["ext"] if g["cfg"]["use_extrinsics"] else None)
    assert y.shape == g["y"].shape
    y.backward(g["gy"].to(DEV))
    rep = [f"y {rel_l1(y, g['y']):.2e}"]
    assert rel_l1(y, g["y"]) < 1e-2, rep
    for k, gk in (("x", "gx"), ("actions", "gactions"), ("states", "gstates")) + (
            (("ext", "gext"),) if g["cfg"]["use_extrinsics"] else ()):
        e = rel_l1(ins[k].grad, g[gk])
        rep.append(f"d{k} {e:.2e}")
        assert e < 3e-2, rep
    for n, p in m.named_parameters():
        if n not in g["gparams"]:  # extrinsics_encoder without extrinsics: no grad in either
            assert p.grad is None or not p.grad.any(), n
            continue
        e = rel_l1(p.grad, g["gparams"][n])
        rep.append(f"d{n} {e:.2e}")
        assert e < 4e-2, "\n".join(rep)
    print("\n".join(rep))


def test_ac_predictor_256px_vs_oracle():
    """256^2 frames (16x16 patches), 4 frames after tubelets, 2 conditioning tokens per frame
    (L = 1032), predictor width 1024 / 16 heads, 2 blocks, B = 2: forward + input / weight gradients
    against the CPU oracle."""
    from oracle import vjepa_oracle as orc
    from vjepa2_amd.ac_predictor import vit_ac_predictor

    torch.manual_seed(5)
    cfg = dict(img_size=256, patch_size=16, num_frames=8, tubelet_size=2, embed_dim=1024, predictor_embed_dim=1024,
               depth=2, num_heads=16, action_embed_dim=7)
    m = vit_ac_predictor(**cfg)
    sd = {k: v.clone().requires_grad_(True) for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 4 * 256, 1024, generator=g)
    a = torch.randn(2, 4, 7, generator=g)
    s = torch.randn(2, 4, 7, generator=g)
    gy = torch.randn(2, 4 * 256, 1024, generator=g)
    xr = x.clone().requires_grad_(True)
    ref = orc.ac_predictor_forward(xr, a, s, sd, dict(grid=16, use_extrinsics=False, is_frame_causal=True,
                                                      num_frames=8, tubelet_size=2, depth=2, num_heads=16))
    ref.backward(gy)
    m = m.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    y = m(xd, a.to(DEV), s.to(DEV))
    y.backward(gy.to(DEV))
    assert rel_l1(y, ref) < 1e-2
    assert rel_l1(xd.grad, xr.grad) < 3e-2
    for n, p in m.named_parameters():
        if n.startswith("extrinsics_encoder"):
            continue
        e = rel_l1(p.grad, sd[n].grad)
        assert e < 4e-2, (n, e)


def test_acblock_standalone_forward():
    """ACBlock.forward / ACRoPEAttention.forward called directly with the reference's arguments
    (modules.py:488-497: attn_mask from build_action_block_causal_attention_mask, T, H, W,
    action_tokens) against the oracle's ac_block; any other attn_mask is refused."""
    import torch.nn as nn

    from oracle import vjepa_oracle as orc
    from vjepa2_amd.modules import ACBlock, build_action_block_causal_attention_mask

    torch.manual_seed(3)
    T, H, W, A, D = 3, 4, 4, 2, 128
    blk = ACBlock(dim=D, num_heads=2, mlp_ratio=4.0, qkv_bias=True, use_rope=True, grid_size=H,
                  norm_layer=lambda d: nn.LayerNorm(d, eps=1e-6))
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    x = torch.randn(2, T * (A + H * W), D)
    mask = build_action_block_causal_attention_mask(T, H, W, A)
    with torch.no_grad():
        ref = orc.ac_block(x, sd, "", 2, T, H, W, A, mask, H)
        got = blk.to(DEV)(x.to(DEV), attn_mask=mask.to(DEV), T=T, H=H, W=W, action_tokens=A)
    assert rel_l1(got, ref) < 1e-2, rel_l1(got, ref)
    with pytest.raises(NotImplementedError):
        blk(x.to(DEV), attn_mask=torch.ones_like(mask).to(DEV), T=T, H=H, W=W, action_tokens=A)
