"""CPU: pin the oracle (oracle/vjepa_oracle.py) to the REFERENCE's own outputs (tests/golden/*.pt,
produced by tests/golden/make_golden.py running weipeilun/vjepa2 on CPU, fp32)."""

import os

import pytest
import torch

from oracle import vjepa_oracle as orc

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    return torch.load(os.path.join(GOLD, name), weights_only=True)


def close(a, b, tol, what):
    err = (a.detach().float() - b.detach().float()).abs().max().item()
    scale = b.detach().float().abs().max().item() + 1e-12
    assert err <= tol * max(1.0, scale), f"{what}: max err {err:.3e} (scale {scale:.3e})"


def test_rope_golden():
    g = gold("rope.pt")
    for s in (20, 10):
        close(orc.rotate_queries_or_keys(g[f"x{s}"], g[f"pos{s}"]), g[f"out{s}"], 1e-6, f"rope{s}")
    close(orc.rotate_queries_or_keys(g["x_flat"], g["pos_flat"]), g["out_flat"], 1e-6, "rope flat")


def test_sincos_golden():
    g = gold("sincos.pt")
    for up in (0, 1):
        t = torch.from_numpy(orc.sincos_3d(96, 4, 2, uniform_power=bool(up)))
        assert torch.equal(t, g[f"f64_up{up}"])


def test_product_sincos_table_matches_reference():
    from vjepa2_amd.vision_transformer import sincos_3d_table

    g = gold("sincos.pt")
    for up in (0, 1):
        assert torch.equal(torch.from_numpy(sincos_3d_table(96, 4, 2, bool(up))), g[f"f64_up{up}"])


@pytest.mark.parametrize("fixture", ["block_enc.pt", "block_pred.pt", "block_swiglu.pt", "block_droppath.pt",
                                     "block_swiglu_dp.pt"])
def test_block_golden(fixture):
    """Block (modules.py:500-563), incl. the SwiGLU MLP and drop_path variants (their per-sample
    draws replayed from the fixture)."""
    g = gold(fixture)
    c = g["cfg"]
    sd = {k: v.clone().requires_grad_(True) for k, v in g["state"].items()}
    x = g["x"].clone().requires_grad_(True)
    grid = c["grid"]
    tpf, tpr = grid * grid, grid  # with T/H/W given the same square grid results
    draws = g["draws"] if g.get("draws") else None
    y = orc.block(x, sd, "", c["heads"], ids=g["mask"], tokens_per_frame=tpf, tokens_per_row=tpr, draws=draws)
    close(y, g["y"], 1e-5, "block y")
    y.backward(g["gy"])
    close(x.grad, g["gx"], 1e-5, "block dx")
    for n, v in g["gparams"].items():
        close(sd[n].grad, v, 1e-5, f"block d{n}")


@pytest.mark.parametrize("rope", [1, 0])
def test_encoder_golden(rope):
    g = gold(f"encoder_rope{rope}.pt")
    sd = {k: v.clone().requires_grad_(k != "pos_embed") for k, v in g["state"].items()}
    cfg = dict(patch_size=16, tubelet_size=2, num_heads=1, depth=2, use_rope=bool(rope))
    close(orc.encoder_forward(g["x"], sd, cfg), g["full"], 1e-5, "encoder full")
    outs = [orc.encoder_forward(g["x"], sd, cfg, masks=m) for m in g["masks"]]
    for o, e in zip(outs, g["outs"]):
        close(o, e, 1e-5, "encoder masked")
    sum((o * gy).sum() for o, gy in zip(outs, g["gys"])).backward()
    for n, v in g["gparams"].items():
        close(sd[n].grad, v, 1e-5, f"encoder d{n}")


def test_predictor_golden():
    g = gold("predictor.pt")
    sd = {k: v.clone().requires_grad_(k != "predictor_pos_embed") for k, v in g["state"].items()}
    cfg = dict(num_heads=3, depth=2, use_rope=True, grid_size=2, num_mask_tokens=2, num_patches=8)
    for inp, exp, gy in zip(g["ins"], g["outs"], g["gys"]):
        z = inp["z"].clone().requires_grad_(True)
        o = orc.predictor_forward(z, inp["mx"], inp["my"], sd, cfg, mask_index=inp["mask_index"])
        close(o, exp, 1e-5, "predictor out")
        (o * gy).sum().backward()
        close(z.grad, inp["gz"], 1e-5, "predictor dz")
    for n, v in g["gparams"].items():
        close(sd[n].grad, v, 1e-5, f"predictor d{n}")


def test_train_steps_golden():
    """Oracle replays 3 iterations of the reference app/vjepa/train.py:main bit-for-bit-ish (fp32)."""
    g = gold("train_steps.pt")
    a = g["args"]
    co = a["optimization"]
    enc_cfg = dict(patch_size=16, tubelet_size=2, num_heads=1, depth=2, use_rope=True)
    pred_cfg = dict(num_heads=2, depth=2, use_rope=True, grid_size=4, num_mask_tokens=2, num_patches=64)
    tr = orc.OracleTrainer(g["init_encoder"], g["init_predictor"], enc_cfg, pred_cfg)
    ipe = co["ipe"]
    sched = orc.WarmupCosine(int(co["warmup"] * ipe), co["start_lr"], co["lr"], int(co["ipe_scale"] * co["epochs"] * ipe),
                             co["final_lr"])
    wds = orc.CosineWD(co["weight_decay"], int(co["ipe_scale"] * co["epochs"] * ipe), co["final_weight_decay"])
    for i, s in enumerate(g["samples"]):
        clips = torch.stack([torch.randn(3, 8, 64, 64, generator=torch.Generator().manual_seed(sd))
                             for sd in s["clip_seeds"]])
        assert abs(clips.double().sum().item() - float(s["clip_sum"])) < 1e-6
        lr, wd = sched.step(), wds.step()
        assert lr == g["lrs"][i] and wd == g["wds"][i]
        loss = tr.step(clips, s["enc"], s["pred"], lr, wd, co["ema"][0])
        assert abs(loss - g["losses"][i]) < 1e-6 * max(1.0, abs(g["losses"][i])), (i, loss, g["losses"][i])
    for k, v in g["final_encoder"].items():
        close(tr.enc[k], v, 1e-6, f"final enc {k}")
    for k, v in g["final_predictor"].items():
        close(tr.pred[k], v, 1e-6, f"final pred {k}")
    for k, v in g["final_target"].items():
        close(tr.tgt[k], v, 1e-6, f"final target {k}")


def test_rope_angle_precision_envelope():
    """The documented RoPE deviation, pinned as an envelope: the reference rotates q / k under
    autocast, so modules.py:26-50 computes its angles in bf16 (x.dtype); the build uses fp32 angles
    (reference op order). On ViT-L positions (frame < 8, row / col < 16, slice width 20) against
    fp64 angles: the build's rotation is within bf16 output rounding of the exact one, the
    reference's bf16-angle rotation is measurably further, and the two differ by at most 2.5e-2 of
    max |x| (the reference's own angle error, up to ~8e-3 rad at these positions)."""
    torch.manual_seed(0)
    x = torch.randn(1, 1, 16, 20, dtype=torch.float64)
    pos = torch.arange(16, dtype=torch.float64)[None, None]
    exact = orc.rotate_queries_or_keys(x, pos)
    ours = orc.rotate_queries_or_keys(x.float(), pos.float()).to(torch.bfloat16).double()
    ref_autocast = orc.rotate_queries_or_keys(x.to(torch.bfloat16), pos.to(torch.bfloat16)).double()
    scale = x.abs().max().item()
    e_ours = (ours - exact).abs().max().item() / scale
    e_ref = (ref_autocast - exact).abs().max().item() / scale
    dev = (ours - ref_autocast).abs().max().item() / scale
    print(f"RoPE vs fp64: fp32 angles {e_ours:.2e}, reference bf16 angles {e_ref:.2e}; deviation {dev:.2e}")
    assert e_ours <= 2 ** -8 and e_ref > e_ours and dev <= 2.5e-2


@pytest.mark.parametrize("which", ["clf", "pool3"])
def test_pooler_golden(which):
    """Frozen-encoder probe (attentive_pooler.py / modules.py:566-610): the oracle's AttentiveClassifier
    (2 Blocks + CrossAttentionBlock, 1 query) and 3-query AttentivePooler with the bare CrossAttention
    reproduce the reference's outputs and every gradient."""
    g = gold("pooler.pt")[which]
    c = g["cfg"]
    sd = {k: v.clone().requires_grad_(True) for k, v in g["state"].items()}
    x = g["x"].clone().requires_grad_(True)
    if which == "clf":
        y = orc.attentive_classifier(x, sd, c["num_heads"], c["depth"])
    else:
        y = orc.attentive_pooler(x, sd, "", c["num_heads"], c["depth"], complete_block=c["complete_block"])
    close(y, g["y"], 1e-5, f"{which} y")
    y.backward(g["gy"])
    close(x.grad, g["gx"], 1e-5, f"{which} dx")
    assert set(g["gparams"]) <= set(sd)
    for n, v in g["gparams"].items():
        close(sd[n].grad, v, 1e-5, f"{which} d{n}")


def test_multiclip_golden():
    """ClipAggregation (vit_encoder_multiclip.py:117-162): clip / view regrouping, time-major
    concatenation and the temporal sincos add at the clips' frame indices, vs the reference."""
    g = gold("multiclip.pt")
    sd = g["state"]
    cfg = dict(patch_size=16, tubelet_size=2, num_heads=1, depth=2, use_rope=True)
    t = torch.from_numpy(orc.sincos_1d(64, torch.arange(8).numpy().astype(float))).float()[None]
    close(t, g["pos_embed"], 1e-7, "temporal sincos table")
    outs = orc.clip_aggregation(g["x"], lambda c: orc.encoder_forward(c, sd, cfg), 2, g["pos_embed"],
                                g["clip_indices"])
    assert len(outs) == len(g["outs"])
    for o, e in zip(outs, g["outs"]):
        close(o, e, 1e-5, "multiclip view")


def _ac_block_draws(g):
    """The fixture's drop_path draws (flat, in the reference's call order) per predictor block: blocks
    with rate 0 (torch.linspace(0, drop_path_rate, depth)[i] == 0) draw nothing, others attention then MLP."""
    c = g["cfg"]
    rates = torch.linspace(0, c.get("drop_path_rate", 0.0), c["depth"]).tolist()
    draws = list(g.get("draws") or [])
    out = []
    for r in rates:
        out.append((draws.pop(0), draws.pop(0)) if r > 0 else None)
    assert not draws
    return out


@pytest.mark.parametrize("which", ["causal", "causal_ext", "causal_silu_dp"])
def test_ac_predictor_golden(which):
    """V-JEPA 2-AC predictor (ac_predictor.py:141-190, ACRoPEAttention modules.py:163-258): the oracle
    reproduces the reference's output and every gradient (frame-causal mask, action / state /
    extrinsics tokens)."""
    g = gold("ac_predictor.pt")
    assert torch.equal(orc.action_block_causal_mask(3, 2, 2, 2), g["mask_T3_2x2_a2"])
    g = g[which]
    c = g["cfg"]
    cfg = dict(grid=c["img_size"] // c["patch_size"], use_extrinsics=c["use_extrinsics"],
               is_frame_causal=c["is_frame_causal"], num_frames=c["num_frames"], tubelet_size=c["tubelet_size"],
               depth=c["depth"], num_heads=c["num_heads"])
    sd = {k: v.clone().requires_grad_(True) for k, v in g["state"].items()}
    ins = {k: g[k].clone().requires_grad_(True) for k in ("x", "actions", "states", "ext")}
    y = orc.ac_predictor_forward(ins["x"], ins["actions"], ins["states"], sd, cfg,
                                 extrinsics=ins["ext"] if c["use_extrinsics"] else None, block_draws=_ac_block_draws(g))
    close(y, g["y"], 1e-5, f"{which} y")
    y.backward(g["gy"])
    close(ins["x"].grad, g["gx"], 1e-5, "dx")
    close(ins["actions"].grad, g["gactions"], 1e-5, "dactions")
    close(ins["states"].grad, g["gstates"], 1e-5, "dstates")
    if c["use_extrinsics"]:
        close(ins["ext"].grad, g["gext"], 1e-5, "dext")
    for n, v in g["gparams"].items():
        close(sd[n].grad, v, 1e-5, f"{which} d{n}")


def test_vitl_seeded_init_matches_reference():
    """vjepa2_amd.vision_transformer.vit_large under torch.manual_seed(239) builds the reference's
    exact initial weights (per-tensor sums of the reference's seeded init, tests/golden/vitl_autocast.pt):
    the premise of the bf16-autocast comparison in test_gpu_model.py."""
    from vjepa2_amd.vision_transformer import vit_large

    d = torch.load(os.path.join(GOLD, "vitl_autocast.pt"), weights_only=True)
    torch.manual_seed(d["seed"])
    enc = vit_large(img_size=64, num_frames=16, tubelet_size=2, use_rope=True, uniform_power=True, use_sdpa=True)
    sd = enc.state_dict()
    assert set(sd) == set(d["param_sums"])
    for k, v in sd.items():
        assert abs(float(v.double().sum()) - d["param_sums"][k]) <= 1e-9 * (1 + abs(d["param_sums"][k])), k


@pytest.mark.parametrize("fixture", ["block_swiglu.pt", "block_droppath.pt", "block_swiglu_dp.pt"])
def test_variant_block_seeded_init_matches_reference(fixture):
    """vjepa2_amd.modules.Block with SwiGLU / drop_path builds the reference's parameters with the same
    RNG consumption: under the fixture's seed (and the generator's perturbation) every tensor of the
    state dict is bitwise the reference's."""
    import torch.nn as nn

    from vjepa2_amd.modules import Block

    g = gold(fixture)
    c = g["cfg"]
    torch.manual_seed(c["seed"])
    blk = Block(dim=c["dim"], num_heads=c["heads"], mlp_ratio=4.0, qkv_bias=True, use_rope=True, grid_size=c["grid"],
                act_layer=nn.SiLU if c["silu"] else nn.GELU, wide_silu=c["wide_silu"], drop_path=c["drop_path"],
                norm_layer=lambda d: nn.LayerNorm(d, eps=1e-6))
    for p in blk.parameters():
        with torch.no_grad():
            p.add_(0.05 * torch.randn_like(p))
    sd = blk.state_dict()
    assert list(sd) == list(g["state"])
    for k, v in g["state"].items():
        assert torch.equal(sd[k], v), k
