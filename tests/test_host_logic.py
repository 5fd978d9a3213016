"""CPU: host-side logic of the product (no kernels): mask generation vs the reference's golden masks
(bit-exact), init-weight parity with the reference, schedulers, optimizer grouping, arena ranges,
all-reduce bucket plans, FLOP accounting."""

import os

import pytest
import torch
import torch.nn as nn

GOLD = os.path.join(os.path.dirname(__file__), "golden")
VITL = [dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=8,
             spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
        dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=2,
             spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0])]


def gold(n):
    return torch.load(os.path.join(GOLD, n), weights_only=True)


@pytest.mark.parametrize("tag", ["vitl", "small"])
def test_masks_bit_exact(tag):
    from vjepa2_amd.masks import MaskCollator

    g = gold("masks.pt")[tag]
    torch.manual_seed(239)
    mc = MaskCollator(VITL, [g["fpc"]], crop_size=g["crop"], patch_size=16, tubelet_size=2)
    for it in g["iters"]:
        (_, e, p), = mc([(torch.zeros(1), 0, [torch.arange(g["fpc"])]) for _ in range(g["B"])])
        for a, b in zip(e + p, it["enc"] + it["pred"]):
            assert a.dtype == torch.int64 and torch.equal(a, b)


def test_mask_options_bit_exact():
    from vjepa2_amd.masks import MaskCollator

    for name, ex in gold("masks.pt")["extras"].items():
        torch.manual_seed(5)
        mc = MaskCollator([ex["cfg"]], [8], crop_size=64, patch_size=16, tubelet_size=2)
        (_, e, p), = mc([(torch.zeros(1), 0, [torch.arange(8)]) for _ in range(3)])
        assert torch.equal(e[0], ex["enc"][0]) and torch.equal(p[0], ex["pred"][0]), name


def _np_build(spec):
    """CPU restatement of vj_mask_count / vj_mask_emit (mode 0) for one MaskSpec."""
    import numpy as np

    D, H, W = spec.grid
    t, h, w = spec.size
    kept = []
    for b in range(spec.boxes.shape[0]):
        g = np.ones((D, H, W), bool)
        g[spec.max_ctx:] = False
        for s_, tp, lf in spec.boxes[b]:
            g[s_:s_ + t, tp:tp + h, lf:lf + w] = False
        kept.append(g.ravel())
    ke = min(int(k.sum()) for k in kept)
    kp = min(int((~k).sum()) for k in kept)
    if spec.max_keep is not None:
        ke = min(ke, spec.max_keep)
    return (torch.tensor(np.stack([np.nonzero(k)[0][:ke] for k in kept])),
            torch.tensor(np.stack([np.nonzero(~k)[0][:kp] for k in kept])))


@pytest.mark.parametrize("extra", [{}, dict(max_temporal_keep=0.5, temporal_scale=[0.5, 1.0]), dict(max_keep=300)])
def test_device_mask_draws_match_host_collate(extra):
    """The device-mask collate (MaskCollator(device_masks=True)) makes exactly the host collate's RNG
    draws: the masks rebuilt on the CPU from its MaskSpecs equal the host masks, and the global RNG
    ends in the same state."""
    from vjepa2_amd.masks import MaskCollator

    cfgs = [dict(c, **extra) for c in VITL]
    for seed in range(4):
        host = MaskCollator(cfgs, [16], crop_size=256, patch_size=16)
        dev = MaskCollator(cfgs, [16], crop_size=256, patch_size=16, device_masks=True)
        torch.manual_seed(seed)
        (_, he, hp), = host([(0, 0, [torch.arange(16)])] * 24)
        after = torch.rand(1)
        torch.manual_seed(seed)
        (_, specs, none), = dev([(0, 0, [torch.arange(16)])] * 24)
        assert none is None and torch.equal(torch.rand(1), after)
        for j, spec in enumerate(specs):
            e, p = _np_build(spec)
            assert torch.equal(e, he[j]) and torch.equal(p, hp[j])


def test_masks_are_sorted_disjoint():
    from vjepa2_amd.masks import MaskCollator

    torch.manual_seed(1)
    mc = MaskCollator(VITL, [16], crop_size=256, patch_size=16)
    (_, e, p), = mc([(0, 0, [torch.arange(16)])] * 3)
    for me, mp in zip(e, p):
        for b in range(3):
            a, c = me[b], mp[b]
            assert torch.all(a[1:] > a[:-1]) and torch.all(c[1:] > c[:-1])
            assert not set(a.tolist()) & set(c.tolist())


def test_init_weights_match_reference():
    from vjepa2_amd import vision_transformer as vt
    from vjepa2_amd.train import init_video_model

    g = gold("train_steps.pt")
    vt.vit_micro = lambda patch_size=16, **kw: vt.VisionTransformer(
        patch_size=patch_size, embed_dim=64, depth=2, num_heads=1, mlp_ratio=4, qkv_bias=True,
        norm_layer=lambda d: nn.LayerNorm(d, eps=1e-6), **kw)
    cm = g["args"]["model"]
    torch.manual_seed(239)
    enc, pred = init_video_model(device="cpu", patch_size=16, max_num_frames=8, tubelet_size=2, model_name="vit_micro",
                                 crop_size=64, pred_depth=cm["pred_depth"], pred_num_heads=cm["pred_num_heads"],
                                 pred_embed_dim=cm["pred_embed_dim"], uniform_power=True, use_mask_tokens=True,
                                 num_mask_tokens=2, use_sdpa=True, use_rope=True)
    esd, psd = enc.backbone.state_dict(), pred.backbone.state_dict()
    assert set(esd) == set(g["init_encoder"]) and set(psd) == set(g["init_predictor"])
    for k, v in g["init_encoder"].items():
        assert torch.equal(esd[k], v), k
    for k, v in g["init_predictor"].items():
        assert torch.equal(psd[k], v), k


def test_state_dict_keys_vitl():
    from vjepa2_amd.predictor import vit_predictor
    from vjepa2_amd.vision_transformer import vit_large

    enc = vit_large(img_size=256, num_frames=16, use_rope=True)
    sd = enc.state_dict()
    assert sd["patch_embed.proj.weight"].shape == (1024, 3, 2, 16, 16)
    assert sd["blocks.23.attn.qkv.weight"].shape == (3072, 1024) and "pos_embed" not in sd
    assert sum(p.numel() for p in enc.parameters()) == 303_885_312  # SURVEY §2 C1 message size
    pred = vit_predictor(img_size=256, use_mask_tokens=True, num_frames=16, embed_dim=1024, predictor_embed_dim=384,
                         depth=12, num_heads=12, num_mask_tokens=6, use_rope=True)
    assert sum(p.numel() for p in pred.parameters()) == 22_084_480
    assert "mask_tokens.5" in pred.state_dict()


def test_schedulers_match_oracle():
    from oracle import vjepa_oracle as orc
    from vjepa2_amd.schedulers import CosineWDSchedule, WarmupCosineSchedule

    class O:
        param_groups = [dict(lr=0, weight_decay=0), dict(lr=0, weight_decay=0, WD_exclude=True)]

    s = WarmupCosineSchedule(O, warmup_steps=40 * 300, start_lr=1e-4, ref_lr=5.25e-4, T_max=int(1.25 * 10 * 300),
                             final_lr=1e-6)
    w = CosineWDSchedule(O, ref_wd=0.04, final_wd=0.4, T_max=int(1.25 * 10 * 300))
    so = orc.WarmupCosine(40 * 300, 1e-4, 5.25e-4, int(1.25 * 10 * 300), 1e-6)
    wo = orc.CosineWD(0.04, int(1.25 * 10 * 300), 0.4)
    for _ in range(5000):
        assert s.step() == so.step() and w.step() == wo.step()
    assert O.param_groups[1]["weight_decay"] == 0


def test_weight_decay_groups():
    from vjepa2_amd.arena import readiness_order, wd_split
    from vjepa2_amd.predictor import vit_predictor

    pred = vit_predictor(img_size=64, use_mask_tokens=True, num_frames=8, embed_dim=64, predictor_embed_dim=64,
                         depth=2, num_heads=2, num_mask_tokens=2, use_rope=True)
    wd, nowd = wd_split(readiness_order(pred.named_parameters()))
    names_wd = [n for n, _ in wd]
    assert names_wd[0] == "predictor_proj.weight" and names_wd[-1] == "predictor_embed.weight"
    assert "mask_tokens.0" in names_wd  # 3-D, no 'bias' -> decayed (app/vjepa/utils.py:224-237)
    assert all(("bias" in n) or p.dim() == 1 for n, p in nowd)


def test_bucket_plan_in_readiness_order():
    import torch.distributed as dist

    from vjepa2_amd.distributed import GradReducer

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29611")
        dist.init_process_group("gloo", rank=0, world_size=1)
    mods = [nn.Linear(256, 256, bias=False) for _ in range(6)]
    flat = torch.zeros(6 * 65536)
    plist = [(m.weight, i * 65536, 65536) for i, m in enumerate(mods)]
    r = GradReducer([(flat, plist)], bucket_mb=0.5)
    assert len(r.buckets) == 3 and all(len(b.params) == 2 for b in r.buckets)
    r.mark_ready(mods[0])
    assert r.next == 0  # bucket 0 still waits for mods[1]
    r.mark_ready(mods[1])
    assert r.next == 1
    r.mark_ready(mods[4])
    r.mark_ready(mods[5])
    assert r.next == 1  # bucket 2 complete but bucket 1 not issued yet: order is preserved
    r.mark_ready(mods[2])
    r.mark_ready(mods[3])
    assert r.next == 3
    r.finish()


def test_step_flops_formula():
    from bench import step_flops

    g = torch.Generator().manual_seed(0)
    me = [torch.zeros(24, 513, dtype=torch.long), torch.zeros(24, 130, dtype=torch.long)]
    mp = [torch.zeros(24, 966, dtype=torch.long), torch.zeros(24, 1437, dtype=torch.long)]
    f = step_flops("vit_large", 24, 2048, me, mp) / 24
    assert 3.4e12 < f < 3.7e12  # 3.56 TF/clip at the mean masks


def test_pooler_init_matches_reference():
    """AttentivePooler / AttentiveClassifier (attentive_pooler.py:16-137): same parameter names, shapes
    and init RNG consumption as the reference (per-tensor sums of the reference's init, seed 11)."""
    from vjepa2_amd.attentive_pooler import AttentiveClassifier, AttentivePooler

    g = torch.load(os.path.join(os.path.dirname(__file__), "golden", "pooler.pt"), weights_only=True)
    for which, ctor in (("clf", AttentiveClassifier), ("pool3", AttentivePooler)):
        torch.manual_seed(11)
        m = ctor(**g[which]["cfg"])
        sd = m.state_dict()
        assert set(sd) == set(g[which]["init"]), which
        for k, (s1, s2) in g[which]["init"].items():
            v = sd[k].double()
            assert v.sum().item() == s1 and v.pow(2).sum().item() == s2, (which, k)


def test_ac_predictor_init_matches_reference():
    """VisionTransformerPredictorAC (ac_predictor.py:17-139): parameter names, shapes and init RNG
    consumption equal the reference's (per-tensor sums of its init, seed 31); the frame-causal mask
    builder equals modules.py:12-23."""
    from vjepa2_amd.ac_predictor import vit_ac_predictor
    from vjepa2_amd.modules import build_action_block_causal_attention_mask

    g = torch.load(os.path.join(os.path.dirname(__file__), "golden", "ac_predictor.pt"), weights_only=True)
    assert torch.equal(build_action_block_causal_attention_mask(3, 2, 2, 2), g["mask_T3_2x2_a2"])
    for which in ("causal", "causal_ext"):
        torch.manual_seed(31)
        m = vit_ac_predictor(**g[which]["cfg"])
        sd = m.state_dict()
        assert set(sd) == set(g[which]["init"]), which
        for k, (s1, s2) in g[which]["init"].items():
            v = sd[k].double()
            assert v.sum().item() == s1 and v.pow(2).sum().item() == s2, (which, k)
