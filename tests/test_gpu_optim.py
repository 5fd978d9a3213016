"""GPU: the fused AdamW over flat arenas is torch.optim.AdamW as the reference builds it
(app/vjepa/utils.py:207-255): same update, same per-parameter step counts (unused mask tokens and
inf/NaN-skipped steps do not advance), and a state_dict() that interchanges with the reference's
optimizer state in checkpoints (app/vjepa/train.py:318-329 writes it, app/vjepa/utils.py:121 loads it).
"""

import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _models():
    from vjepa2_amd.predictor import vit_predictor
    from vjepa2_amd.vision_transformer import VisionTransformer
    from vjepa2_amd.wrappers import MultiSeqWrapper, PredictorMultiSeqWrapper

    torch.manual_seed(0)
    enc = VisionTransformer(img_size=32, patch_size=16, num_frames=4, tubelet_size=2, embed_dim=64, depth=2,
                            num_heads=1, mlp_ratio=4, qkv_bias=True, use_rope=False, uniform_power=True,
                            norm_layer=lambda d: nn.LayerNorm(d, eps=1e-6))  # pos_embed: a frozen Parameter
    pred = vit_predictor(img_size=32, use_mask_tokens=True, patch_size=16, num_frames=4, tubelet_size=2,
                         embed_dim=64, predictor_embed_dim=64, depth=1, num_heads=2, uniform_power=True,
                         num_mask_tokens=3, use_rope=True)
    return MultiSeqWrapper(enc), PredictorMultiSeqWrapper(pred)


def _ref_opt(encoder, predictor):
    """app/vjepa/utils.py:224-239 restated: the reference's 4 AdamW param groups."""
    groups = [
        {"params": [p for n, p in encoder.named_parameters() if ("bias" not in n) and (len(p.shape) != 1)]},
        {"params": [p for n, p in predictor.named_parameters() if ("bias" not in n) and (len(p.shape) != 1)]},
        {"params": [p for n, p in encoder.named_parameters() if ("bias" in n) or (len(p.shape) == 1)],
         "WD_exclude": True, "weight_decay": 0},
        {"params": [p for n, p in predictor.named_parameters() if ("bias" in n) or (len(p.shape) == 1)],
         "WD_exclude": True, "weight_decay": 0},
    ]
    return torch.optim.AdamW(groups, betas=(0.9, 0.999), eps=1e-8)


def _set_lr_wd(opt, lr, wd):
    for g in opt.param_groups:
        g["lr"] = lr
        if not g.get("WD_exclude", False):
            g["weight_decay"] = wd


def _grads(named, seed, skip=()):
    g = torch.Generator().manual_seed(seed)
    return {n: (None if n in skip or not p.requires_grad else torch.randn(p.shape, generator=g))
            for n, p in named}


def test_fused_adamw_matches_torch_and_interchanges_state():
    from vjepa2_amd.train import init_opt

    enc, pred = _models()
    enc_ref, pred_ref = copy.deepcopy(enc), copy.deepcopy(pred)
    enc.to(DEV)
    pred.to(DEV)
    opt, _, _, _ = init_opt(enc, pred, iterations_per_epoch=10, start_lr=1e-4, ref_lr=1e-4, warmup=0, num_epochs=1,
                            mixed_precision=True)
    ref = _ref_opt(enc_ref, pred_ref)
    named = list(enc.named_parameters()) + [("p." + n, p) for n, p in pred.named_parameters()]
    named_ref = dict(list(enc_ref.named_parameters()) + [("p." + n, p) for n, p in pred_ref.named_parameters()])
    unused = {"p.backbone.mask_tokens.1", "p.backbone.mask_tokens.2"}  # grad None in the reference
    tokens = [pred.backbone.mask_tokens[1], pred.backbone.mask_tokens[2]]
    for step, (lr, wd) in enumerate([(5e-4, 0.04), (4e-4, 0.05), (3e-4, 0.06)]):
        grads = _grads(named, 100 + step, skip=unused)
        for n, p in named:
            if grads[n] is not None:
                p.grad.copy_(grads[n])
            named_ref[n].grad = grads[n]
        _set_lr_wd(opt, lr, wd)
        _set_lr_wd(ref, lr, wd)
        opt.step(exclude=tokens)
        ref.step()
        opt.zero_grad()
    torch.cuda.synchronize()
    for n, p in named:
        torch.testing.assert_close(p.detach().cpu(), named_ref[n].detach(), rtol=2e-6, atol=2e-7, msg=n)
    # state_dict: same numbering, keys, step counts and moments as torch's
    sd, sr = opt.state_dict(), ref.state_dict()
    assert [len(g["params"]) for g in sd["param_groups"]] == [len(g["params"]) for g in sr["param_groups"]]
    assert [g["params"] for g in sd["param_groups"]] == [g["params"] for g in sr["param_groups"]]
    assert sorted(sd["state"]) == sorted(sr["state"]), "state for the same parameters (none for unused ones)"
    for k in sr["state"]:
        assert float(sd["state"][k]["step"]) == float(sr["state"][k]["step"])
        for m in ("exp_avg", "exp_avg_sq"):
            # fp32 elementwise math in a different op order (lerp / fma): ~1 ulp of the O(1) moments
            torch.testing.assert_close(sd["state"][k][m], sr["state"][k][m], rtol=1e-5, atol=1e-6)
    for gd, gr in zip(sd["param_groups"], sr["param_groups"]):
        for key in gr:
            if key != "params":
                assert gd[key] == gr[key], (key, gd[key], gr[key])
    # ours -> torch.optim.AdamW (what the reference's load_checkpoint does) and torch -> ours
    ref2 = _ref_opt(copy.deepcopy(enc_ref), copy.deepcopy(pred_ref))
    ref2.load_state_dict(sd)
    enc2, pred2 = _models()
    enc2.to(DEV)
    pred2.to(DEV)
    opt2, _, _, _ = init_opt(enc2, pred2, iterations_per_epoch=10, start_lr=1e-4, ref_lr=1e-4, warmup=0,
                             num_epochs=1, mixed_precision=True)
    opt2.load_state_dict(sr)
    sd2 = opt2.state_dict()
    for k in sr["state"]:
        torch.testing.assert_close(sd2["state"][k]["exp_avg"], sr["state"][k]["exp_avg"], rtol=0, atol=0)
        assert float(sd2["state"][k]["step"]) == float(sr["state"][k]["step"])


def test_inf_skip_does_not_advance_step():
    """GradScaler.step skips optimizer.step on inf/NaN (train.py:446-451): nothing moves and the
    bias correction of the next step uses the un-advanced count."""
    from vjepa2_amd.train import init_opt

    enc, pred = _models()
    enc_ref, pred_ref = copy.deepcopy(enc), copy.deepcopy(pred)
    enc.to(DEV)
    pred.to(DEV)
    opt, _, _, _ = init_opt(enc, pred, iterations_per_epoch=10, start_lr=1e-4, ref_lr=1e-4, warmup=0, num_epochs=1,
                            mixed_precision=True)
    ref = _ref_opt(enc_ref, pred_ref)
    named = list(enc.named_parameters()) + [("p." + n, p) for n, p in pred.named_parameters()]
    named_ref = dict(list(enc_ref.named_parameters()) + [("p." + n, p) for n, p in pred_ref.named_parameters()])
    for step in range(3):
        grads = _grads(named, 7 + step)
        if step == 1:  # an inf in one gradient: the whole step is skipped
            first = next(n for n in grads if grads[n] is not None)
            grads[first][0] = float("inf")
        for n, p in named:
            if grads[n] is not None:
                p.grad.copy_(grads[n])
            named_ref[n].grad = grads[n]
        _set_lr_wd(opt, 5e-4, 0.04)
        _set_lr_wd(ref, 5e-4, 0.04)
        before = [a.data.clone() for a in opt.arenas]
        opt.step(found_inf=opt.check_finite())
        if step != 1:
            ref.step()  # the reference's scaler.step() skips it on inf
        else:
            torch.cuda.synchronize()
            assert all(torch.equal(b, a.data) for b, a in zip(before, opt.arenas))
        opt.zero_grad()
    torch.cuda.synchronize()
    assert opt.steps == [2, 2, 2, 2]
    for n, p in named:
        torch.testing.assert_close(p.detach().cpu(), named_ref[n].detach(), rtol=2e-6, atol=2e-7, msg=n)


def test_lazy_zero_overwrite_marked_grad_not_written_is_zero():
    """FlatArena.zero_grad leaves the gradients of weights a weight-gradient GEMM overwrites
    (functions.wgrad_buf marks them) untouched until their first write of the step. A marked weight
    that nothing writes in a step (here: p1) must reach check_finite / AdamW as zeros, not as the
    previous step's values; a marked weight first touched by an accumulating write (grad_buf) is
    zeroed before it. Checked against torch AdamW fed the true gradients (p1: zero)."""
    from vjepa2_amd.arena import FlatArena, FusedAdamW
    from vjepa2_amd.functions import grad_buf, wgrad_buf

    torch.manual_seed(3)
    ps = [nn.Parameter(torch.randn(8, 16)) for _ in range(3)]
    ref = [nn.Parameter(p.detach().clone()) for p in ps]
    arena = FlatArena([(f"w{i}", p) for i, p in enumerate(ps)], DEV)
    opt = FusedAdamW([arena], [None], lr=1e-2, weight_decay=0.04)
    ropt = torch.optim.AdamW(ref, lr=1e-2, weight_decay=0.04)
    g = torch.Generator().manual_seed(5)
    # step 1: every weight written through the weight-gradient path (marks them overwrite-on-first-
    # write; on the fresh arena the gradients are zero and current, so this first call accumulates)
    g1 = [torch.randn(8, 16, generator=g) for _ in ps]
    for p, gg in zip(ps, g1):
        buf, acc = wgrad_buf(p)
        if acc:
            buf.add_(gg.to(DEV))
        else:
            buf.copy_(gg)
    for r, gg in zip(ref, g1):
        r.grad = gg.clone()
    opt.step(found_inf=opt.check_finite())
    ropt.step()
    opt.zero_grad()
    assert all(getattr(p, "_vj_ow", False) for p in ps)
    # step 2: p0 overwritten, p1 not written at all (stale step-1 values still in the arena), p2 first
    # touched by an accumulating write (must start from zero), then by an overwrite-path call
    g2 = [torch.randn(8, 16, generator=g) for _ in ps]
    buf, acc = wgrad_buf(ps[0])
    assert not acc
    buf.copy_(g2[0])
    grad_buf(ps[2]).add_(g2[2].to(DEV))
    buf, acc = wgrad_buf(ps[2])
    assert acc  # already touched this step: accumulate
    buf.add_(g2[2].to(DEV))
    found = opt.check_finite()  # finalize_grads zeroes p1
    torch.cuda.synchronize()
    assert int(found.item()) == 0
    assert ps[1].grad.abs().max().item() == 0.0, "stale gradient of an unwritten overwrite-marked weight"
    torch.testing.assert_close(ps[2].grad.cpu(), 2 * g2[2])
    opt.step(found_inf=found)
    ref[0].grad, ref[1].grad, ref[2].grad = g2[0].clone(), torch.zeros(8, 16), 2 * g2[2]
    ropt.step()
    torch.cuda.synchronize()
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p.detach().cpu(), r.detach(), rtol=2e-6, atol=2e-7)


def test_staged_update_matches_one_pass():
    """The staged AdamW + EMA issue (JEPATrainer.inputs_resident: the next step's target forward waits
    per stage on the side stream) gives bitwise the losses, parameters and target weights of the
    one-pass update over 3 steps."""
    import copy

    from vjepa2_amd.masks import MaskCollator
    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model

    dev = torch.device("cuda", 0)
    T, S, B = 8, 64, 2
    masks = [dict(aspect_ratio=[0.75, 1.5], num_blocks=8, spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
             dict(aspect_ratio=[0.75, 1.5], num_blocks=2, spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0])]
    torch.manual_seed(0)
    mc = MaskCollator(masks, [T], crop_size=S, patch_size=16)
    data = []
    for i in range(3):
        (_, me, mp), = mc([(0, 0, [torch.arange(T)])] * B)
        clips = torch.randn(B, 3, T, S, S, generator=torch.Generator().manual_seed(i)).to(dev)
        data.append(([clips], [[m.to(dev) for m in me]], [[m.to(dev) for m in mp]]))
    torch.cuda.synchronize()

    def run(staged):
        torch.manual_seed(239)
        enc, pred = init_video_model(device=dev, patch_size=16, max_num_frames=T, tubelet_size=2,
                                     model_name="vit_small", crop_size=S, pred_depth=2, pred_num_heads=12,
                                     pred_embed_dim=384, uniform_power=True, use_mask_tokens=True, num_mask_tokens=2,
                                     use_sdpa=True, use_rope=True)
        tgt = copy.deepcopy(enc)
        opt, _, _, _ = init_opt(enc, pred, iterations_per_epoch=10, start_lr=1e-4, ref_lr=1e-4, warmup=0,
                                num_epochs=1, wd=0.04, final_wd=0.04, mixed_precision=True)
        tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True)
        tr.inputs_resident = staged
        losses = [tr.train_step(c, me, mp, 0.99).clone() for c, me, mp in data]
        assert (tr._staged is not None) == staged  # the last step staged its update (unused yet)
        torch.cuda.synchronize()
        return ([l.item() for l in losses], [a.data.clone() for a in tr.opt.arenas],
                [a.data.clone() for a in tr.tgt_arenas])

    a, b = run(False), run(True)
    assert a[0] == b[0]
    for x, y in zip(a[1] + a[2], b[1] + b[2]):
        assert torch.equal(x, y)
