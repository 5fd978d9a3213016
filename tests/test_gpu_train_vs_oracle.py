"""One fused V-JEPA train step (target fwd, context fwd+bwd, predictor fwd+bwd, loss, AdamW, EMA) on
the HIP kernels vs the fp32 CPU oracle trainer, with the target encoder's residual stream in bf16
(the trainer's default, the reference's autocast precision) and in f32. Same tiny config as the
driver's smoke check (vit_small, 8x64^2, B=2, predictor depth 2)."""
import copy

import pytest
import torch

from oracle import vjepa_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bf16_target,silu", [(True, False), (False, False), (True, True)])
def test_train_step_vs_oracle(bf16_target, silu):
    """silu: encoder and predictor on the SwiGLU MLP (model.use_silu / use_pred_silu, wide_silu)."""
    from vjepa2_amd.masks import MaskCollator
    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model

    dev = torch.device("cuda", 0)
    torch.manual_seed(239)
    T, S, B = 8, 64, 2
    enc, pred = init_video_model(device=dev, patch_size=16, max_num_frames=T, tubelet_size=2, model_name="vit_small",
                                 crop_size=S, pred_depth=2, pred_num_heads=12, pred_embed_dim=384, uniform_power=True,
                                 use_mask_tokens=True, num_mask_tokens=2, use_sdpa=True, use_rope=True,
                                 use_silu=silu, use_pred_silu=silu, wide_silu=True)
    assert silu == hasattr(enc.backbone.blocks[0].mlp, "fc3") == hasattr(pred.backbone.predictor_blocks[0].mlp, "fc3")
    enc_sd = {k: v.detach().cpu().clone() for k, v in enc.backbone.state_dict().items()}
    pred_sd = {k: v.detach().cpu().clone() for k, v in pred.backbone.state_dict().items()}
    tgt = copy.deepcopy(enc)
    opt, _, _, _ = init_opt(enc, pred, iterations_per_epoch=10, start_lr=1e-4, ref_lr=1e-4, warmup=0, num_epochs=1,
                            wd=0.04, final_wd=0.04, mixed_precision=True)
    for g in opt.param_groups:
        g["lr"] = 1e-4
        if not g.get("WD_exclude", False):
            g["weight_decay"] = 0.04
    tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True, target_bf16_residual=bf16_target)
    masks = [dict(aspect_ratio=[0.75, 1.5], num_blocks=8, spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
             dict(aspect_ratio=[0.75, 1.5], num_blocks=2, spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0])]
    torch.manual_seed(0)
    (_, me, mp), = MaskCollator(masks, [T], crop_size=S, patch_size=16)([(0, 0, [torch.arange(T)])] * B)
    clips = torch.randn(B, 3, T, S, S, generator=torch.Generator().manual_seed(1))
    loss = tr.train_step([clips.to(dev)], [[m.to(dev) for m in me]], [[m.to(dev) for m in mp]], 0.99925).item()
    ref = orc.OracleTrainer(enc_sd, pred_sd, dict(patch_size=16, tubelet_size=2, num_heads=6, depth=12, use_rope=True),
                            dict(num_heads=12, depth=2, use_rope=True, grid_size=S // 16, num_mask_tokens=2,
                                 num_patches=(T // 2) * (S // 16) ** 2))
    ref_loss = ref.step(clips, me, mp, 1e-4, 0.04, 0.99925)
    rel = abs(loss - ref_loss) / abs(ref_loss)
    w = enc.backbone.blocks[0].attn.qkv.weight.detach().cpu()
    w0 = enc_sd["blocks.0.attn.qkv.weight"]
    agree = (torch.sign(w - w0) == torch.sign(ref.enc["blocks.0.attn.qkv.weight"].detach() - w0)).float().mean().item()
    print(f"bf16 target residual={bf16_target} silu={silu}: loss {loss:.6f} vs oracle {ref_loss:.6f} (rel {rel:.2e}), "
          f"AdamW update sign agreement {agree:.4f}")
    assert rel < 1e-2
    assert agree > 0.9


def test_target_residual_precision_follows_mixed_precision(monkeypatch):
    """The target encoder's bf16 residual stream is the reference's autocast precision, so it is the
    default only under bf16 mixed precision: a float32 config (mixed_precision False, the reference
    runs forward_target in f32) keeps the residual in f32; VJ_TARGET_BF16=0 turns it off."""
    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model

    def trainer(mp):
        torch.manual_seed(239)
        enc, pred = init_video_model(device="cuda", patch_size=16, max_num_frames=4, tubelet_size=2,
                                     model_name="vit_small", crop_size=32, pred_depth=1, pred_num_heads=12,
                                     pred_embed_dim=384, use_mask_tokens=True, num_mask_tokens=2, use_rope=True)
        opt, _, _, _ = init_opt(enc, pred, iterations_per_epoch=1, start_lr=1e-4, ref_lr=1e-4, warmup=0,
                                num_epochs=1, mixed_precision=mp)
        return JEPATrainer(enc, pred, copy.deepcopy(enc), opt, mixed_precision=mp)

    monkeypatch.delenv("VJ_TARGET_BF16", raising=False)
    assert trainer(True).target_bf16_residual is True
    assert trainer(False).target_bf16_residual is False
    monkeypatch.setenv("VJ_TARGET_BF16", "0")
    assert trainer(True).target_bf16_residual is False


def test_two_fpc_groups_vs_oracle():
    """Several frames-per-clip groups in one step (data.dataset_fpcs with distinct values, e.g.
    [8, 4]): the MaskCollator yields one (clips, masks) entry per group; the reference runs the
    wrappers' per-group loop (wrappers.py:20-43, predictor mask_index = group) and averages the loss
    over every (group, mask) pair (train.py:425-435). HIP fused step vs the CPU oracle's
    loss_groups on the same weights / clips / masks: loss within 1e-2 relative, every parameter
    gradient within rel-L1 6e-2 of fp32 autograd (bf16 operands; a single group measures 3.4e-2 on
    this tiny config), unused mask tokens untouched. The 4-frame group has fewer tokens per clip than
    the model's 8-frame maximum: its loss rows index the target by the clip's own token count."""
    from vjepa2_amd.masks import MaskCollator
    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model

    dev = torch.device("cuda", 0)
    torch.manual_seed(239)
    S, B = 64, 2
    enc, pred = init_video_model(device=dev, patch_size=16, max_num_frames=8, tubelet_size=2, model_name="vit_small",
                                 crop_size=S, pred_depth=2, pred_num_heads=12, pred_embed_dim=384, uniform_power=True,
                                 use_mask_tokens=True, num_mask_tokens=4, zero_init_mask_tokens=False, use_sdpa=True,
                                 use_rope=True)
    enc_sd = {k: v.detach().cpu().clone() for k, v in enc.backbone.state_dict().items()}
    pred_sd = {k: v.detach().cpu().clone() for k, v in pred.backbone.state_dict().items()}
    tgt = copy.deepcopy(enc)
    opt, _, _, _ = init_opt(enc, pred, iterations_per_epoch=10, start_lr=1e-4, ref_lr=1e-4, warmup=0, num_epochs=1,
                            wd=0.04, final_wd=0.04, mixed_precision=True)
    for g in opt.param_groups:
        g["lr"] = 1e-4
        if not g.get("WD_exclude", False):
            g["weight_decay"] = 0.04
    tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True)
    masks = [dict(aspect_ratio=[0.75, 1.5], num_blocks=8, spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
             dict(aspect_ratio=[0.75, 1.5], num_blocks=2, spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0])]
    torch.manual_seed(0)
    batch = [(0, 0, [torch.arange(8)])] * B + [(0, 0, [torch.arange(4)])] * B
    groups = MaskCollator(masks, [8, 4], crop_size=S, patch_size=16)(batch)
    assert len(groups) == 2
    gen = torch.Generator().manual_seed(1)
    clips = [torch.randn(B, 3, T, S, S, generator=gen) for T in (8, 4)]
    tok0 = [t.detach().cpu().clone() for t in tr.mask_tokens]
    args = ([c.to(dev) for c in clips], [[m.to(dev) for m in g[1]] for g in groups],
            [[m.to(dev) for m in g[2]] for g in groups])

    def grads():
        torch.cuda.synchronize()
        d = {("enc", k): p.grad.detach().cpu().clone() for k, p in enc.backbone.named_parameters()}
        d.update({("pred", k): p.grad.detach().cpu().clone() for k, p in pred.backbone.named_parameters()
                  if p.grad is not None})
        return d

    # A first pass marks the weight-gradient outputs overwrite-on-first-write; after opt.zero_grad()
    # they still hold this pass's values, so the measured pass runs the lazy-zero paths across groups
    # (group 0 overwrites, group 1 accumulates). Its gradients must equal the first pass's bitwise.
    loss0 = tr.compute_grads(*args).item()
    first = grads()
    opt.zero_grad()
    loss = tr.compute_grads(*args).item()
    got = grads()
    assert loss == loss0
    for key, gk in got.items():
        assert torch.equal(gk, first[key]), f"{key}: gradient differs on the lazily zeroed pass"
    tr.apply_update(0.99925)
    ref = orc.OracleTrainer(enc_sd, pred_sd, dict(patch_size=16, tubelet_size=2, num_heads=6, depth=12, use_rope=True),
                            dict(num_heads=12, depth=2, use_rope=True, grid_size=S // 16, num_mask_tokens=4,
                                 num_patches=4 * (S // 16) ** 2))
    ref_loss_t = ref.loss_groups([(c, g[1], g[2]) for c, g in zip(clips, groups)])
    ref_loss_t.backward()
    ref_loss = ref_loss_t.item()
    rel = abs(loss - ref_loss) / abs(ref_loss)
    rep = [f"2 fpc groups: loss {loss:.6f} vs oracle {ref_loss:.6f} (rel {rel:.2e})"]
    assert rel < 1e-2, rep
    # gradients (before the optimizer) vs fp32 autograd of the oracle, bf16-operand envelope
    worst = 0.0
    for (which, k), gk in got.items():
        rp = (ref.enc if which == "enc" else ref.pred)[k]
        if rp.grad is None:
            assert gk.abs().max() == 0, f"{which}.{k}: gradient where the reference has none"
            continue
        e = ((gk - rp.grad).abs().sum() / rp.grad.abs().sum().clamp_min(1e-30)).item()
        worst = max(worst, e)
        if e > 4e-2:
            rep.append(f"{which}.{k}: rel_l1 {e:.3e}")
    rep.append(f"worst gradient rel_l1 {worst:.3e}")
    print("\n".join(rep))
    # bf16 operands on this tiny config (D = 384, <= 64 tokens per clip): one group alone measures a
    # worst gradient rel-L1 of 3.4e-2 against the same oracle (tools/debug_groups.py)
    assert worst < 6e-2, "\n".join(rep)
    # mask tokens 0 and 1 (one per group) took a step; tokens 2 and 3 (unused) did not move
    for i, t in enumerate(tr.mask_tokens):
        moved = not torch.equal(t.detach().cpu(), tok0[i])
        assert moved == (i < 2), f"mask token {i}: moved={moved}"
