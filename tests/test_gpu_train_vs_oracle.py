"""One fused V-JEPA train step (target fwd, context fwd+bwd, predictor fwd+bwd, loss, AdamW, EMA) on
the HIP kernels vs the fp32 CPU oracle trainer, with the target encoder's residual stream in bf16
(the trainer's default, the reference's autocast precision) and in f32. Same tiny config as the
driver's smoke check (vit_small, 8x64^2, B=2, predictor depth 2)."""
import copy

import pytest
import torch

from oracle import vjepa_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bf16_target", [True, False])
def test_train_step_vs_oracle(bf16_target):
    from vjepa2_amd.masks import MaskCollator
    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model

    dev = torch.device("cuda", 0)
    torch.manual_seed(239)
    T, S, B = 8, 64, 2
    enc, pred = init_video_model(device=dev, patch_size=16, max_num_frames=T, tubelet_size=2, model_name="vit_small",
                                 crop_size=S, pred_depth=2, pred_num_heads=12, pred_embed_dim=384, uniform_power=True,
                                 use_mask_tokens=True, num_mask_tokens=2, use_sdpa=True, use_rope=True)
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
    print(f"bf16 target residual={bf16_target}: loss {loss:.6f} vs oracle {ref_loss:.6f} (rel {rel:.2e}), "
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
