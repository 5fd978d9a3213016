"""Debug: two frames-per-clip groups, our grads vs the oracle's per-group grads."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vjepa_oracle as orc  # noqa: E402
from vjepa2_amd.masks import MaskCollator  # noqa: E402
from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model  # noqa: E402

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
tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True)
masks = [dict(aspect_ratio=[0.75, 1.5], num_blocks=8, spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
         dict(aspect_ratio=[0.75, 1.5], num_blocks=2, spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0])]
torch.manual_seed(0)
batch = [(0, 0, [torch.arange(8)])] * B + [(0, 0, [torch.arange(4)])] * B
groups = MaskCollator(masks, [8, 4], crop_size=S, patch_size=16)(batch)
gen = torch.Generator().manual_seed(1)
clips = [torch.randn(B, 3, T, S, S, generator=gen) for T in (8, 4)]


def ours(sel):
    for a in opt.arenas:
        a.grad.zero_()
        a.epoch += 1
    for a in opt.arenas:
        for p in a.params:
            p._vj_gepoch = a.epoch
    loss = tr.compute_grads([clips[i].to(dev) for i in sel], [[m.to(dev) for m in groups[i][1]] for i in sel],
                            [[m.to(dev) for m in groups[i][2]] for i in sel]).item()
    torch.cuda.synchronize()
    return loss, {k: p.grad.detach().cpu().clone() for k, p in enc.backbone.named_parameters()}


def oracle(sel, mask_index=None, norm=None):
    ref = orc.OracleTrainer(enc_sd, pred_sd, dict(patch_size=16, tubelet_size=2, num_heads=6, depth=12, use_rope=True),
                            dict(num_heads=12, depth=2, use_rope=True, grid_size=S // 16, num_mask_tokens=4,
                                 num_patches=4 * (S // 16) ** 2))
    gs = [(clips[i], groups[i][1], groups[i][2]) for i in range(2)]
    tot, n = 0.0, 0
    for j, i in enumerate(sel):
        c, me, mp = gs[i]
        with torch.no_grad():
            h = orc.forward_target(c, ref.tgt, ref.enc_cfg)
        z = [orc.encoder_forward(c, ref.enc, ref.enc_cfg, masks=m) for m in me]
        mi = j if mask_index is None else mask_index
        z = [orc.predictor_forward(zi, mx, my, ref.pred, ref.pred_cfg, mask_index=mi) for zi, mx, my in zip(z, me, mp)]
        tot = tot + orc.jepa_loss(z, h, mp, 1.0) * len(me)
        n += len(me)
    loss = tot / n
    loss.backward()
    return loss.item(), {k: v.grad.clone() for k, v in ref.enc.items() if v.grad is not None}


def rl(a, b):
    return ((a - b).abs().sum() / b.abs().sum()).item()


keys = ("blocks.0.attn.qkv.weight", "blocks.5.mlp.fc1.weight", "patch_embed.proj.bias")
for name, s2 in [("[0,1]", [0, 1]), ("[1,0]", [1, 0]), ("[0]", [0]), ("[1]", [1]), ("[0,0]", [0, 0]), ("[1,1]", [1, 1])]:
    lo, go = ours(s2)
    lr_, gr = oracle(s2)
    print(f"groups {name}: ours loss {lo:.6f} oracle {lr_:.6f}: grad rel_l1 {[round(rl(go[k], gr[k]), 4) for k in keys]}")
