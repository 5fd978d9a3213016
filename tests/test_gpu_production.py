"""The production step pinned bitwise at the bench's own configuration.

bench.py times ViT-L/16 at 16x256^2 (24 blocks, RoPE, predictor 12x384, the two reference mask
configs) with the target-encoder side stream, the weight-gradient stream and the staged AdamW + EMA
issue all on. The kernels are deterministic (fixed-order reductions, no float atomics), so the
stream configuration must not change a single bit: a cross-stream ordering bug (a reader not waiting
for its producer) would show up here as a mismatch, where the tolerance tests could absorb it.

Three arms of 2 steps each (app/vjepa/train.py:409-471 per step), B = 4 clips:
  * serialised: VJ_TGT_STREAM=0 VJ_WGRAD_STREAM=0, one-pass update;
  * streams on, one-pass update (inputs_resident False);
  * streams on, staged update (inputs_resident True, as bench.py runs it).
Losses, every online arena (weights, gradients, AdamW moments, bf16 shadow) and the target arenas
(EMA weights, bf16 shadow) must be torch.equal across the three.
"""

import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

MASK_CFGS = [
    dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=8,
         spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
    dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=2,
         spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0]),
]


def _data(dev, B, T, S, steps):
    from vjepa2_amd.masks import MaskCollator

    torch.manual_seed(239)
    mc = MaskCollator(cfgs_mask=MASK_CFGS, dataset_fpcs=[T], crop_size=S, patch_size=16, tubelet_size=2)
    g = torch.Generator(device=dev).manual_seed(1000)
    out = []
    for _ in range(steps):
        (_, me, mp), = mc([(torch.zeros(1), 0, [torch.arange(T)]) for _ in range(B)])
        clips = torch.randn(B, 3, T, S, S, device=dev, generator=g)
        out.append(([clips], [[m.to(dev) for m in me]], [[m.to(dev) for m in mp]]))
    torch.cuda.synchronize()
    return out


def _run(dev, data, T, S, tgt_stream, wgrad_stream, staged):
    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model

    os.environ["VJ_TGT_STREAM"] = "1" if tgt_stream else "0"
    os.environ["VJ_WGRAD_STREAM"] = "1" if wgrad_stream else "0"
    torch.manual_seed(239)
    enc, pred = init_video_model(device=dev, patch_size=16, max_num_frames=T, tubelet_size=2, model_name="vit_large",
                                 crop_size=S, pred_depth=12, pred_num_heads=12, pred_embed_dim=384, uniform_power=True,
                                 use_mask_tokens=True, num_mask_tokens=6, zero_init_mask_tokens=True, use_sdpa=True,
                                 use_rope=True)
    tgt = copy.deepcopy(enc)
    opt, _, sched, wds = init_opt(enc, pred, iterations_per_epoch=300, start_lr=1e-4, ref_lr=5.25e-4, warmup=40,
                                  num_epochs=10, wd=0.04, final_wd=0.04, final_lr=5.25e-4, ipe_scale=1.25,
                                  mixed_precision=True)
    tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True, loss_exp=1.0)
    tr.inputs_resident = staged
    losses = []
    for clips, me, mp in data:
        sched.step()
        wds.step()
        losses.append(tr.train_step(clips, me, mp, 0.99925).clone())
    assert (tr._staged is not None) == staged
    torch.cuda.synchronize()
    state = []
    for a in tr.opt.arenas:
        state += [a.data.clone(), a.grad.clone(), a.exp_avg.clone(), a.exp_avg_sq.clone(), a.bf16.clone()]
    for a in tr.tgt_arenas:
        state += [a.data.clone(), a.bf16.clone()]
    out = (torch.stack(losses).cpu(), state)
    del tr, opt, enc, pred, tgt
    torch.cuda.empty_cache()
    return out


def test_production_step_bitwise_across_stream_configs():
    dev = torch.device("cuda", 0)
    T, S, B = 16, 256, 4
    data = _data(dev, B, T, S, steps=2)
    saved = {e: os.environ.get(e) for e in ("VJ_TGT_STREAM", "VJ_WGRAD_STREAM")}
    try:
        ser = _run(dev, data, T, S, False, False, False)
        par = _run(dev, data, T, S, True, True, False)
        stg = _run(dev, data, T, S, True, True, True)
    finally:
        for e, v in saved.items():
            if v is None:
                os.environ.pop(e, None)
            else:
                os.environ[e] = v
    assert torch.isfinite(ser[0]).all() and ser[0].min() > 0
    for name, arm in (("streams on", par), ("streams on + staged update", stg)):
        assert torch.equal(ser[0], arm[0]), (name, ser[0].tolist(), arm[0].tolist())
        assert len(ser[1]) == len(arm[1])
        for k, (x, y) in enumerate(zip(ser[1], arm[1])):
            assert torch.equal(x, y), f"{name}: state tensor {k} differs (max |d| {(x.float() - y.float()).abs().max().item()})"
