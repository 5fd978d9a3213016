"""GPU: the app-plugin boundary (app/vjepa/train.py:main, its checkpoints) and the standalone layer
modules, against fixtures the REFERENCE wrote (tests/golden/make_golden.py runs it on CPU, fp32).

 * main(args) at BASELINE configs[0] (ViT-S/16 8x128^2 B=2, seed 239, ipe 6) reproduces the
   reference's masks bit for bit and its loss trajectory within the bf16-operand envelope;
 * a checkpoint the reference's save_checkpoint wrote (train.py:315-333) resumes here: weights,
   target and the torch.optim.AdamW state (mapped into the flat arenas) give the reference's next
   step;
 * a checkpoint written here loads into the reference's layout (DDP + wrapper key prefixes, the
   4-group torch.optim.AdamW of app/vjepa/utils.py:224-239) with strict key matching;
 * RoPEAttention / Attention / MLP forward() (modules.py:77-83, 326-382, 408-429) are callable on
   their own and match the fp32 oracle in value and gradient.
"""

import copy
import os

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

from oracle import vjepa_oracle as orc  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


def gold(name):
    return torch.load(os.path.join(GOLD, name), weights_only=True)


def rel_l1(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().mean() / b.abs().mean().clamp_min(1e-12)).item()


# ------------------------------------------------------------------------------------------------
def test_main_matches_reference_trajectory(tmp_path, monkeypatch):
    from vjepa2_amd import train

    g = gold("main_vits.pt")
    args = copy.deepcopy(g["args"])
    args["folder"] = str(tmp_path)
    seen = []
    orig = train.init_data

    def init_data(**kw):  # record what the collator hands the step (masks are the bit-exact part)
        coll = kw["collator"]

        def rec(batch):
            s = coll(batch)
            seen.append(s)
            return s

        kw["collator"] = rec
        return orig(**kw)

    monkeypatch.setattr(train, "init_data", init_data)
    losses = train.main(args)
    assert len(losses) == len(g["losses"]) == 6
    rep = []
    from vjepa2_amd.masks import MaskSpec, materialize

    for i, (s, ref) in enumerate(zip(seen, g["samples"])):
        entry, = s
        assert all(isinstance(m, MaskSpec) for m in entry[1]), "main builds its masks on the GPU (data.gpu_masks)"
        batch, menc, mpred = materialize(entry, "cuda")  # the same device build the step consumed
        assert abs(batch[0][0].double().sum().item() - float(ref["clip_sum"])) < 1e-3, f"clips of step {i}"
        for a, b in zip(menc + mpred, ref["enc"] + ref["pred"]):
            assert torch.equal(a.cpu(), b), f"masks of step {i} differ from the reference's"
    for i, (l, r) in enumerate(zip(losses, g["losses"])):
        e = abs(l - r) / abs(r)
        rep.append(f"step {i}: loss {l:.6f} reference {r:.6f} rel {e:.2e}")
    print("\n".join(rep))
    # bf16 GEMM / attention operands vs the reference's fp32 CPU run, 12 + 12 blocks
    assert all(abs(l - r) / abs(r) < 3e-3 for l, r in zip(losses, g["losses"])), "\n".join(rep)
    # the app's side effects: per-rank CSV log and the train.py:315-333 checkpoint
    log = (tmp_path / "log_r0.csv").read_text().strip().splitlines()
    assert len(log) == 6
    ck = torch.load(tmp_path / "latest.pt", map_location="cpu", weights_only=True)
    assert set(ck) == {"encoder", "predictor", "opt", "scaler", "target_encoder", "epoch", "loss", "batch_size",
                       "world_size", "lr"} and ck["epoch"] == 1


def _micro_models():
    from vjepa2_amd import vision_transformer as vt
    from vjepa2_amd.train import init_video_model

    vt.vit_micro = lambda patch_size=16, **kw: vt.VisionTransformer(
        patch_size=patch_size, embed_dim=64, depth=2, num_heads=1, mlp_ratio=4, qkv_bias=True,
        norm_layer=lambda d: nn.LayerNorm(d, eps=1e-6), **kw)
    torch.manual_seed(239)
    return init_video_model(device=DEV, patch_size=16, max_num_frames=8, tubelet_size=2, model_name="vit_micro",
                            crop_size=64, pred_depth=2, pred_num_heads=2, pred_embed_dim=64, uniform_power=True,
                            use_mask_tokens=True, num_mask_tokens=2, zero_init_mask_tokens=True, use_sdpa=True,
                            use_rope=True)


def test_resume_from_reference_checkpoint(tmp_path):
    """The reference's epoch-1 checkpoint (encoder, predictor, target, torch.optim.AdamW state in its
    own numbering) resumed here; the next step matches the reference's loss and weight update."""
    from vjepa2_amd.train import JEPATrainer, init_opt, load_checkpoint

    r = gold("ref_resume.pt")
    co = r["args"]["optimization"]
    enc, pred = _micro_models()
    tgt = copy.deepcopy(enc)
    opt, scaler, sched, wds = init_opt(enc, pred, iterations_per_epoch=co["ipe"], start_lr=co["start_lr"],
                                       ref_lr=co["lr"], warmup=co["warmup"], num_epochs=co["epochs"],
                                       wd=co["weight_decay"], final_wd=co["final_weight_decay"],
                                       final_lr=co["final_lr"], ipe_scale=co["ipe_scale"])
    tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=False, loss_exp=1.0)
    path = tmp_path / "latest.pt"
    torch.save(r["ckpt"], path)
    *_, epoch = load_checkpoint(str(path), enc, pred, tgt, opt, scaler, trainer=tr)
    assert epoch == 1
    sd = opt.state_dict()
    ro = r["ckpt"]["opt"]
    assert sorted(sd["state"]) == sorted(ro["state"])
    for k in ro["state"]:  # the reference's moments, by the reference's numbering, round-trip exactly
        assert torch.equal(sd["state"][k]["exp_avg"], ro["state"][k]["exp_avg"])
        assert float(sd["state"][k]["step"]) == float(ro["state"][k]["step"])
    for _ in range(epoch * co["ipe"]):  # train.py:309-313 replays the schedulers
        sched.step()
        wds.step()
    lr, wd = sched.step(), wds.step()
    assert abs(lr - r["lr"]) < 1e-12 and abs(wd - r["wd"]) < 1e-12
    s = r["sample"]
    clips = torch.stack([torch.randn(3, 8, 64, 64, generator=torch.Generator().manual_seed(sd_))
                         for sd_ in s["clip_seeds"]])
    before = {k: v.detach().cpu().clone() for k, v in enc.backbone.state_dict().items()}
    before_p = {k: v.detach().cpu().clone() for k, v in pred.backbone.state_dict().items()}
    loss = tr.train_step([clips.to(DEV)], [[m.to(DEV) for m in s["enc"]]], [[m.to(DEV) for m in s["pred"]]],
                         co["ema"][0]).item()
    e = abs(loss - r["loss"]) / r["loss"]
    rep = [f"resumed step loss {loss:.6f} vs reference {r['loss']:.6f} (rel {e:.1e})"]
    assert e < 3e-3, rep
    # the update of this step uses the checkpoint's Adam moments (3 steps of history), so it is
    # well conditioned: compare it directly (bf16-operand gradients -> a few % of the update)
    worst = 0.0
    for name, mod, b0, ref in (("encoder", enc.backbone, before, r["after"]["encoder"]),
                               ("predictor", pred.backbone, before_p, r["after"]["predictor"])):
        cur = mod.state_dict()
        for n, v in ref.items():
            dr = v - b0[n]
            du = cur[n].cpu() - b0[n]
            if dr.abs().max() == 0:
                assert du.abs().max() == 0, f"{name}.{n} moved but the reference's did not"
                continue
            if n.endswith("attn.qkv.bias"):  # key-bias gradient is 0 in exact arithmetic (softmax shift)
                d = du.numel() // 3
                du, dr = torch.cat([du[:d], du[2 * d:]]), torch.cat([dr[:d], dr[2 * d:]])
            err = rel_l1(du, dr)
            worst = max(worst, err)
            rep.append(f"{name}.{n}: update rel_l1 {err:.2e}")
    print("\n".join(rep))
    assert worst < 0.1, "\n".join(rep)


class _DDP(nn.Module):
    """Key layout of the reference's DistributedDataParallel(MultiSeqWrapper(model)): module.backbone.*"""

    def __init__(self, m):
        super().__init__()
        self.module = m


def _reference_adamw(encoder, predictor):
    """app/vjepa/utils.py:224-239 restated."""
    groups = [
        {"params": [p for n, p in encoder.named_parameters() if ("bias" not in n) and (len(p.shape) != 1)]},
        {"params": [p for n, p in predictor.named_parameters() if ("bias" not in n) and (len(p.shape) != 1)]},
        {"params": [p for n, p in encoder.named_parameters() if ("bias" in n) or (len(p.shape) == 1)],
         "WD_exclude": True, "weight_decay": 0},
        {"params": [p for n, p in predictor.named_parameters() if ("bias" in n) or (len(p.shape) == 1)],
         "WD_exclude": True, "weight_decay": 0},
    ]
    return torch.optim.AdamW(groups, betas=(0.9, 0.999), eps=1e-8)


def test_checkpoint_loads_into_reference_layout(tmp_path):
    """A checkpoint written here, loaded the way the reference's load_checkpoint does
    (app/vjepa/utils.py:90-135: strict load_state_dict of DDP-wrapped models, opt.load_state_dict)."""
    from vjepa2_amd.masks import MaskCollator
    from vjepa2_amd.train import JEPATrainer, init_opt, save_checkpoint
    from vjepa2_amd.wrappers import MultiSeqWrapper, PredictorMultiSeqWrapper

    enc, pred = _micro_models()
    tgt = copy.deepcopy(enc)
    opt, scaler, sched, wds = init_opt(enc, pred, iterations_per_epoch=3, start_lr=1e-4, ref_lr=5e-4, warmup=1,
                                       num_epochs=1, wd=0.04, final_wd=0.04, mixed_precision=True)
    tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True)
    mcfg = [dict(aspect_ratio=[0.75, 1.5], num_blocks=8, spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
            dict(aspect_ratio=[0.75, 1.5], num_blocks=2, spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0])]
    coll = MaskCollator(mcfg, [8], crop_size=64, patch_size=16)
    for i in range(2):
        (_, me, mp), = coll([(0, 0, [torch.arange(8)])] * 2)
        clips = torch.randn(2, 3, 8, 64, 64, generator=torch.Generator().manual_seed(i))
        sched.step()
        wds.step()
        tr.train_step([clips.to(DEV)], [[m.to(DEV) for m in me]], [[m.to(DEV) for m in mp]], 0.99925)
    path = str(tmp_path / "latest.pt")
    save_checkpoint(path, enc, pred, tgt, opt, scaler, epoch=1, loss=0.5, batch_size=2, world_size=1, lr=5e-4)
    if os.environ.get("VJ_CKPT_OUT"):  # for tests/golden/check_reference_load.py (run where the reference is)
        import shutil

        os.makedirs(os.path.dirname(os.environ["VJ_CKPT_OUT"]), exist_ok=True)
        shutil.copy(path, os.environ["VJ_CKPT_OUT"])
    ck = torch.load(path, map_location="cpu", weights_only=True)
    # the reference's side, on CPU: fresh modules of the same architecture, DDP-style key prefixes
    from vjepa2_amd import vision_transformer as vt
    from vjepa2_amd.predictor import vit_predictor

    e2 = _DDP(MultiSeqWrapper(vt.vit_micro(img_size=64, num_frames=8, tubelet_size=2, use_rope=True,
                                           uniform_power=True)))
    p2 = _DDP(PredictorMultiSeqWrapper(vit_predictor(img_size=64, use_mask_tokens=True, patch_size=16, num_frames=8,
                                                     tubelet_size=2, embed_dim=64, predictor_embed_dim=64, depth=2,
                                                     num_heads=2, uniform_power=True, num_mask_tokens=2,
                                                     use_rope=True)))
    t2 = _DDP(MultiSeqWrapper(vt.vit_micro(img_size=64, num_frames=8, tubelet_size=2, use_rope=True,
                                           uniform_power=True)))
    e2.load_state_dict(ck["encoder"])  # strict: every key present, no extras
    p2.load_state_dict(ck["predictor"])
    t2.load_state_dict(ck["target_encoder"])
    ropt = _reference_adamw(e2.module, p2.module)
    ropt.load_state_dict(ck["opt"])
    for (n, p), q in zip(enc.named_parameters(), e2.module.parameters()):
        assert torch.equal(p.detach().cpu(), q.detach()), n
    # the loaded torch.optim state sits on the right parameters: moments have each parameter's shape
    # and equal the arena moments of the parameter with the same name
    ours = {n: p for n, p in list(enc.named_parameters()) + [("p." + n, p) for n, p in pred.named_parameters()]}
    theirs = list(e2.module.named_parameters()) + [("p." + n, p) for n, p in p2.module.named_parameters()]
    checked = 0
    for n, q in theirs:
        st = ropt.state.get(q)
        if not st:
            continue
        a = next(a for a in opt.arenas if any(x is ours[n] for x in a.params))
        o, k = a.segment(ours[n])
        assert st["exp_avg"].shape == q.shape, n
        assert torch.equal(st["exp_avg"].reshape(-1), a.exp_avg[o:o + k].cpu()), n
        checked += 1
    assert checked >= 30


# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("rope,mask", [(True, True), (True, False), (False, False)])
def test_attention_module_forward(rope, mask):
    """RoPEAttention.forward / Attention.forward on their own: fwd + input / parameter grads vs the
    fp32 oracle (oracle.attention = modules.py:326-382 / 408-429 restated)."""
    from vjepa2_amd.modules import Attention, RoPEAttention

    torch.manual_seed(5)
    dim, H, B, N, grid = 128, 2, 2, 40, 4
    m = (RoPEAttention(dim, num_heads=H, qkv_bias=True, grid_size=grid) if rope else
         Attention(dim, num_heads=H, qkv_bias=True))
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.05 * torch.randn_like(p))
    sd = {"attn." + k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    x = torch.randn(B, N, dim)
    ids = torch.stack([torch.randperm(grid * grid * 4)[:N].sort().values for _ in range(B)]) if mask else None
    xd = x.to(DEV).requires_grad_(True)
    y = m(xd, mask=ids.to(DEV) if mask else None)
    gy = torch.randn(B, N, dim)
    y.backward(gy.to(DEV))
    xr = x.clone().requires_grad_(True)
    sdr = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    yr = orc.attention(xr, sdr, "attn.", H, ids=ids, tokens_per_frame=grid * grid, tokens_per_row=grid,
                       use_rope=rope)
    yr.backward(gy)
    rep = [f"y rel_l1 {rel_l1(y, yr):.2e}", f"dx rel_l1 {rel_l1(xd.grad, xr.grad):.2e}"]
    assert rel_l1(y, yr) < 1e-2 and rel_l1(xd.grad, xr.grad) < 2e-2, rep
    for n, p in m.named_parameters():
        e = rel_l1(p.grad, sdr["attn." + n].grad)
        rep.append(f"d{n} rel_l1 {e:.2e}")
        assert e < 3e-2, rep
    print("\n".join(rep))


def test_mlp_module_forward():
    from vjepa2_amd.modules import MLP

    torch.manual_seed(6)
    m = MLP(96, 384)
    x = torch.randn(3, 50, 96)
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    y = m(xd)
    gy = torch.randn_like(x)
    y.backward(gy.to(DEV))
    xr = x.clone().requires_grad_(True)
    yr = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(xr, sd["fc1.weight"],
                                                                                          sd["fc1.bias"])),
                                    sd["fc2.weight"], sd["fc2.bias"])
    yr.backward(gy)
    assert rel_l1(y, yr) < 1e-2 and rel_l1(xd.grad, xr.grad) < 2e-2
    for n, p in m.named_parameters():
        assert rel_l1(p.grad, sd[n].grad) < 3e-2, n
