"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

This script is the only place the reference (weipeilun/vjepa2, mounted read-only at
/root/reference) is executed. It runs on CPU, fp32, in the build container only; the fixtures it
writes are plain tensors (torch.save of dicts of tensors / python scalars, loaded back with
``torch.load(..., weights_only=True)``). No reference source is copied: only inputs and outputs.

Stubs: ``timm.models.layers.drop_path`` (timm's published algorithm restated; inert at
drop_path_rate=0, which every fixture but gen_block_variants' uses) and
``app.vjepa.transforms.make_transforms`` (torchvision absent; synthetic clips need no augmentation).

Usage:  python tests/golden/make_golden.py            (writes tests/golden/*.pt)
"""

import copy
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
REF = os.environ.get("VJEPA_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

import torch  # noqa: E402

# ---- stubs -------------------------------------------------------------------------------
timm = types.ModuleType("timm")
timm_models = types.ModuleType("timm.models")
timm_layers = types.ModuleType("timm.models.layers")


_DP = {"gen": None, "log": []}  # drop_path draws: seeded generator, and every draw made (fixture data)


def _drop_path(x, drop_prob=0.0, training=False, scale_by_keep=True):
    """timm.layers.drop_path (timm 0.9.x; absent here), restated: per-sample Bernoulli(keep) mask,
    scaled by 1 / keep. Inert at rate 0 / eval (every fixture but the drop_path blocks)."""
    if drop_prob == 0.0 or not training:
        return x
    keep_prob = 1 - drop_prob
    shape = (x.shape[0],) + (1,) * (x.ndim - 1)
    random_tensor = x.new_empty(shape).bernoulli_(keep_prob, generator=_DP["gen"])
    if keep_prob > 0.0 and scale_by_keep:
        random_tensor.div_(keep_prob)
    _DP["log"].append(random_tensor.flatten().clone())
    return x * random_tensor


timm_layers.drop_path = _drop_path
timm.models = timm_models
timm_models.layers = timm_layers
sys.modules.update({"timm": timm, "timm.models": timm_models, "timm.models.layers": timm_layers})
sys.path.insert(0, REF)
tr_mod = types.ModuleType("app.vjepa.transforms")
tr_mod.make_transforms = lambda **kw: (lambda x: x)
sys.modules["app.vjepa.transforms"] = tr_mod

from src.models.utils.modules import Block, rotate_queries_or_keys  # noqa: E402
from src.models.utils.pos_embs import get_3d_sincos_pos_embed  # noqa: E402
import src.models.vision_transformer as vit  # noqa: E402
import src.models.predictor as vpred  # noqa: E402
from src.masks.multiseq_multiblock3d import MaskCollator  # noqa: E402
from src.masks.utils import apply_masks  # noqa: E402

torch.set_num_threads(8)


def save(name, d):
    path = os.path.join(OUT, name)
    torch.save(d, path)
    print(f"wrote {path} ({os.path.getsize(path)/1e3:.1f} kB)")


def sorted_unique_rows(B, K, N, g):
    return torch.stack([torch.randperm(N, generator=g)[:K].sort().values for _ in range(B)])


def grads_of(module):
    return {n: p.grad.detach().clone() for n, p in module.named_parameters() if p.grad is not None}


def gen_rope():
    g = torch.Generator().manual_seed(1)
    out = {}
    for s in (20, 10):  # encoder (hd=64 -> 20-wide slices) and predictor (hd=32 -> 10-wide)
        x = torch.randn(2, 3, 7, s, generator=g)
        pos = torch.randint(0, 8, (2, 3, 7), generator=g)
        out[f"x{s}"], out[f"pos{s}"] = x, pos
        out[f"out{s}"] = rotate_queries_or_keys(x, pos=pos)
    x = torch.randn(1, 2, 6, 20, generator=g)
    pos = torch.arange(6) // 2
    out["x_flat"], out["pos_flat"], out["out_flat"] = x, pos, rotate_queries_or_keys(x, pos=pos)
    save("rope.pt", out)


def gen_sincos():
    out = {}
    for up in (False, True):
        t = get_3d_sincos_pos_embed(96, 4, 2, cls_token=False, uniform_power=up)
        out[f"f64_up{int(up)}"] = torch.from_numpy(t)
    save("sincos.pt", out)


def gen_block(name, dim, heads, grid, T, N, K, with_thw, seed):
    torch.manual_seed(seed)
    blk = Block(dim=dim, num_heads=heads, mlp_ratio=4.0, qkv_bias=True, use_rope=True, grid_size=grid,
                norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6), use_sdpa=True)
    for p in blk.parameters():  # non-trivial LN/bias values
        with torch.no_grad():
            p.add_(0.05 * torch.randn_like(p))
    g = torch.Generator().manual_seed(seed + 1)
    B = 2
    x = torch.randn(B, K, dim, generator=g, requires_grad=True)
    mask = sorted_unique_rows(B, K, N, g)
    kw = dict(T=T, H_patches=grid, W_patches=grid) if with_thw else {}
    y = blk(x, mask=mask, **kw)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy)
    save(name, dict(state={k: v.detach().clone() for k, v in blk.state_dict().items()}, x=x.detach(),
                    mask=mask, y=y.detach(), gy=gy, gx=x.grad.detach(), gparams=grads_of(blk),
                    cfg=dict(dim=dim, heads=heads, grid=grid, T=T, with_thw=with_thw)))


def gen_block_variants():
    """Block variants the shipped configs leave off: SwiGLU MLP (act_layer=nn.SiLU -> SwiGLUFFN,
    modules.py:86-106, wide / narrow hidden) and stochastic depth (drop_path > 0, modules.py:546-562),
    in training mode; the per-sample drop_path draws (attn branch, then MLP branch) are saved."""
    for name, act, wide, dp, B, seed in (("block_swiglu.pt", torch.nn.SiLU, True, 0.0, 2, 11),
                                         ("block_droppath.pt", torch.nn.GELU, True, 0.5, 4, 12),
                                         ("block_swiglu_dp.pt", torch.nn.SiLU, False, 0.4, 4, 14)):
        torch.manual_seed(seed)
        blk = Block(dim=64, num_heads=2, mlp_ratio=4.0, qkv_bias=True, use_rope=True, grid_size=4, act_layer=act,
                    wide_silu=wide, drop_path=dp, norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6), use_sdpa=True)
        for p in blk.parameters():
            with torch.no_grad():
                p.add_(0.05 * torch.randn_like(p))
        g = torch.Generator().manual_seed(seed + 1)
        x = torch.randn(B, 10, 64, generator=g, requires_grad=True)
        mask = sorted_unique_rows(B, 10, 32, g)
        _DP["gen"], _DP["log"] = torch.Generator().manual_seed(seed + 2), []
        y = blk(x, mask=mask, T=2, H_patches=4, W_patches=4)
        draws = list(_DP["log"])
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy)
        save(name, dict(state={k: v.detach().clone() for k, v in blk.state_dict().items()}, x=x.detach(),
                        mask=mask, y=y.detach(), gy=gy, gx=x.grad.detach(), gparams=grads_of(blk),
                        draws=draws, cfg=dict(dim=64, heads=2, grid=4, T=2, silu=act is torch.nn.SiLU,
                                              wide_silu=wide, drop_path=dp, seed=seed)))


def gen_encoder():
    for use_rope in (True, False):
        torch.manual_seed(7)
        enc = vit.VisionTransformer(img_size=32, patch_size=16, num_frames=4, tubelet_size=2, embed_dim=64,
                                    depth=2, num_heads=1, mlp_ratio=4, qkv_bias=True, use_rope=use_rope,
                                    uniform_power=True, norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6))
        g = torch.Generator().manual_seed(8)
        x = torch.randn(2, 3, 4, 32, 32, generator=g)
        N = 2 * 2 * 2
        masks = [sorted_unique_rows(2, 5, N, g), sorted_unique_rows(2, 3, N, g)]
        full = enc(x)
        outs = [enc(x, masks=m) for m in masks]
        gys = [torch.randn(o.shape, generator=g) for o in outs]
        sum((o * gy).sum() for o, gy in zip(outs, gys)).backward()
        save(f"encoder_rope{int(use_rope)}.pt",
             dict(state={k: v.clone() for k, v in enc.state_dict().items()}, x=x, masks=masks, full=full.detach(),
                  outs=[o.detach() for o in outs], gys=gys, gparams=grads_of(enc)))


def gen_vitl_autocast():
    """The reference ViT-L/16 (vision_transformer.py:275 vit_large, RoPE, uniform_power) at 16 frames of
    64^2 (N = 128 tokens, one clip), seeded init, run twice on the same input: in fp32 and under
    torch.autocast("cpu", bfloat16) (the reference's own bf16 precision: bf16 Linear / SDPA operands,
    RoPE angles in bf16, LayerNorm in f32). Stores the seed, the input, both outputs and per-tensor
    sums of the initial weights (the GPU test rebuilds the same weights from the seed and checks them
    against these sums before comparing outputs): no weights in the fixture."""
    seed = 239
    torch.manual_seed(seed)
    enc = vit.vit_large(img_size=64, num_frames=16, tubelet_size=2, use_rope=True, uniform_power=True,
                        use_sdpa=True)
    enc.eval()
    g = torch.Generator().manual_seed(240)
    x = torch.randn(1, 3, 16, 64, 64, generator=g)
    mask = sorted_unique_rows(1, 48, 128, g)  # a context pass: 48 kept tokens of 128
    with torch.no_grad():
        full32 = enc(x)
        ctx32 = enc(x, masks=[mask])
        with torch.autocast("cpu", dtype=torch.bfloat16):
            full16 = enc(x)
            ctx16 = enc(x, masks=[mask])
    sums = {k: float(v.double().sum()) for k, v in enc.state_dict().items()}
    save("vitl_autocast.pt", dict(seed=seed, x=x, mask=mask, full_f32=full32, ctx_f32=ctx32,
                                  full_bf16=full16.float(), ctx_bf16=ctx16.float(), param_sums=sums,
                                  cfg=dict(model="vit_large", img_size=64, num_frames=16, tubelet_size=2)))


def gen_predictor():
    torch.manual_seed(11)
    pred = vpred.vit_predictor(img_size=32, use_mask_tokens=True, patch_size=16, num_frames=4, tubelet_size=2,
                               embed_dim=128, predictor_embed_dim=96, depth=2, num_heads=3, uniform_power=True,
                               num_mask_tokens=2, zero_init_mask_tokens=False, use_rope=True)
    g = torch.Generator().manual_seed(12)
    N = 8
    B = 2
    outs, gys, ins = [], [], []
    for K, Kp, midx in ((3, 4, 0), (5, 2, 1)):
        perm = [torch.randperm(N, generator=g) for _ in range(B)]
        mx = torch.stack([p[:K].sort().values for p in perm])
        my = torch.stack([p[K:K + Kp].sort().values for p in perm])
        z = torch.randn(B, K, 128, generator=g, requires_grad=True)
        o = pred(z, mx, my, mask_index=midx)
        gy = torch.randn(o.shape, generator=g)
        (o * gy).sum().backward()
        ins.append(dict(z=z.detach(), mx=mx, my=my, mask_index=midx, gz=z.grad.detach()))
        outs.append(o.detach())
        gys.append(gy)
    save("predictor.pt", dict(state={k: v.clone() for k, v in pred.state_dict().items()}, ins=ins, outs=outs,
                              gys=gys, gparams=grads_of(pred)))


VITL_MASKS = [
    dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=8,
         spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
    dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=2,
         spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0]),
]


def gen_masks():
    out = {}
    for tag, crop, fpc, B in (("vitl", 256, 16, 4), ("small", 128, 8, 2)):
        torch.manual_seed(239)
        mc = MaskCollator(cfgs_mask=VITL_MASKS, dataset_fpcs=[fpc], crop_size=crop, patch_size=16, tubelet_size=2)
        its = []
        for itr in range(3):
            batch = [(torch.zeros(1), 0, [torch.arange(fpc)]) for _ in range(B)]
            (_, menc, mpred), = mc(batch)
            its.append(dict(enc=menc, pred=mpred))
        out[tag] = dict(crop=crop, fpc=fpc, B=B, iters=its)
    # extra generator options: max_keep, full_complement, pred_full_complement, inv_block, temporal keep
    extras = {}
    for name, over in (("max_keep", dict(max_keep=20)), ("full_complement", dict(full_complement=True)),
                       ("pred_full_complement", dict(pred_full_complement=True)), ("inv_block", dict(inv_block=True)),
                       ("temporal", dict(max_temporal_keep=0.5, temporal_scale=[0.5, 1.0]))):
        cfg = dict(VITL_MASKS[0], **over)
        torch.manual_seed(5)
        mc = MaskCollator(cfgs_mask=[cfg], dataset_fpcs=[8], crop_size=64, patch_size=16, tubelet_size=2)
        batch = [(torch.zeros(1), 0, [torch.arange(8)]) for _ in range(3)]
        (_, menc, mpred), = mc(batch)
        extras[name] = dict(cfg=cfg, enc=menc, pred=mpred)
    out["extras"] = extras
    save("masks.pt", out)


def gen_train_steps():
    """Run the reference app/vjepa/train.py:main for 3 iterations on a micro model (CPU, fp32)."""
    _train_steps(bf16=False)


def gen_train_steps_bf16():
    """The same 3 iterations of the reference's main() run inside torch.autocast("cpu", bfloat16): the
    reference's own bf16 training precision (Linear / SDPA operands bf16, LayerNorm f32). Only the
    losses and final weights are stored (train_steps_bf16.pt); the GPU test reads its update envelope
    against the fp32 run (train_steps.pt)."""
    _train_steps(bf16=True)


def _train_steps(bf16):
    import torch.distributed as dist
    import app.vjepa.train as rtrain

    def vit_micro(patch_size=16, **kw):
        return vit.VisionTransformer(patch_size=patch_size, embed_dim=64, depth=2, num_heads=1, mlp_ratio=4,
                                     qkv_bias=True, norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6), **kw)

    vit.vit_micro = vit_micro
    B, fpc, crop = 2, 8, 64
    captured = dict(samples=[], losses=[])

    class SynthClips(torch.utils.data.Dataset):
        def __len__(self):
            return 1000

        def __getitem__(self, i):
            clip = torch.randn(3, fpc, crop, crop, generator=torch.Generator().manual_seed(1000 + i))
            return [clip], 0, [torch.arange(fpc)]

    def init_data(batch_size, collator=None, **kw):
        def collate(batch):
            s = collator(batch)
            captured["samples"].append(s)
            return s

        dl = torch.utils.data.DataLoader(SynthClips(), batch_size=batch_size, collate_fn=collate, shuffle=False,
                                         num_workers=0)
        sampler = types.SimpleNamespace(set_epoch=lambda e: None)
        return dl, sampler

    orig_init_opt = rtrain.init_opt

    def init_opt(encoder, predictor, **kw):
        captured["init_encoder"] = {k: v.clone() for k, v in encoder.backbone.state_dict().items()}
        captured["init_predictor"] = {k: v.clone() for k, v in predictor.backbone.state_dict().items()}
        return orig_init_opt(encoder=encoder, predictor=predictor, **kw)

    def gpu_timer(closure, log_timings=True):
        res = closure()
        captured["losses"].append(res[0])
        captured.setdefault("lrs", []).append(res[1])
        captured.setdefault("wds", []).append(res[2])
        return res, 0.0

    rtrain.init_data = init_data
    rtrain.init_opt = init_opt
    rtrain.gpu_timer = gpu_timer
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", rank=0, world_size=1)
    folder = tempfile.mkdtemp(prefix="vjepa_golden_")
    args = dict(
        folder=folder,
        meta=dict(dtype="float32", seed=239, use_sdpa=True, load_checkpoint=False, save_every_freq=-1),
        mask=VITL_MASKS,
        model=dict(model_name="vit_micro", pred_depth=2, pred_embed_dim=64, pred_num_heads=2, uniform_power=True,
                   use_activation_checkpointing=False, use_mask_tokens=True, use_rope=True,
                   zero_init_mask_tokens=True),
        data=dict(batch_size=B, crop_size=crop, patch_size=16, dataset_fpcs=[fpc], tubelet_size=2, fps=4,
                  num_workers=0),
        data_aug=dict(),
        loss=dict(loss_exp=1.0),
        optimization=dict(ema=[0.99925, 0.99925], epochs=1, final_lr=0.000525, final_weight_decay=0.04, ipe=3,
                          ipe_scale=1.25, lr=0.000525, start_lr=0.0001, warmup=1, weight_decay=0.04),
    )
    if bf16:
        with torch.autocast("cpu", dtype=torch.bfloat16):
            rtrain.main(args)
    else:
        rtrain.main(args)
    ck = torch.load(os.path.join(folder, "latest.pt"), map_location="cpu", weights_only=False)  # own file

    def strip(sd):
        return {k.replace("module.backbone.", ""): v.clone() for k, v in sd.items()}

    if bf16:
        save("train_steps_bf16.pt", dict(losses=captured["losses"], final_encoder=strip(ck["encoder"]),
                                         final_predictor=strip(ck["predictor"]),
                                         final_target=strip(ck["target_encoder"])))
        return

    samples = []
    for s in captured["samples"][:3]:
        (batch, menc, mpred), = s
        # clips are regenerated from their seeds (1000 + item index); keep a checksum to pin them
        samples.append(dict(clip_seeds=[1000 + B * len(samples) + j for j in range(B)],
                            clip_sum=batch[0][0].double().sum(), enc=menc, pred=mpred))
    save("train_steps.pt", dict(args=args, init_encoder=captured["init_encoder"],
                                init_predictor=captured["init_predictor"], samples=samples,
                                losses=captured["losses"], lrs=captured["lrs"], wds=captured["wds"],
                                final_encoder=strip(ck["encoder"]), final_predictor=strip(ck["predictor"]),
                                final_target=strip(ck["target_encoder"])))


def _run_reference_main(args, B, fpc, crop, captured, snapshot_iter=None):
    """app/vjepa/train.py:main on synthetic clips (seed 1000 + item index), CPU fp32. Records the
    collated samples, per-iteration loss / lr / wd, and (optionally) the encoder / predictor weights
    right after iteration `snapshot_iter`."""
    import torch.distributed as dist
    import app.vjepa.train as rtrain

    class SynthClips(torch.utils.data.Dataset):
        def __len__(self):
            return 1000

        def __getitem__(self, i):
            clip = torch.randn(3, fpc, crop, crop, generator=torch.Generator().manual_seed(1000 + i))
            return [clip], 0, [torch.arange(fpc)]

    def init_data(batch_size, collator=None, **kw):
        def collate(batch):
            s = collator(batch)
            captured["samples"].append(s)
            return s

        dl = torch.utils.data.DataLoader(SynthClips(), batch_size=batch_size, collate_fn=collate, shuffle=False,
                                         num_workers=0)
        return dl, types.SimpleNamespace(set_epoch=lambda e: None)

    orig_init_opt = rtrain.init_opt

    def init_opt(encoder, predictor, **kw):
        captured["models"] = (encoder, predictor)
        return orig_init_opt(encoder=encoder, predictor=predictor, **kw)

    def gpu_timer(closure, log_timings=True):
        res = closure()
        captured["losses"].append(res[0])
        captured.setdefault("lrs", []).append(res[1])
        captured.setdefault("wds", []).append(res[2])
        if snapshot_iter is not None and len(captured["losses"]) == snapshot_iter + 1:
            enc, pred = captured["models"]
            captured["after"] = dict(encoder={k: v.clone() for k, v in enc.backbone.state_dict().items()},
                                     predictor={k: v.clone() for k, v in pred.backbone.state_dict().items()})
        return res, 0.0

    saves = []
    orig_save = torch.save

    def save(obj, path, *a, **kw):  # keep a detached copy of every checkpoint the reference writes
        if isinstance(obj, dict) and "opt" in obj:
            saves.append(copy.deepcopy(obj))
        return orig_save(obj, path, *a, **kw)

    rtrain.init_data, rtrain.init_opt, rtrain.gpu_timer = init_data, init_opt, gpu_timer
    torch.save = save
    try:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("gloo", rank=0, world_size=1)
        args = dict(args, folder=tempfile.mkdtemp(prefix="vjepa_golden_"))
        rtrain.main(args)
    finally:
        torch.save = orig_save
        rtrain.init_opt = orig_init_opt
    captured["saves"] = saves
    samples = []
    for s in captured["samples"]:
        (batch, menc, mpred), = s
        samples.append(dict(clip_seeds=[1000 + B * len(samples) + j for j in range(B)],
                            clip_sum=batch[0][0].double().sum(), enc=menc, pred=mpred))
    return samples


def gen_main_vits():
    """BASELINE configs[0]: the reference's own app/vjepa/train.py:main at ViT-S/16 8x128^2 B=2, seed 239,
    ipe 6 (configs/train/vitl16/pretrain-256px-16f.yaml with model_name vit_small). Records the loss /
    lr / wd trajectory and every step's masks and clip seeds; no weights (both sides build them from
    the seed)."""
    B, fpc, crop = 2, 8, 128
    args = dict(
        meta=dict(dtype="bfloat16", seed=239, use_sdpa=True, load_checkpoint=False, save_every_freq=-1),
        mask=VITL_MASKS,
        model=dict(model_name="vit_small", pred_depth=12, pred_embed_dim=384, pred_num_heads=12, uniform_power=True,
                   use_activation_checkpointing=True, use_mask_tokens=True, use_rope=True,
                   zero_init_mask_tokens=True),
        data=dict(batch_size=B, crop_size=crop, patch_size=16, dataset_fpcs=[fpc], tubelet_size=2, fps=4,
                  num_workers=0),
        data_aug=dict(),
        loss=dict(loss_exp=1.0),
        optimization=dict(ema=[0.99925, 0.99925], epochs=1, final_lr=0.000525, final_weight_decay=0.04, ipe=6,
                          ipe_scale=1.25, lr=0.000525, start_lr=0.0001, warmup=40, weight_decay=0.04),
    )
    cap = dict(samples=[], losses=[])
    samples = _run_reference_main(args, B, fpc, crop, cap)
    save("main_vits.pt", dict(args=args, samples=samples, losses=cap["losses"], lrs=cap["lrs"], wds=cap["wds"]))


def gen_resume():
    """A checkpoint the reference's save_checkpoint writes (app/vjepa/train.py:315-333; micro model,
    fp32, after epoch 1 = 3 iterations) and what the reference's next iteration does from it: its
    inputs, loss and the encoder / predictor weights after it."""
    def vit_micro(patch_size=16, **kw):
        return vit.VisionTransformer(patch_size=patch_size, embed_dim=64, depth=2, num_heads=1, mlp_ratio=4,
                                     qkv_bias=True, norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6), **kw)

    vit.vit_micro = vit_micro
    B, fpc, crop = 2, 8, 64
    args = dict(
        meta=dict(dtype="float32", seed=239, use_sdpa=True, load_checkpoint=False, save_every_freq=-1),
        mask=VITL_MASKS,
        model=dict(model_name="vit_micro", pred_depth=2, pred_embed_dim=64, pred_num_heads=2, uniform_power=True,
                   use_activation_checkpointing=False, use_mask_tokens=True, use_rope=True,
                   zero_init_mask_tokens=True),
        data=dict(batch_size=B, crop_size=crop, patch_size=16, dataset_fpcs=[fpc], tubelet_size=2, fps=4,
                  num_workers=0),
        data_aug=dict(),
        loss=dict(loss_exp=1.0),
        optimization=dict(ema=[0.99925, 0.99925], epochs=2, final_lr=0.000525, final_weight_decay=0.04, ipe=3,
                          ipe_scale=1.25, lr=0.000525, start_lr=0.0001, warmup=1, weight_decay=0.04),
    )
    cap = dict(samples=[], losses=[])
    samples = _run_reference_main(args, B, fpc, crop, cap, snapshot_iter=3)
    ck = cap["saves"][0]  # end of epoch 1
    assert ck["epoch"] == 1
    save("ref_resume.pt", dict(args=args, ckpt=ck, sample=samples[3], loss=cap["losses"][3], lr=cap["lrs"][3],
                               wd=cap["wds"][3], after=cap["after"]))


def gen_pooler():
    """Frozen-encoder probe (src/models/attentive_pooler.py): an AttentiveClassifier (depth 3 = two
    self-attention Blocks + the cross-attention block, 1 query, 10 classes) and a 3-query pooler
    with the bare CrossAttention (complete_block=False); forward + backward on random tokens."""
    from src.models.attentive_pooler import AttentiveClassifier, AttentivePooler

    out = {}
    for name, ctor, kw in (("clf", AttentiveClassifier, dict(embed_dim=64, num_heads=2, depth=3, num_classes=10)),
                           ("pool3", AttentivePooler, dict(num_queries=3, embed_dim=64, num_heads=2, depth=2,
                                                           complete_block=False))):
        torch.manual_seed(11)
        m = ctor(**kw)
        init = {k: (v.double().sum().item(), v.double().pow(2).sum().item()) for k, v in m.state_dict().items()}
        for p in m.parameters():  # non-trivial LN / bias / query values
            with torch.no_grad():
                p.add_(0.05 * torch.randn_like(p))
        g = torch.Generator().manual_seed(12)
        x = torch.randn(2, 40, 64, generator=g, requires_grad=True)
        y = m(x)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy)
        out[name] = dict(state={k: v.detach().clone() for k, v in m.state_dict().items()}, x=x.detach(),
                         y=y.detach(), gy=gy, gx=x.grad.detach(), gparams=grads_of(m), cfg=kw, init=init)
    save("pooler.pt", out)


def gen_multiclip():
    """ClipAggregation (evals/video_classification_frozen/modelcustom/vit_encoder_multiclip.py:87-162):
    micro encoder, 2 clips x 2 views of 2 samples, temporal sincos pos-embed at the clips' frame indices."""
    sys.path.insert(0, os.path.join(REF, "evals", "video_classification_frozen", "modelcustom"))
    from vit_encoder_multiclip import ClipAggregation

    torch.manual_seed(21)
    enc = vit.VisionTransformer(img_size=32, patch_size=16, num_frames=4, tubelet_size=2, embed_dim=64, depth=2,
                                num_heads=1, mlp_ratio=4, qkv_bias=True, use_rope=True, uniform_power=True,
                                norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6))
    agg = ClipAggregation(enc, tubelet_size=2, max_frames=16, use_pos_embed=True)
    g = torch.Generator().manual_seed(22)
    x = [[torch.randn(2, 3, 4, 32, 32, generator=g) for _ in range(2)] for _ in range(2)]
    clip_indices = [torch.randint(0, 8, (2, 4), generator=g) for _ in range(2)]
    with torch.no_grad():
        outs = agg(x, clip_indices=clip_indices)
    save("multiclip.pt", dict(state={k: v.clone() for k, v in enc.state_dict().items()}, x=x,
                              clip_indices=clip_indices, outs=outs, pos_embed=agg.pos_embed.detach().clone()))


def gen_ac_predictor():
    """Action-conditioned predictor (src/models/ac_predictor.py:17-200): micro vit_ac_predictor
    (2x2 patches per frame, 3 frames after tubelets, 2 blocks, head dim 32), frame-causal with and without
    extrinsics; forward + backward."""
    from src.models.ac_predictor import vit_ac_predictor
    from src.models.utils.modules import build_action_block_causal_attention_mask

    out = {}
    for name, kw in (("causal", dict(use_extrinsics=False, is_frame_causal=True)),
                     ("causal_ext", dict(use_extrinsics=True, is_frame_causal=True)),
                     # SwiGLU MLP + stochastic depth (block 1 at rate 0.5: linspace(0, 0.5, 2)), training mode
                     ("causal_silu_dp", dict(use_extrinsics=False, is_frame_causal=True, use_silu=True,
                                             drop_path_rate=0.5))):
        # (is_frame_causal=False raises in the reference: ac_predictor.py:174 slices attn_mask = None)
        cfg = dict(img_size=32, patch_size=16, num_frames=6, tubelet_size=2, embed_dim=96, predictor_embed_dim=64,
                   depth=2, num_heads=2, action_embed_dim=7, **kw)
        torch.manual_seed(31)
        m = vit_ac_predictor(**cfg)
        init = {k: (v.double().sum().item(), v.double().pow(2).sum().item()) for k, v in m.state_dict().items()}
        for p in m.parameters():
            with torch.no_grad():
                p.add_(0.05 * torch.randn_like(p))
        g = torch.Generator().manual_seed(32)
        B, T = 2, 3
        x = torch.randn(B, T * 4, 96, generator=g, requires_grad=True)
        actions = torch.randn(B, T, 7, generator=g, requires_grad=True)
        states = torch.randn(B, T, 7, generator=g, requires_grad=True)
        ext = torch.randn(B, T, 6, generator=g, requires_grad=True)
        _DP["gen"], _DP["log"] = torch.Generator().manual_seed(38), []
        y = m(x, actions, states, ext if kw["use_extrinsics"] else None)
        draws = list(_DP["log"])
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy)
        out[name] = dict(draws=draws, state={k: v.detach().clone() for k, v in m.state_dict().items()}, x=x.detach(),
                         actions=actions.detach(), states=states.detach(), ext=ext.detach(), y=y.detach(), gy=gy,
                         gx=x.grad.detach(), gactions=actions.grad.detach(), gstates=states.grad.detach(),
                         gext=ext.grad.detach() if kw["use_extrinsics"] else None, gparams=grads_of(m), cfg=cfg,
                         init=init)
    out["mask_T3_2x2_a2"] = build_action_block_causal_attention_mask(3, 2, 2, add_tokens=2)
    save("ac_predictor.pt", out)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # regenerate selected fixtures only: make_golden.py gen_main_vits gen_resume
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    gen_rope()
    gen_sincos()
    gen_block("block_enc.pt", dim=128, heads=2, grid=4, T=2, N=32, K=10, with_thw=True, seed=3)
    gen_block("block_pred.pt", dim=96, heads=3, grid=4, T=2, N=32, K=9, with_thw=False, seed=4)
    gen_block_variants()
    gen_encoder()
    gen_predictor()
    gen_masks()
    gen_train_steps()
    gen_main_vits()
    gen_resume()
    gen_pooler()
    gen_multiclip()
    gen_ac_predictor()
    gen_vitl_autocast()
    gen_train_steps_bf16()
