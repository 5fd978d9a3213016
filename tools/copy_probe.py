"""Where do the train step's device copies (__amd_rocclr_copyBuffer launches) come from?

One bench-configuration train step (ViT-L/16, 16x256^2, B=24) under torch.profiler with Python
stacks; prints the host ops that issue memory copies (aten::copy_ / hipMemcpy*) grouped by their
innermost vjepa2_amd frame.   usage: python tools/copy_probe.py [steps]"""
import collections
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import MASK_CFGS  # noqa: E402
from vjepa2_amd.masks import MaskCollator  # noqa: E402
from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model  # noqa: E402


def main(steps=1):
    dev = torch.device("cuda", 0)
    B, T, S = 24, 16, 256
    torch.manual_seed(239)
    enc, pred = init_video_model(device=dev, patch_size=16, max_num_frames=T, tubelet_size=2, model_name="vit_large",
                                 crop_size=S, pred_depth=12, pred_num_heads=12, pred_embed_dim=384, uniform_power=True,
                                 use_mask_tokens=True, num_mask_tokens=6, zero_init_mask_tokens=True, use_sdpa=True,
                                 use_rope=True)
    tgt = copy.deepcopy(enc)
    opt, scaler, sched, wds = init_opt(enc, pred, iterations_per_epoch=300, start_lr=1e-4, ref_lr=5.25e-4, warmup=40,
                                       num_epochs=10, wd=0.04, final_wd=0.04, final_lr=5.25e-4, ipe_scale=1.25,
                                       mixed_precision=True)
    tr = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True, loss_exp=1.0, world_size=1)
    tr.inputs_resident = True
    mc = MaskCollator(cfgs_mask=MASK_CFGS, dataset_fpcs=[T], crop_size=S, patch_size=16, tubelet_size=2)
    g = torch.Generator(device=dev).manual_seed(1000)
    clip = torch.randn(B, 3, T, S, S, device=dev, generator=g)
    data = []
    for _ in range(3 + steps):
        (_, me, mp), = mc([(torch.zeros(1), 0, [torch.arange(T)]) for _ in range(B)])
        data.append(([m.to(dev) for m in me], [m.to(dev) for m in mp]))
    torch.cuda.synchronize()

    def run(i):
        sched.step()
        wds.step()
        return tr.train_step([clip], [data[i][0]], [data[i][1]], 0.99925)

    for i in range(3):
        run(i)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        for i in range(steps):
            run(3 + i)
        torch.cuda.synchronize()
    by_site = collections.Counter()
    kinds = collections.Counter()
    for e in prof.events():
        name = e.name
        if not (name in ("aten::copy_", "aten::_to_copy", "aten::clone") or "Memcpy" in name or "memcpy" in name):
            continue
        kinds[name] += 1
        if name != "aten::copy_" and "Memcpy" not in name:
            continue
        site = "?"
        for fr in (e.stack or []):
            if "vjepa2_amd" in fr or "bench" in fr:
                site = fr
                break
        shapes = tuple(tuple(s) for s in (e.input_shapes or [])[:2])
        by_site[(name, site, str(shapes)[:60])] += 1
    print("per step:")
    for k, v in kinds.most_common():
        print(f"  {v / steps:8.1f}  {k}")
    print("copy sites (per step):")
    for (name, site, shp), v in by_site.most_common(40):
        print(f"  {v / steps:8.1f}  {name:24s} {site[:90]:90s} {shp}")
    gpu = collections.Counter()
    for e in prof.key_averages():
        if "copyBuffer" in e.key or "Memcpy" in e.key or "memcpy" in e.key.lower():
            gpu[e.key] = e.count
    print("device-side copy entries:", {k: v / steps for k, v in gpu.items()})


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
