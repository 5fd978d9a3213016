"""Benchmark: V-JEPA 2 ViT-L/16 16x256^2 JEPA train step (fwd + bwd + AdamW + EMA), bf16, synthetic.

    python bench.py [--gpus N] [--steps K] [--warmup W]      (N > 1: starts N rank processes itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (one rank per GPU)

Workload (BASELINE.json configs[1]; per-GPU batch 24 = configs/train/vitl16/pretrain-256px-16f.yaml):
ViT-L/16 RoPE encoder (24x1024, 16 heads), EMA target encoder, predictor 12x384 (12 heads), the two
reference mask configs (8 blocks @15 %, 2 blocks @70 %), masks from the reference MaskCollator
(torch seed 239 + rank), synthetic randn clips already resident in HBM. Weak scaling: every rank
runs B=24 clips per step; RCCL all-reduce of the 326 M fp32 gradients per step for N > 1.

Output: ONE JSON line (rank 0). `roofline` is the dominant kernel (largest total time) measured with
HIP events around each of its launches inside the timed region; `cpu_baseline` times the CPU
oracle (oracle/vjepa_oracle.py, fp32) on a bounded sample of the same workload.
"""

import argparse
import contextlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "clips/sec/GPU (ViT-L/16, 16×256², bf16) fwd+bwd; 1→8 GPU scaling"
MODEL_LABELS = {"vit_large": "ViT-L", "vit_small": "ViT-S", "vit_huge": "ViT-H", "vit_giant": "ViT-g",
                "vit_giant_xformers": "ViT-g"}


def metric_for(model, frames, crop, fp8=False):
    """BASELINE's metric string, naming the model / clip shape / precision the line actually ran
    (BASELINE.json's own string for its ViT-L/16 16x256^2 bf16 config)."""
    if (model, frames, crop, fp8) == ("vit_large", 16, 256, False):
        return METRIC
    dt = "bf16, fp8 target QKV/fc1" if fp8 else "bf16"
    return f"clips/sec/GPU ({MODEL_LABELS.get(model, model)}/16, {frames}×{crop}², {dt}) fwd+bwd; 1→8 GPU scaling"
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0  # dense fp8 (block-scaled e4m3 MFMA: 2x bf16 per clock)
PEAK_HBM_GBS = 8000.0

MASK_CFGS = [
    dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=8,
         spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
    dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0, num_blocks=2,
         spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0]),
]
MODELS = {"vit_large": dict(D=1024, depth=24, heads=16, mlp=4096), "vit_small": dict(D=384, depth=12, heads=6, mlp=1536),
          "vit_huge": dict(D=1280, depth=32, heads=16, mlp=5120),
          "vit_giant": dict(D=1408, depth=40, heads=16, mlp=6144),
          "vit_giant_xformers": dict(D=1408, depth=40, heads=22, mlp=6144)}


@contextlib.contextmanager
def _serialised():
    """Both side streams off (VJ_TGT_STREAM=0, VJ_WGRAD_STREAM=0) for the enclosed steps."""
    old = {e: os.environ.get(e) for e in ("VJ_TGT_STREAM", "VJ_WGRAD_STREAM")}
    os.environ.update({e: "0" for e in old})
    try:
        yield
    finally:
        for e, v in old.items():
            if v is None:
                os.environ.pop(e, None)
            else:
                os.environ[e] = v


def step_flops(model, B, N, masks_enc, masks_pred, pd=384, pdepth=12, pmlp=1536, kdim=1536):
    """SURVEY §8d algorithmic FLOPs of one step (no recompute, bwd = 2x fwd)."""
    cfg = MODELS[model]
    D, depth, mlp = cfg["D"], cfg["depth"], cfg["mlp"]

    def lin(n, d, h):
        return 2 * n * (4 * d * d + 2 * d * h)

    def att(n, d):
        return 4 * n * n * d

    f = B * (depth * (lin(N, D, mlp) + att(N, D)) + 2 * N * kdim * D)
    for me, mp in zip(masks_enc, masks_pred):
        K, Kp = me.shape[1], mp.shape[1]
        n = K + Kp
        f += B * 3 * (depth * (lin(K, D, mlp) + att(K, D)) + 2 * K * kdim * D * 2 / 3)
        f += B * 3 * (pdepth * (lin(n, pd, pmlp) + att(n, pd)) + 2 * K * D * pd + 2 * Kp * pd * D)
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=24)
    ap.add_argument("--model", default="vit_large")
    ap.add_argument("--crop", type=int, default=256)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--kernel-events", type=int, default=1)
    ap.add_argument("--fp8-target", type=int, default=0, help="target encoder QKV / fc1 GEMMs on the fp8 MFMA")
    ap.add_argument("--synced-steps", type=int, default=5,
                    help="untimed comparison steps with a float(loss) host sync per step (0: skip)")
    ap.add_argument("--arm-reducer", type=int, default=0,
                    help="at --gpus 1: arm the bucketed gradient all-reduce over a one-rank process group "
                         "(VJ_DIST_BACKEND, default nccl = RCCL) to price what N > 1 adds to the step")
    ap.add_argument("--rccl-proxy-cus", type=int, default=0,
                    help="with the reducer armed: a copy of 2x every bucket on N persistent workgroups beside its "
                         "all-reduce, pricing the CUs RCCL's channel kernels hold at world > 1 (diagnostic)")
    args = ap.parse_args()
    if args.gpus > 1 and "RANK" not in os.environ:
        # no launcher: start one rank process per GPU from this GPU-free parent
        sys.exit(spawn_ranks(args.gpus))

    from vjepa2_amd import ops
    from vjepa2_amd.distributed import init_distributed
    from vjepa2_amd.masks import MaskCollator
    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model
    import torch.distributed as dist

    # one rank per GPU: the device is LOCAL_RANK (modulo the device count only when rehearsing several
    # ranks on one device with VJ_DIST_BACKEND=gloo)
    local_rank = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    world, rank = init_distributed()
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the process group has {world} rank(s)")
    dev = torch.device("cuda", local_rank)
    if args.arm_reducer and world == 1 and not dist.is_initialized():
        import socket

        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        backend = os.environ.get("VJ_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                **({"device_id": dev} if backend == "nccl" else {}))
    # every rank states its process group (RCCL carried the buckets iff backend == "nccl")
    print(f"[bench rank {rank}/{world}] backend={dist.get_backend() if dist.is_initialized() else None} device={dev}",
          file=sys.stderr, flush=True)
    B, T, S = args.batch, args.frames, args.crop
    N = (T // 2) * (S // 16) ** 2

    torch.manual_seed(239)
    enc, pred = init_video_model(device=dev, patch_size=16, max_num_frames=T, tubelet_size=2, model_name=args.model,
                                 crop_size=S, pred_depth=12, pred_num_heads=12, pred_embed_dim=384, uniform_power=True,
                                 use_mask_tokens=True, num_mask_tokens=6, zero_init_mask_tokens=True, use_sdpa=True,
                                 use_rope=True)
    import copy

    tgt = copy.deepcopy(enc)
    opt, scaler, sched, wds = init_opt(enc, pred, iterations_per_epoch=300, start_lr=1e-4, ref_lr=5.25e-4, warmup=40,
                                       num_epochs=10, wd=0.04, final_wd=0.04, final_lr=5.25e-4, ipe_scale=1.25,
                                       mixed_precision=True)
    armed = args.arm_reducer == 1 or world > 1  # --arm-reducer 2: the process group only (diagnostics)
    trainer = JEPATrainer(enc, pred, tgt, opt, mixed_precision=True, loss_exp=1.0, world_size=world,
                          fp8_target=bool(args.fp8_target), arm_reducer=armed)
    if args.rccl_proxy_cus and trainer.reducer is not None:
        _install_rccl_proxy(trainer.reducer, args.rccl_proxy_cus, dev)
    # every step's clips and masks are on the device before the first step (below): the next step's
    # target forward may start under the previous step's staged update (JEPATrainer.apply_update)
    trainer.inputs_resident = os.environ.get("VJ_STAGED_UPDATE", "1") == "1"

    # inputs resident in HBM before timing: clips + masks for every step (dataloader prefetch)
    torch.manual_seed(239 + rank)
    mc = MaskCollator(cfgs_mask=MASK_CFGS, dataset_fpcs=[T], crop_size=S, patch_size=16, tubelet_size=2)
    nsteps = args.warmup + args.steps
    data = []
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    nclip = min(nsteps, 4)
    clips = [torch.randn(B, 3, T, S, S, device=dev, generator=g) for _ in range(nclip)]
    for i in range(nsteps):
        (_, me, mp), = mc([(torch.zeros(1), 0, [torch.arange(T)]) for _ in range(B)])
        data.append((clips[i % nclip], [m.to(dev) for m in me], [m.to(dev) for m in mp]))
    torch.cuda.synchronize()

    def run(i):
        c, me, mp = data[i]
        sched.step()
        wds.step()
        return trainer.train_step([c], [me], [mp], 0.99925)

    # Per-launch breakdown from the last (untimed) warmup step: a HIP event pair around every one of
    # its ~1500 launches. Inside the timed region only the dominant kernel's launches carry events
    # (the roofline's live average), so the timing is not inflated by the breakdown.
    # That step runs SERIALISED (target-encoder and weight-gradient side streams off): with the streams
    # on, concurrent kernels share the CUs and every per-launch time (events or rocprof) includes the
    # other stream's work, so neither the per-kernel rooflines nor the choice of the dominant kernel
    # would describe the kernels themselves.
    breakdown = None
    for i in range(args.warmup):
        full = ops.KernelEvents() if (args.kernel_events and i == args.warmup - 1) else None
        if full:
            with _serialised():
                full.start()
                run(i)
                full.stop()
            breakdown = full.summary()
        else:
            run(i)
    torch.cuda.synchronize()

    dominant = max(breakdown, key=lambda k: breakdown[k]["total_ms"]) if breakdown else None
    prof = ops.KernelEvents(only={dominant}) if dominant else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if prof:
        prof.start()
    # step-boundary events on the compute stream (no host sync between steps): per-step times for
    # the median; the contract's ms_per_step stays wall-clock over the K steps
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    trainer.time_allreduce = True  # two events per step on the compute stream (no host sync)
    trainer.ar_events.clear()
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.warmup, nsteps):
        loss = run(i)
        marks[i - args.warmup + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    trainer.time_allreduce = False
    if prof:
        prof.stop()
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms = elapsed * 1000.0 / args.steps
    step_ms = [a.elapsed_time(b) for a, b in zip(marks[:-1], marks[1:])]  # in step order
    per_step = sorted(step_ms)
    ms_median = per_step[len(per_step) // 2] if len(per_step) % 2 else 0.5 * (
        per_step[len(per_step) // 2 - 1] + per_step[len(per_step) // 2])
    if world > 1:
        t = torch.tensor([ms_median], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms_median = t.item()
    # exposed all-reduce: backward end -> GradReducer.finish() end, median over the timed steps, max
    # over ranks (0 at world 1: there is no reducer)
    ar = sorted(a.elapsed_time(b) for a, b in trainer.ar_events)
    ar_ms = (ar[len(ar) // 2] if len(ar) % 2 else 0.5 * (ar[len(ar) // 2 - 1] + ar[len(ar) // 2])) if ar else 0.0
    if world > 1:
        t = torch.tensor([ar_ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ar_ms = t.item()
    total_clips = B * world * args.steps
    value = total_clips / elapsed
    flops = sum(step_flops(args.model, B, N, d[1], d[2]) for d in data[args.warmup:]) / args.steps

    roof = None
    kstats = breakdown
    if prof:
        dom = dominant
        st = prof.summary()[dom]
        achieved = st["flops"] / (st["total_ms"] * 1e-3) / 1e12
        peak = PEAK_FP8_TFLOPS if dom.startswith("k_gemm_fp8") else PEAK_BF16_TFLOPS
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 1), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None,
                "launches_per_step": st["count"] / args.steps, "avg_launch_us": round(st["total_ms"] * 1e3 / st["count"], 2),
                "flops_per_launch": st["flops"] / st["count"]}
        tr = _pmc_traffic(dom, f"{args.model} {T}x{S}^2 B={B}")
        if tr:
            roof["traffic"] = tr["hbm_bytes_per_launch"]
            roof["traffic_unit"] = "B/launch"
            roof["traffic_source"] = tr["source"]

    # By default the target encoder's forward and the backward's weight-gradient GEMMs run on side
    # streams (train.py, functions.py), so inside the timed region the dominant kernel shares the CUs
    # with them. One more UNTIMED step with both streams off gives the same kernel's unshared launch
    # duration (what the serialised rocprofv3 profile under profiles/ shows).
    shared = [n for n, e, d in (("target-encoder side stream", "VJ_TGT_STREAM", "1"),
                                ("weight-gradient stream", "VJ_WGRAD_STREAM", "1")) if os.environ.get(e, d) == "1"]
    if roof and shared:
        solo = ops.KernelEvents(only={dom})
        torch.cuda.synchronize()
        with _serialised():
            solo.start()
            run(nsteps - 1)
            solo.stop()
        torch.cuda.synchronize()
        st1 = solo.summary()[dom]
        a1 = st1["flops"] / (st1["total_ms"] * 1e-3) / 1e12
        roof["timed_region_shares_cus_with"] = " and ".join(shared)
        roof["unshared"] = {"achieved": round(a1, 1), "frac": round(a1 / PEAK_BF16_TFLOPS, 4),
                            "avg_launch_us": round(st1["total_ms"] * 1e3 / st1["count"], 2),
                            "measured": "one extra untimed step with both side streams off"}

    # Untimed comparison (not the headline): the same steps with the reference loop's per-step host
    # sync (float(loss) every iteration, app/vjepa/train.py:468), to state what the free-running
    # timed loop above leaves out.
    synced = None
    if args.synced_steps > 0:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for i in range(args.synced_steps):
            float(run(args.warmup + i % args.steps))
        torch.cuda.synchronize()
        te = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([te], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            te = t.item()
        # the synced steps replay the timed region's inputs (masks, hence sequence lengths) from its
        # first step on: compare with the free-running per-step times of those same inputs
        same = [step_ms[i % args.steps] for i in range(args.synced_steps)]
        free_same = sum(same) / len(same)
        synced = {"ms_per_step": round(te * 1e3 / args.synced_steps, 2), "steps": args.synced_steps,
                  "sync": "float(loss) after every step (app/vjepa/train.py:468); untimed for value",
                  "free_running_ms_same_inputs": round(free_same, 2),
                  "vs_free_running": round(te * 1e3 / args.synced_steps / free_same, 4)}

    cpu = None
    if rank == 0 and args.cpu_baseline:
        cpu = cpu_baseline(args, data[0])

    if rank == 0:
        out = {"metric": metric_for(args.model, T, S, bool(args.fp8_target)), "value": round(value, 3), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "bf16+fp8(target QKV/fc1)" if args.fp8_target else "bf16",
               "data": "synthetic",
               "config": {"workload": f"{args.model} (RoPE) + predictor 12x384, {T}x{S}^2 clips, B={B}/GPU, JEPA "
                                      "train step: target fwd + ctx fwd/bwd (2 masks) + predictor fwd/bwd + L1 + "
                                      "AdamW + EMA", "model": args.model, "global_batch": B * world,
                          "seq_len": N, "parallelism": f"dp{world}"},
               "value_is": "whole-job clips/s (all ranks' clips / max-over-ranks time); per GPU: clips_per_s_per_gpu",
               "clips_per_s_per_gpu": round(value / world, 3), "ms_per_step_median": round(ms_median, 2),
               "clips_per_s_per_gpu_median": round(B / (ms_median * 1e-3), 3),
               "dist_backend": dist.get_backend() if dist.is_initialized() else None,
               "reducer_armed": armed, "rccl_proxy_cus": args.rccl_proxy_cus,
               "rccl_proxy_mode": int(os.environ.get("VJ_RCCL_PROXY_MODE", "0")) if args.rccl_proxy_cus else None,
               "step_tflop": round(flops / 1e12, 2),
               "step_tflops_per_gpu": round(flops / (ms * 1e-3) / 1e12, 1),
               "mfu_bf16": round(flops / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
               "loss_last": round(float(loss.item()), 5), "allreduce_exposed_ms": round(ar_ms, 3),
               "synced_comparison": synced, "roofline": roof, "cpu_baseline": cpu}
        if kstats:  # one untimed warmup step, every launch timed
            out["kernels"] = {k: {"ms_per_step": round(v["total_ms"], 3), "count_per_step": v["count"],
                                  "tflops": round(v["flops"] / (v["total_ms"] * 1e-3) / 1e12, 1) if v["flops"] else None}
                              for k, v in sorted(kstats.items(), key=lambda kv: -kv[1]["total_ms"])}
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def _install_rccl_proxy(red, blocks, dev):
    """--rccl-proxy-cus N: what RCCL's channel kernels cost the step at world > 1,
    priced on one GPU. Beside every bucket's all-reduce (over a one-rank group RCCL runs no kernel) a
    copy of twice the bucket's bytes (read + write, the HBM traffic of a ring all-reduce's reduce-scatter
    and all-gather, 2 (W - 1) / W of the bucket each at W = 8) runs on a stream of its own, on N persistent
    workgroups (RCCL's channels hold one CU each); the optimizer waits for it, as for the collectives."""
    from vjepa2_amd import ops

    mode = int(os.environ.get("VJ_RCCL_PROXY_MODE", "0"))  # 1: nt loads / stores, 2: CUs held, no bytes
    side = torch.cuda.Stream(device=dev)
    cap = max(b.view.numel() for b in red.buckets + red.tail)
    cap = (cap + 3) // 4 * 4
    scratch = torch.empty(2 * cap, device=dev)
    inner_ar, inner_finish = red._all_reduce, red.finish

    def all_reduce(b):
        inner_ar(b)
        side.wait_stream(torch.cuda.current_stream())
        n = b.view.numel() // 4 * 4  # whole 16-B chunks
        with torch.cuda.stream(side):
            for h in range(2):
                ops.proxy_copy(scratch[h * cap:h * cap + n], b.view[:n], blocks, mode)

    def finish():
        inner_finish()
        torch.cuda.current_stream().wait_stream(side)

    red._all_reduce, red.finish = all_reduce, finish


def spawn_ranks(n):
    """`bench.py --gpus N` without torchrun: one child process per rank (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in its env), started before this process makes any HIP call
    (torch.cuda.device_count() does not initialise the runtime). Returns the exit code: the first
    failing rank's, after terminating the others."""
    import socket
    import subprocess

    from vjepa2_amd import rank_env

    backend = os.environ.get("VJ_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and ndev < n:
        print(f"bench.py --gpus {n}: RCCL needs one device per rank but {ndev} HIP device(s) are visible "
              f"(VJ_DIST_BACKEND=gloo rehearses {n} ranks on fewer devices)", file=sys.stderr, flush=True)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = rank_env(dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                            MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    code = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            try:
                rc = p.wait(timeout=1.0)
            except subprocess.TimeoutExpired:
                continue
            alive.remove(p)
            if rc != 0 and code == 0:
                code = rc if rc > 0 else 1
                for q in alive:
                    q.terminate()
    return code


def _pmc_traffic(label, workload):
    """HBM bytes per launch of `label` measured by rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over
    this same bench, reduced by tools/traffic.py into profiles/traffic.json; None if the committed
    measurement is for another kernel or another workload."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic.json")
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None
    for tr in data if isinstance(data, list) else [data]:  # one entry per (kernel, workload)
        if tr.get("kernel") == label and tr.get("workload", "vit_large 16x256^2 B=24") == workload:
            tr["source"] = ("profiles/traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py; "
                            "L2-to-fabric bytes, Infinity-Cache hits included, so an upper bound on HBM bytes)")
            return tr
    return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, sample, timed=2):
    """The CPU oracle (fp32, the reference algorithm restated) on a bounded sample: ONE clip of the same
    workload (the same two masks truncated to B=1), one untimed warm-up step, then the median of
    `timed` full steps (fwd + bwd + AdamW + EMA). Threads: the process's CPU share (OMP_NUM_THREADS on
    the GPU box = 16; os.cpu_count() there counts the whole machine)."""
    from oracle import vjepa_oracle as orc

    threads = int(os.environ.get("VJ_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS") or
                  len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    torch.manual_seed(239)
    from vjepa2_amd import vision_transformer as vt
    from vjepa2_amd.predictor import vit_predictor

    T, S = args.frames, args.crop
    enc = getattr(vt, args.model)(img_size=S, num_frames=T, tubelet_size=2, use_rope=True, uniform_power=True)
    pred = vit_predictor(img_size=S, use_mask_tokens=True, patch_size=16, num_frames=T, tubelet_size=2,
                         embed_dim=enc.embed_dim, predictor_embed_dim=384, depth=12, num_heads=12, uniform_power=True,
                         num_mask_tokens=6, use_rope=True)
    ecfg = dict(patch_size=16, tubelet_size=2, num_heads=enc.num_heads, depth=len(enc.blocks), use_rope=True)
    pcfg = dict(num_heads=12, depth=12, use_rope=True, grid_size=S // 16, num_mask_tokens=6,
                num_patches=(T // 2) * (S // 16) ** 2)
    tr = orc.OracleTrainer(enc.state_dict(), pred.state_dict(), ecfg, pcfg)
    clips = sample[0][:1].cpu()
    me = [m[:1].cpu() for m in sample[1]]
    mp = [m[:1].cpu() for m in sample[2]]
    tr.step(clips, me, mp, 5.25e-4, 0.04, 0.99925)  # warm-up (allocator, thread pool)
    times = []
    for _ in range(timed):
        t0 = time.perf_counter()
        tr.step(clips, me, mp, 5.25e-4, 0.04, 0.99925)
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[len(times) // 2]
    return {"value": round(1.0 / dt, 4), "unit": "clips/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"1 clip ({args.model} {T}x{S}^2, masks K={[m.shape[1] for m in me]}, "
                      f"Kp={[m.shape[1] for m in mp]}): one warm-up + median of {timed} full fp32 steps "
                      f"(fwd+bwd+AdamW+EMA) of the CPU oracle, {dt:.1f} s/step, torch {threads} threads"}


if __name__ == "__main__":
    main()
