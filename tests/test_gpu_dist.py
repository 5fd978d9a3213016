"""GPU: the data-parallel train step at world size 2 (replaces the reference's DDP wraps,
app/vjepa/train.py:279-281), both ranks on the one GPU of the box with the gloo backend on device
tensors (RCCL refuses two ranks on one device). Each rank runs JEPATrainer(world_size=2) on its own
clips and masks; the bucketed gradient all-reduce fires from inside the backward.

Checked:
 * the reduced gradients on both ranks are bitwise the sum of the two single-process gradients
   (the gradient is the average of per-rank gradients; unused mask tokens untouched);
 * after AdamW (which folds in the 1/world average) both ranks hold bitwise-identical weights,
   equal to a single-process step on the rank-averaged gradients;
 * the first bucket's all-reduce is issued while the backward is still running (before the last
   block's backward finishes): the exchange overlaps the backward.
"""

import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T, S, B = 8, 64, 2
MASKS = [dict(aspect_ratio=[0.75, 1.5], num_blocks=8, spatial_scale=[0.15, 0.15], temporal_scale=[1.0, 1.0]),
         dict(aspect_ratio=[0.75, 1.5], num_blocks=2, spatial_scale=[0.7, 0.7], temporal_scale=[1.0, 1.0])]


def _inputs(rank):
    from vjepa2_amd.masks import MaskCollator

    torch.manual_seed(100 + rank)
    (_, me, mp_), = MaskCollator(MASKS, [T], crop_size=S, patch_size=16)([(0, 0, [torch.arange(T)])] * B)
    clips = torch.randn(B, 3, T, S, S, generator=torch.Generator().manual_seed(200 + rank))
    return clips, me, mp_


def _build(world, group=None):
    import copy

    from vjepa2_amd.train import JEPATrainer, init_opt, init_video_model

    torch.manual_seed(239)
    enc, pred = init_video_model(device="cuda", patch_size=16, max_num_frames=T, tubelet_size=2,
                                 model_name="vit_small", crop_size=S, pred_depth=2, pred_num_heads=12,
                                 pred_embed_dim=384, uniform_power=True, use_mask_tokens=True, num_mask_tokens=2,
                                 use_sdpa=True, use_rope=True)
    tgt = copy.deepcopy(enc)
    opt, _, _, _ = init_opt(enc, pred, iterations_per_epoch=10, start_lr=1e-4, ref_lr=1e-4, warmup=0, num_epochs=1,
                            wd=0.04, final_wd=0.04, mixed_precision=True)
    for g in opt.param_groups:
        g["lr"] = 2e-4
        if not g.get("WD_exclude", False):
            g["weight_decay"] = 0.04
    # small buckets so the backward issues several of them
    return JEPATrainer(enc, pred, tgt, opt, mixed_precision=True, world_size=world, bucket_mb=4, group=group), opt


def _rank_main(rank, world, port, out_dir):
    import torch.distributed as dist

    from vjepa2_amd import distributed as vdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    w, r = vdist.init_distributed(backend="gloo")
    assert (w, r) == (world, rank)
    tr, opt = _build(world)
    log = []  # (host time, event) of bucket issues and of every module's grad-ready hook
    issue0 = tr.reducer._issue

    def issue(b):
        log.append((time.perf_counter(), "issue", tr.reducer.buckets.index(b) if b in tr.reducer.buckets else -1))
        issue0(b)

    tr.reducer._issue = issue
    mark0 = tr.reducer.mark_ready

    def mark(mod):
        log.append((time.perf_counter(), "ready", type(mod).__name__))
        mark0(mod)

    for m in [getattr(x, "_vj_grad_ready", None) and x for x in list(tr.pred.predictor_blocks) + list(tr.enc.blocks)
              + [tr.pred.predictor_norm, tr.pred.predictor_proj, tr.pred.predictor_embed, tr.enc.norm,
                 tr.enc.patch_embed, tr.pred.mask_tokens]]:
        if m is not None:
            m._vj_grad_ready = mark
    clips, me, mp_ = _inputs(rank)
    loss = tr.compute_grads([clips.cuda()], [[m.cuda() for m in me]], [[m.cuda() for m in mp_]])
    torch.cuda.synchronize()
    grads = [a.grad.detach().cpu().clone() for a in opt.arenas]
    tr.apply_update(0.99925)
    torch.cuda.synchronize()
    params = [a.data.detach().cpu().clone() for a in opt.arenas + tr.tgt_arenas]
    torch.save(dict(grads=grads, params=params, log=log, loss=float(loss),
                    nbuckets=len(tr.reducer.buckets)), os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_data_parallel_step_world2(tmp_path):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    # single-process gradients of each rank's inputs (this process, world 1)
    single = []
    for r in range(2):
        tr, opt = _build(1)
        clips, me, mp_ = _inputs(r)
        tr.compute_grads([clips.cuda()], [[m.cuda() for m in me]], [[m.cuda() for m in mp_]])
        torch.cuda.synchronize()
        single.append([a.grad.detach().cpu().clone() for a in opt.arenas])
    for i in range(len(single[0])):
        summed = single[0][i] + single[1][i]
        assert torch.equal(res[0]["grads"][i], summed), f"rank 0 arena {i}: reduced grads != sum of per-rank grads"
        assert torch.equal(res[1]["grads"][i], summed), f"rank 1 arena {i}"
    for a, b in zip(res[0]["params"], res[1]["params"]):
        assert torch.equal(a, b), "ranks diverged after the step"
    # single-process step on the summed gradients with the 1/world average folded into AdamW
    tr, opt = _build(1)
    for a, g0, g1 in zip(opt.arenas, single[0], single[1]):
        a.grad.copy_((g0 + g1).cuda())
    tr.world = 2
    tr.apply_update(0.99925)
    torch.cuda.synchronize()
    ref = [a.data.detach().cpu() for a in opt.arenas + tr.tgt_arenas]
    for a, b in zip(res[0]["params"], ref):
        assert torch.equal(a, b), "DP step != single-process step on the averaged gradients"
    # overlap: buckets are issued from inside the backward, before its last module is done
    for r in range(2):
        log = res[r]["log"]
        issues = [t for t, kind, _ in log if kind == "issue"]
        readies = [t for t, kind, _ in log if kind == "ready"]
        assert res[r]["nbuckets"] >= 3 and len(issues) >= res[r]["nbuckets"]
        assert issues[0] < readies[-1], "no all-reduce was issued before the backward finished"
        print(f"rank {r}: {res[r]['nbuckets']} buckets, first issued after {sum(t < issues[0] for t in readies)} "
              f"of {len(readies)} module backwards; loss {res[r]['loss']:.5f}")
