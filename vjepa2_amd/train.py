"""V-JEPA pre-training app (drop-in for app/vjepa/train.py + app/vjepa/utils.py).

`main(args, resume_preempt)` reads the same YAML keys (meta / mask / model / data / data_aug / loss /
optimization) and runs the same step (train.py:409-471): target encoder forward (no grad) ->
context encoder on every mask -> predictor -> L1 JEPA loss -> backward -> [grad all-reduce] ->
AdamW -> EMA of the target encoder. The step itself is JEPATrainer.train_step, MI355X-native:
  * both mask passes of the encoder and of the predictor run as ONE ragged pass each
    (same math as the reference's per-mask loop, wrappers.py:20-43, but full-size GEMMs);
  * the target encoder's final LayerNorm, the extra F.layer_norm, the gather by masks_pred and the
    L1 loss + its gradient are one kernel;
  * gradients land in flat arenas; RCCL all-reduce of contiguous buckets overlaps the backward;
  * AdamW (+ GradScaler inf-skip) and the EMA are single fused kernels that also refresh the
    bf16 weight shadows the GEMMs read.
Activation checkpointing is not needed (ViT-L B=24 activations ~25 GB of 288 GB HBM); it would
change no numerics, so the config key is accepted and ignored.
"""

import copy
import csv
import logging
import os
import time

import numpy as np
import torch

from . import ops
from . import predictor as vit_pred
from . import vision_transformer as video_vit
from .arena import FlatArena, FusedAdamW, fused_ema, readiness_order, wd_split
from .distributed import GradReducer, init_distributed
from .functions import join_wgrad_stream, refresh_weight_transposes
from .masks import MaskCollator, materialize
from .schedulers import CosineWDSchedule, WarmupCosineSchedule
from .wrappers import MultiSeqWrapper, PredictorMultiSeqWrapper

logger = logging.getLogger(__name__)
_GLOBAL_SEED = 0
_WT_BATCH = os.environ.get("VJ_WT_BATCH", "1") != "0"
_FUSED_EMA = os.environ.get("VJ_FUSED_EMA", "1") != "0"


# ------------------------------------------------------------------------------------------------
# app/vjepa/utils.py equivalents
def init_video_model(device, patch_size=16, max_num_frames=16, tubelet_size=2, model_name="vit_base", crop_size=224,
                     pred_depth=6, pred_num_heads=None, pred_embed_dim=384, uniform_power=False, use_mask_tokens=False,
                     num_mask_tokens=2, zero_init_mask_tokens=True, use_sdpa=False, use_rope=False, use_silu=False,
                     use_pred_silu=False, wide_silu=False, use_activation_checkpointing=False):
    """app/vjepa/utils.py:138-204 (same construction order -> same initial weights per seed)."""
    encoder = video_vit.__dict__[model_name](img_size=crop_size, patch_size=patch_size, num_frames=max_num_frames,
                                             tubelet_size=tubelet_size, uniform_power=uniform_power,
                                             use_sdpa=use_sdpa, use_silu=use_silu, wide_silu=wide_silu,
                                             use_activation_checkpointing=use_activation_checkpointing,
                                             use_rope=use_rope)
    encoder = MultiSeqWrapper(encoder)
    predictor = vit_pred.vit_predictor(img_size=crop_size, use_mask_tokens=use_mask_tokens, patch_size=patch_size,
                                       num_frames=max_num_frames, tubelet_size=tubelet_size,
                                       embed_dim=encoder.backbone.embed_dim, predictor_embed_dim=pred_embed_dim,
                                       depth=pred_depth,
                                       num_heads=encoder.backbone.num_heads if pred_num_heads is None else pred_num_heads,
                                       uniform_power=uniform_power, num_mask_tokens=num_mask_tokens,
                                       zero_init_mask_tokens=zero_init_mask_tokens, use_rope=use_rope,
                                       use_sdpa=use_sdpa, use_silu=use_pred_silu, wide_silu=wide_silu,
                                       use_activation_checkpointing=use_activation_checkpointing)
    predictor = PredictorMultiSeqWrapper(predictor)
    encoder.to(device)
    predictor.to(device)
    return encoder, predictor


def _trainable(m):
    return [(n, p) for n, p in m.named_parameters() if p.requires_grad]


def init_opt(encoder, predictor, iterations_per_epoch, start_lr, ref_lr, warmup, num_epochs, wd=1e-6, final_wd=1e-6,
             final_lr=0.0, mixed_precision=False, ipe_scale=1.25, betas=(0.9, 0.999), eps=1e-8, zero_init_bias_wd=True):
    """app/vjepa/utils.py:207-255. The four AdamW param groups become four flat arenas; the
    returned optimizer is the fused HIP AdamW. `scaler` is the GradScaler flag (bf16 needs no
    loss scaling: its exponent range is fp32's; the inf/NaN step-skip is kept)."""
    device = next(encoder.parameters()).device
    enc_wd, enc_nowd = wd_split(readiness_order(_trainable(encoder)))
    pred_wd, pred_nowd = wd_split(readiness_order(_trainable(predictor)))
    arenas = [FlatArena(enc_wd, device, name="encoder"), FlatArena(pred_wd, device, name="predictor"),
              FlatArena(enc_nowd, device, name="encoder_nowd"), FlatArena(pred_nowd, device, name="predictor_nowd")]
    # the reference's param groups (utils.py:224-237) in named_parameters() order, frozen params
    # included: the numbering of the optimizer state in checkpoints
    ref_groups = list(wd_split(encoder.named_parameters())) + list(wd_split(predictor.named_parameters()))
    ref_groups = [ref_groups[0], ref_groups[2], ref_groups[1], ref_groups[3]]
    optimizer = FusedAdamW(arenas, wd_exclude=[None, None, zero_init_bias_wd, zero_init_bias_wd], betas=betas,
                           eps=eps, ref_groups=ref_groups)
    scheduler = WarmupCosineSchedule(optimizer, warmup_steps=int(warmup * iterations_per_epoch), start_lr=start_lr,
                                     ref_lr=ref_lr, final_lr=final_lr,
                                     T_max=int(ipe_scale * num_epochs * iterations_per_epoch))
    wd_scheduler = CosineWDSchedule(optimizer, ref_wd=wd, final_wd=final_wd,
                                    T_max=int(ipe_scale * num_epochs * iterations_per_epoch))
    scaler = GradScalerFlag() if mixed_precision else None
    return optimizer, scaler, scheduler, wd_scheduler


class GradScalerFlag:
    """Stands in for torch.cuda.amp.GradScaler: the fused path checks grads for inf/NaN and skips
    the AdamW update exactly when GradScaler.step would; loss scale is fixed at 1."""

    def state_dict(self):
        return {"scale": 1.0, "growth_factor": 2.0, "backoff_factor": 0.5, "growth_interval": 2000, "_growth_tracker": 0}

    def load_state_dict(self, sd):
        pass


# ------------------------------------------------------------------------------------------------
class JEPATrainer:
    """The fused V-JEPA train step (app/vjepa/train.py:409-471) over arena-owned parameters."""

    def __init__(self, encoder, predictor, target_encoder, optimizer, mixed_precision=True, loss_exp=1.0, world_size=1,
                 bucket_mb=64, group=None, fp8_target=False, target_bf16_residual=None, ctx_bf16_residual=None,
                 arm_reducer=False):
        unwrap = lambda m: getattr(m, "backbone", getattr(m, "module", m))  # noqa: E731
        self.enc, self.pred, self.tgt = unwrap(encoder), unwrap(predictor), unwrap(target_encoder)
        self.opt = optimizer
        self.mixed_precision = mixed_precision
        self.loss_exp = loss_exp
        self.world = world_size
        # opt-in: the no-grad target encoder's QKV / fc1 GEMMs on the fp8 MFMA (functions.block_forward_fp8)
        self.fp8_target = fp8_target
        # the no-grad target encoder's residual stream in bf16 (the reference's autocast precision;
        # half the bytes of its proj / fc2 epilogues and LayerNorm reads). Default on under bf16
        # mixed precision (the reference's forward_target runs under autocast there); env
        # VJ_TARGET_BF16=0 or target_bf16_residual=False keeps it f32.
        if target_bf16_residual is None:  # float32 configs (mixed_precision False) keep the reference's f32
            target_bf16_residual = mixed_precision and os.environ.get("VJ_TARGET_BF16", "1") != "0"
        self.target_bf16_residual = bool(target_bf16_residual)
        # The trained context encoder's residual stream in bf16 too, where the reference's autocast keeps
        # it there (RoPE encoder: bf16 Conv3d tokens, every x = x + branch(...) a bf16 add,
        # modules.py:561-562; its gradient is bf16 as well). Half the bytes of its proj / fc2 residual
        # epilogues, LayerNorm reads and LayerNorm backward. The predictor keeps f32: there
        # torch.cat([bf16 tokens, f32 mask tokens]) promotes the stream to f32 (predictor.py:206).
        # VJ_CTX_BF16=0 (or ctx_bf16_residual=False) keeps the context encoder's stream f32.
        if ctx_bf16_residual is None:
            ctx_bf16_residual = (mixed_precision and os.environ.get("VJ_CTX_BF16", "1") != "0"
                                 and self.enc.bf16_residual_ok())
        self.ctx_bf16_residual = bool(ctx_bf16_residual)
        enc_w, pred_w, enc_n, pred_n = optimizer.arenas
        device = enc_w.data.device
        tnamed = dict(target_encoder.named_parameters())
        for p in tnamed.values():
            p.requires_grad = False
        self.tgt_arenas = [FlatArena([(n, tnamed[n]) for n in a.names], device, grads=False, opt_state=False,
                                     name="target" + a.name[7:]) for a in (enc_w, enc_n)]
        self.enc_arenas = [enc_w, enc_n]
        self.mask_tokens = list(self.pred.mask_tokens) if self.pred.mask_tokens is not None else []
        # inputs_resident: the caller guarantees every step's clips are on the device before the
        # previous step's update begins (bench.py: all inputs prepared up front); enables the staged
        # update overlap (apply_update). Default off: the target forward waits for all prior work.
        self.inputs_resident = False
        self._staged = None
        self.reducer = None
        # time_allreduce: per step, a HIP event pair on the compute stream from the end of the backward
        # (last gradient written) to the end of GradReducer.finish() (the stream waits for every
        # bucket): the all-reduce time NOT hidden under the backward. Appended to ar_events.
        self.time_allreduce = False
        self.ar_events = []
        # arm_reducer: the gradient all-reduce even at world 1 (a one-rank process group): prices what the
        # bucketed all-reduce and its stream joins add to the step on one GPU (bench.py --arm-reducer)
        if world_size > 1 or arm_reducer:
            seg = lambda a: (a.grad, [(p, o, p.numel()) for p, o in zip(a.params, a.offsets)])  # noqa: E731
            self.reducer = GradReducer([seg(pred_w), seg(enc_w)], tail_segments=[seg(pred_n), seg(enc_n)],
                                       bucket_mb=bucket_mb, group=group)
            mods = list(self.pred.predictor_blocks) + list(self.enc.blocks)
            mods += [self.pred.predictor_norm, self.pred.predictor_proj, self.pred.predictor_embed, self.enc.norm,
                     self.enc.patch_embed]
            if self.pred.mask_tokens is not None:
                mods.append(self.pred.mask_tokens)
            self.reducer.install(mods)

    def forward_loss(self, clips, masks_enc, masks_pred, mask_index=0, npairs=None):
        """Forward of one frames-per-clip group: returns (loss [1], z_pred, dz).

        The target encoder's forward (train.py:414-418, no grad) depends only on the clips and the
        EMA weights, so it runs on a second HIP stream concurrently with the context encoder and
        predictor: its GEMM / attention tiles fill the CUs the ragged context-side launches leave
        idle in their last wave of tiles. The loss waits for both."""
        B = clips.shape[0]
        side = self._side_stream()
        if side is not None:
            main = torch.cuda.current_stream()
            staged, self._staged = (self._staged if mask_index == 0 else None), None
            if staged is not None:
                # staged update (apply_update): the clips were resident before it began, so the side
                # stream waits for that point and then for each stage's EMA'd weights as its forward
                # reaches them, instead of for the whole optimizer pass
                side.wait_event(staged[0])
                for m, ev in zip(self._stage_tgt, staged[1]):
                    m._vj_ready = ev
            else:
                side.wait_stream(main)  # clips + this step's EMA'd target weights are ready
            with torch.cuda.stream(side), torch.no_grad():
                h = self.tgt.forward_features(clips, fp8=self.fp8_target, bf16_residual=self.target_bf16_residual)
            if staged is not None:
                for m in self._stage_tgt:
                    m._vj_ready = None
        else:
            with torch.no_grad():
                h = self.tgt.forward_features(clips, fp8=self.fp8_target, bf16_residual=self.target_bf16_residual)
        z, _ = self.enc.forward_ragged(clips, masks_enc, out_dtype=torch.bfloat16, bf16_residual=self.ctx_bf16_residual)
        _, Tp, Hp, Wp, _, _ = self.enc._geometry(clips)  # this group's tokens per clip (h's rows per sample)
        if h.shape[0] != B * Tp * Hp * Wp:
            raise RuntimeError(f"target rows {h.shape[0]} != {B} clips x {Tp * Hp * Wp} tokens")
        zp, pl = self.pred.forward_ragged(z, masks_enc, masks_pred, mask_index=mask_index, out_dtype=torch.bfloat16,
                                          n_target=Tp * Hp * Wp)
        if side is not None:
            main.wait_stream(side)
            h.record_stream(main)
        loss, dz, _ = ops.jepa_loss(zp, h, pl.loss_rows, self.tgt.norm.weight, self.tgt.norm.bias,
                                    [B * int(m.shape[1]) for m in masks_pred], eps1=self.tgt.norm.eps, eps2=1e-5,
                                    loss_exp=self.loss_exp, npairs=npairs)
        return loss, zp, dz

    def _update_stages(self):
        """Online-encoder parameters per stage of the forward (embedding: every parameter outside the
        blocks and the final norm; block 0 ... block L-1; final norm), and the matching target
        modules, for the staged update."""
        if getattr(self, "_stages", None) is None:
            e, t = self.enc, self.tgt
            emb = [p for n, p in e.named_parameters() if not n.startswith(("blocks.", "norm."))]
            self._stages = [emb] + [list(b.parameters()) for b in e.blocks]
            self._stage_tgt = [t.patch_embed] + list(t.blocks)
            if e.norm is not None:
                self._stages.append(list(e.norm.parameters()))
                self._stage_tgt.append(t.norm)
        return self._stages

    def _enc_param_ids(self):
        return {id(p) for a in self.enc_arenas for p in a.params}

    def _side_stream(self):
        # On by default since round 4: with the persistent one-workgroup-per-CU GEMMs and the faster
        # epilogues the overlap is worth +2.0 % clips/s (207.5 / 207.6 -> 211.5 / 211.7, bench.py A/B
        # in one call, profiles/r04_tgt_stream_step_ab.txt); in round 1 it gave ~1 % while inflating
        # the memory-bound kernels it shared CUs with. VJ_TGT_STREAM=0 runs everything on one stream.
        if os.environ.get("VJ_TGT_STREAM", "1") != "1" or not torch.cuda.is_available():
            return None
        if getattr(self, "_tgt_stream", None) is None:
            self._tgt_stream = torch.cuda.Stream()
        return self._tgt_stream

    def train_step(self, clips, masks_enc, masks_pred, momentum):
        """clips / masks_* are per frames-per-clip group lists (train.py:393-400 layout). LR / WD
        must already be set on the optimizer's param_groups (schedulers). Returns the loss tensor."""
        loss = self.compute_grads(clips, masks_enc, masks_pred)
        self.apply_update(momentum)
        return loss

    def compute_grads(self, clips, masks_enc, masks_pred):
        """Forward + backward (train.py:414-445): gradients land in the arenas, all-reduced (summed)
        across ranks when world > 1. Several frames-per-clip groups (one entry per group in clips /
        masks_*) run one after the other, group i's predictor with mask token i (wrappers.py:20-43,
        mask_index = i); the loss is the mean over every (group, mask) pair (train.py:425-435), so
        each group's loss and dL/dz carry 1 / (all pairs). The gradient all-reduce is armed only for
        the last group's backward: a parameter's gradient is complete only after every group's."""
        G = len(clips)
        if not (G == len(masks_enc) == len(masks_pred)) or G == 0:
            raise ValueError("clips / masks_enc / masks_pred: one entry per frames-per-clip group")
        npairs = sum(len(m) for m in masks_enc)
        total = None
        for i in range(G):
            if self.reducer is not None:
                self.reducer.armed = i == G - 1
            loss, zp, dz = self.forward_loss(clips[i], masks_enc[i], masks_pred[i], mask_index=i, npairs=npairs)
            zp.backward(dz)
            total = loss if total is None else total + loss
        self._groups = G
        join_wgrad_stream()  # weight gradients issued on the side stream (no-op when off)
        for a in self.opt.arenas:  # lazily zeroed gradients nothing wrote (before the tail buckets)
            a.finalize_grads()
        ev = None
        if self.time_allreduce:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if self.reducer is not None:
            self.reducer.finish()
        if ev is not None:
            ev[1].record()
            self.ar_events.append(ev)
        return total

    def apply_update(self, momentum):
        """GradScaler inf-check + AdamW (train.py:446-454) + EMA (train.py:456-465). The 1/world
        average of the summed gradients is folded into AdamW. Mask tokens other than the one this
        step used have grad None in the reference, so they take no step (no decay either)."""
        # Staged issue (inputs_resident set by the caller, target side stream on): the AdamW + EMA pass
        # is issued stage by stage in the order the next forward uses the weights (patch embedding,
        # block 0, ...), an event after each; the next step's target forward (side stream) waits for
        # each stage's event instead of the whole pass, so it overlaps the rest of the update.
        staged = (self.inputs_resident and _FUSED_EMA and self._side_stream() is not None
                  and not any(id(t) in self._enc_param_ids() for t in self.mask_tokens))
        pre = None
        if staged:
            pre = torch.cuda.Event()
            pre.record()
        found = self.opt.check_finite() if self.mixed_precision else None
        used = {i % max(1, len(self.mask_tokens)) for i in range(getattr(self, "_groups", 1))}
        unused = [t for i, t in enumerate(self.mask_tokens) if i not in used]
        if _FUSED_EMA:  # the EMA inside the encoder arenas' AdamW pass (one read of the online weights)
            tmap = {id(o): t for t, o in zip(self.tgt_arenas, self.enc_arenas)}
            evs = self.opt.step(grad_scale=1.0 / self.world, found_inf=found, exclude=unused,
                                ema=([tmap.get(id(a)) for a in self.opt.arenas], momentum),
                                stages=self._update_stages() if staged else None)
            self._staged = (pre, evs) if staged else None
            self.opt.zero_grad()
        else:
            self.opt.step(grad_scale=1.0 / self.world, found_inf=found, exclude=unused)
            self.opt.zero_grad()
            fused_ema(self.tgt_arenas, self.enc_arenas, momentum)
        if _WT_BATCH:  # the next backward's W^T operands, one launch (VJ_WT_BATCH=0: lazily, one per weight)
            refresh_weight_transposes()

    def sync_bf16(self):
        for a in self.opt.arenas + self.tgt_arenas:
            a.sync_bf16()


# ------------------------------------------------------------------------------------------------
# data (the reference's VideoDataset/decord pipeline is out of scope: synthetic clips of the
# same sample structure, train.py:373-400 / video_dataset.py:246)
class SyntheticVideoDataset(torch.utils.data.Dataset):
    def __init__(self, num_samples, frames_per_clip, crop_size, seed_offset=1000):
        self.n, self.fpc, self.crop, self.seed_offset = num_samples, frames_per_clip, crop_size, seed_offset

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed_offset + i)
        clip = torch.randn(3, self.fpc, self.crop, self.crop, generator=g)
        return [clip], 0, [torch.arange(self.fpc)]


def init_data(batch_size, collator, dataset_fpcs, crop_size, rank=0, world_size=1, num_workers=0, num_samples=None,
              **kw):
    n = num_samples or 1_000_000
    ds = SyntheticVideoDataset(n, max(dataset_fpcs), crop_size)
    sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world_size, rank=rank, shuffle=False)
    dl = torch.utils.data.DataLoader(ds, batch_size=batch_size, sampler=sampler, collate_fn=collator,
                                     num_workers=num_workers, drop_last=True, persistent_workers=num_workers > 0)
    return dl, sampler


# ------------------------------------------------------------------------------------------------
def _prefixed(sd):
    return {"module.backbone." + k: v for k, v in sd.items()}


def _strip(sd):
    out = {}
    for k, v in sd.items():
        for pre in ("module.", "backbone."):
            if k.startswith(pre):
                k = k[len(pre):]
        out[k] = v
    return out


def save_checkpoint(path, encoder, predictor, target_encoder, optimizer, scaler, epoch, loss, batch_size, world_size,
                    lr):
    """train.py:315-333 format (keys with the DDP + wrapper prefix 'module.backbone.')."""
    unwrap = lambda m: getattr(m, "backbone", m)  # noqa: E731
    torch.save({"encoder": _prefixed(unwrap(encoder).state_dict()),
                "predictor": _prefixed(unwrap(predictor).state_dict()),
                "opt": optimizer.state_dict(), "scaler": None if scaler is None else scaler.state_dict(),
                "target_encoder": _prefixed(unwrap(target_encoder).state_dict()), "epoch": epoch, "loss": loss,
                "batch_size": batch_size, "world_size": world_size, "lr": lr}, path)


def load_checkpoint(r_path, encoder, predictor, target_encoder, opt, scaler, trainer=None):
    """app/vjepa/utils.py:90-135 (tensor-only checkpoints: loaded with weights_only=True)."""
    ck = torch.load(r_path, map_location="cpu", weights_only=True)
    unwrap = lambda m: getattr(m, "backbone", m)  # noqa: E731
    unwrap(encoder).load_state_dict(_strip(ck["encoder"]))
    unwrap(predictor).load_state_dict(_strip(ck["predictor"]))
    if target_encoder is not None:
        unwrap(target_encoder).load_state_dict(_strip(ck["target_encoder"]))
    if opt is not None and ck.get("opt"):
        opt.load_state_dict(ck["opt"])
    if trainer is not None:
        trainer.sync_bf16()
    elif opt is not None:
        for a in opt.arenas:
            a.sync_bf16()
    return encoder, predictor, target_encoder, opt, scaler, ck["epoch"]


def gpu_timer(closure):
    """src/utils/logging.py:14-31: HIP events around the step closure."""
    if not torch.cuda.is_available():
        return closure(), -1.0
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    res = closure()
    end.record()
    torch.cuda.synchronize()
    return res, start.elapsed_time(end)


# ------------------------------------------------------------------------------------------------
def main(args, resume_preempt=False):
    """app/vjepa/train.py:54-521 on the fused HIP step."""
    folder = args.get("folder", ".")
    cfgs_meta = args.get("meta")
    load_model = cfgs_meta.get("load_checkpoint") or resume_preempt
    r_file = cfgs_meta.get("read_checkpoint", None)
    seed = cfgs_meta.get("seed", _GLOBAL_SEED)
    save_every_freq = cfgs_meta.get("save_every_freq", -1)
    use_sdpa = cfgs_meta.get("use_sdpa", False)
    which_dtype = str(cfgs_meta.get("dtype", "float32")).lower()
    mixed_precision = which_dtype in ("bfloat16", "float16")
    if which_dtype == "float16":
        logger.warning("float16 autocast requested: the HIP path computes bf16 GEMM operands instead")
    cfgs_mask = args.get("mask")
    cm = args.get("model")
    cd = args.get("data")
    dataset_fpcs = cd.get("dataset_fpcs")
    batch_size = cd.get("batch_size")
    crop_size = cd.get("crop_size", 224)
    patch_size = cd.get("patch_size")
    tubelet_size = cd.get("tubelet_size")
    loss_exp = args.get("loss").get("loss_exp")
    co = args.get("optimization")
    ipe, ipe_scale = co.get("ipe", None), co.get("ipe_scale", 1.0)
    wd, final_wd = float(co.get("weight_decay")), float(co.get("final_weight_decay"))
    num_epochs, warmup = co.get("epochs"), co.get("warmup")
    start_lr, lr, final_lr = co.get("start_lr"), co.get("lr"), co.get("final_lr")
    ema = co.get("ema")
    betas, eps = co.get("betas", (0.9, 0.999)), co.get("eps", 1.0e-8)

    np.random.seed(seed)
    torch.manual_seed(seed)
    if not torch.cuda.is_available():
        raise RuntimeError("the V-JEPA HIP train step needs an MI355X (no CPU path)")
    # bind this rank's GPU BEFORE the process group: RCCL binds its communicator to the current device
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(device)
    world_size, rank = init_distributed()
    os.makedirs(folder, exist_ok=True)
    latest_path = os.path.join(folder, "latest.pt")
    load_path = os.path.join(folder, r_file) if r_file is not None else latest_path
    if not os.path.exists(load_path):
        load_model = False

    encoder, predictor = init_video_model(
        device=device, patch_size=patch_size, max_num_frames=max(dataset_fpcs), tubelet_size=tubelet_size,
        model_name=cm.get("model_name"), crop_size=crop_size, pred_depth=cm.get("pred_depth"),
        pred_num_heads=cm.get("pred_num_heads", None), pred_embed_dim=cm.get("pred_embed_dim"),
        uniform_power=cm.get("uniform_power", False), use_mask_tokens=cm.get("use_mask_tokens", False),
        num_mask_tokens=int(len(cfgs_mask) * len(dataset_fpcs)),
        zero_init_mask_tokens=cm.get("zero_init_mask_tokens", True), use_sdpa=use_sdpa,
        use_rope=cm.get("use_rope", False), use_silu=cm.get("use_silu", False),
        use_pred_silu=cm.get("use_pred_silu", False), wide_silu=cm.get("wide_silu", True),
        use_activation_checkpointing=cm.get("use_activation_checkpointing", False))
    target_encoder = copy.deepcopy(encoder)
    # masks built on the GPU from the collate's RNG draws (bit-exact with the host collate);
    # data.gpu_masks: false keeps the reference's host-side masks
    mask_collator = MaskCollator(cfgs_mask=cfgs_mask, dataset_fpcs=dataset_fpcs, crop_size=crop_size,
                                 patch_size=patch_size, tubelet_size=tubelet_size,
                                 device_masks=bool(cd.get("gpu_masks", True)))
    loader, sampler = init_data(batch_size=batch_size, collator=mask_collator, dataset_fpcs=dataset_fpcs,
                                crop_size=crop_size, rank=rank, world_size=world_size,
                                num_workers=cd.get("num_workers", 0))
    if ipe is None:
        ipe = len(loader)
    optimizer, scaler, scheduler, wd_scheduler = init_opt(
        encoder=encoder, predictor=predictor, wd=wd, final_wd=final_wd, start_lr=start_lr, ref_lr=lr,
        final_lr=final_lr, iterations_per_epoch=ipe, warmup=warmup, num_epochs=num_epochs, ipe_scale=ipe_scale,
        mixed_precision=mixed_precision, betas=betas, eps=eps)
    # meta.fp8_target (this build's opt-in key; the reference has no fp8 and ignores unknown keys)
    trainer = JEPATrainer(encoder, predictor, target_encoder, optimizer, mixed_precision=mixed_precision,
                          loss_exp=loss_exp, world_size=world_size, fp8_target=bool(cfgs_meta.get("fp8_target", False)))
    momentum_scheduler = (ema[0] + i * (ema[1] - ema[0]) / (ipe * num_epochs * ipe_scale)
                          for i in range(int(ipe * num_epochs * ipe_scale) + 1))
    start_epoch = 0
    if load_model:
        *_, start_epoch = load_checkpoint(load_path, encoder, predictor, target_encoder, optimizer, scaler, trainer)
        for _ in range(start_epoch * ipe):
            scheduler.step()
            wd_scheduler.step()
            next(momentum_scheduler)
            mask_collator.step()

    log_path = os.path.join(folder, f"log_r{rank}.csv")
    losses = []
    loader_it = iter(loader)
    for epoch in range(start_epoch, num_epochs):
        sampler.set_epoch(epoch)
        loss_sum = 0.0
        for itr in range(ipe):
            t0 = time.time()
            try:
                sample = next(loader_it)
            except StopIteration:
                loader_it = iter(loader)
                sample = next(loader_it)
            sample = [materialize(s, device) for s in sample]
            clips = [s[0][0][0].to(device, non_blocking=True) for s in sample]
            menc = [s[1] for s in sample]
            mpred = [s[2] for s in sample]
            data_ms = (time.time() - t0) * 1000.0

            def step():
                new_lr = scheduler.step()
                new_wd = wd_scheduler.step()
                m = next(momentum_scheduler)
                return float(trainer.train_step(clips, menc, mpred, m)), new_lr, new_wd

            (loss, new_lr, new_wd), gpu_ms = gpu_timer(step)
            losses.append(loss)
            loss_sum += loss
            with open(log_path, "a", newline="") as f:
                csv.writer(f).writerow([epoch + 1, itr, f"{loss:.5f}", int((time.time() - t0) * 1000), int(gpu_ms),
                                        int(data_ms)])
            if itr % 10 == 0 or itr == ipe - 1:
                logger.info("[%d, %5d] loss: %.3f [wd: %.2e] [lr: %.2e] [gpu: %.1f ms]", epoch + 1, itr, loss, new_wd,
                            new_lr, gpu_ms)
            assert not np.isnan(loss), "loss is nan"
        if rank == 0:
            save_checkpoint(latest_path, encoder, predictor, target_encoder, optimizer, scaler, epoch + 1,
                            loss_sum / max(1, ipe), batch_size, world_size, lr)
            if save_every_freq > 0 and epoch % save_every_freq == 0:
                save_checkpoint(os.path.join(folder, f"e{epoch}.pt"), encoder, predictor, target_encoder, optimizer,
                                scaler, epoch + 1, loss_sum / max(1, ipe), batch_size, world_size, lr)
    return losses
