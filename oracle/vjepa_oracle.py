"""ORACLE — test infrastructure only. CPU fp32 restatement of the reference V-JEPA 2 train step.

This module restates, in plain PyTorch CPU ops (fp32), the algorithm of weipeilun/vjepa2's hot path
so that the HIP product (vjepa2_amd/) can be checked against it. It is imported ONLY by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg — never by the product path.

Pinning: every function here is checked against golden fixtures produced by running the reference
itself (tests/golden/make_golden.py -> tests/golden/*.pt; tests/test_oracle_golden.py), i.e. the
oracle is "parity pinned" to the reference's own outputs at fp32.

Each function cites the reference file:line it follows (paths relative to the reference root).
Weights are passed as plain state-dict mappings using the reference's key names.
"""

import math

import numpy as np
import torch
import torch.nn.functional as F


# ------------------------------------------------------------------------------------------------
# src/models/utils/modules.py:26-50
def rotate_queries_or_keys(x, pos):
    """Quirky 'RoPE' of the reference: sin/cos tiled [t0..t(h-1), t0..t(h-1)], partner = adjacent pair."""
    D = x.shape[-1]
    half = D // 2
    omega = torch.arange(half, dtype=x.dtype)
    omega /= D / 2.0
    omega = 1.0 / 10000**omega
    freq = pos.to(x.dtype)[..., None] * omega  # (..., N, D/2)
    s = freq.sin()
    c = freq.cos()
    s = torch.cat([s, s], dim=-1)
    c = torch.cat([c, c], dim=-1)
    y = x.unflatten(-1, (-1, 2))
    y = torch.stack((-y[..., 1], y[..., 0]), dim=-1).flatten(-2)
    return x * c + y * s


def rope_tables(hd, max_pos):
    """cos/sin [max_pos, half] of the per-axis angles, computed with the reference's fp32 op order
    (modules.py:30-39): omega = 1 / 10000 ** (arange(half) / (sw/2)); theta = pos * omega."""
    sw = 2 * ((hd // 3) // 2)
    half = sw // 2
    omega = torch.arange(half, dtype=torch.float32)
    omega /= sw / 2.0
    omega = 1.0 / 10000**omega
    pos = torch.arange(max_pos, dtype=torch.float32)
    freq = pos[:, None] * omega[None, :]
    return freq.cos().contiguous(), freq.sin().contiguous()


# src/models/utils/modules.py:293-324
def separate_positions(ids, tokens_per_frame, tokens_per_row):
    frame = ids // tokens_per_frame
    rem = ids - tokens_per_frame * frame
    height = rem // tokens_per_row
    width = rem - tokens_per_row * height
    return frame, height, width


def apply_rope_qk(q, k, ids, tokens_per_frame, tokens_per_row):
    """q, k: [B, H, N, hd]; ids: [B, N] or [N] token ids (modules.py:333-365)."""
    hd = q.shape[-1]
    sw = 2 * ((hd // 3) // 2)
    if ids.dim() == 2:
        ids = ids[:, None, :].expand(-1, q.shape[1], -1)
    d, h, w = separate_positions(ids, tokens_per_frame, tokens_per_row)
    outs_q, outs_k = [], []
    s = 0
    for pos in (d, h, w):
        outs_q.append(rotate_queries_or_keys(q[..., s:s + sw], pos))
        outs_k.append(rotate_queries_or_keys(k[..., s:s + sw], pos))
        s += sw
    if s < hd:
        outs_q.append(q[..., s:])
        outs_k.append(k[..., s:])
    return torch.cat(outs_q, -1), torch.cat(outs_k, -1)


# ------------------------------------------------------------------------------------------------
# src/models/utils/modules.py:326-382 (RoPEAttention) and :385-429 (Attention)
def attention(x, sd, prefix, num_heads, ids=None, tokens_per_frame=None, tokens_per_row=None, use_rope=True):
    B, N, C = x.shape
    qkv = F.linear(x, sd[prefix + "qkv.weight"], sd[prefix + "qkv.bias"])
    qkv = qkv.unflatten(-1, (3, num_heads, -1)).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    if use_rope:
        if ids is None:
            ids = torch.arange(N)
        q, k = apply_rope_qk(q, k, ids, tokens_per_frame, tokens_per_row)
    o = F.scaled_dot_product_attention(q, k, v)
    o = o.transpose(1, 2).reshape(B, N, C)
    return F.linear(o, sd[prefix + "proj.weight"], sd[prefix + "proj.bias"])


# src/models/utils/modules.py:77-83 (MLP, GELU exact) / :102-106 (SwiGLUFFN: state dict with fc3)
def mlp(y, sd, prefix):
    if prefix + "fc3.weight" in sd:
        h = F.silu(F.linear(y, sd[prefix + "fc1.weight"], sd[prefix + "fc1.bias"]))
        h = h * F.linear(y, sd[prefix + "fc2.weight"], sd[prefix + "fc2.bias"])
        return F.linear(h, sd[prefix + "fc3.weight"], sd[prefix + "fc3.bias"])
    y = F.gelu(F.linear(y, sd[prefix + "fc1.weight"], sd[prefix + "fc1.bias"]))
    return F.linear(y, sd[prefix + "fc2.weight"], sd[prefix + "fc2.bias"])


# src/models/utils/modules.py:556-563 (Block). draws = the drop_path per-sample scales (timm
# drop_path: Bernoulli(1 - p) / (1 - p)) of the attention and MLP branches, [B] each, or None.
def block(x, sd, prefix, num_heads, eps=1e-6, draws=None, **rope_kw):
    D = x.shape[-1]
    y = F.layer_norm(x, (D,), sd[prefix + "norm1.weight"], sd[prefix + "norm1.bias"], eps)
    y = attention(y, sd, prefix + "attn.", num_heads, **rope_kw)
    x = x + (y if draws is None else y * draws[0].view(-1, 1, 1))
    y = F.layer_norm(x, (D,), sd[prefix + "norm2.weight"], sd[prefix + "norm2.bias"], eps)
    y = mlp(y, sd, prefix + "mlp.")
    return x + (y if draws is None else y * draws[1].view(-1, 1, 1))


# ------------------------------------------------------------------------------------------------
# src/models/utils/pos_embs.py:9-38, 75-93 (numpy float64)
def sincos_1d(embed_dim, pos):
    omega = np.arange(embed_dim // 2, dtype=float)
    omega /= embed_dim / 2.0
    omega = 1.0 / 10000**omega
    out = np.einsum("m,d->md", pos.reshape(-1), omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1)


def sincos_3d(embed_dim, grid_size, grid_depth, uniform_power=False):
    gd = np.arange(grid_depth, dtype=float)
    gh = np.arange(grid_size, dtype=float)
    gw = np.arange(grid_size, dtype=float)
    gh, gd, gw = np.meshgrid(gh, gd, gw)
    if not uniform_power:
        hdim = wdim = embed_dim // 4
        ddim = embed_dim // 2
    else:
        hdim = wdim = ddim = int(np.ceil(embed_dim / 6) * 2)
    e = np.concatenate([sincos_1d(ddim, gd), sincos_1d(hdim, gh), sincos_1d(wdim, gw)], axis=1)
    return e[:, :embed_dim]


# ------------------------------------------------------------------------------------------------
# src/masks/utils.py:9-21
def apply_masks(x, masks, concat=True):
    outs = [torch.gather(x, 1, m.unsqueeze(-1).expand(-1, -1, x.size(-1))) for m in masks]
    return torch.cat(outs, 0) if concat else outs


# src/models/vision_transformer.py:161-213 (video path, optional RoPE / sincos pos-embed)
def encoder_forward(x, sd, cfg, masks=None, eps=1e-6, final_norm=True):
    """cfg: dict(patch_size, tubelet_size, num_heads, depth, use_rope). x: [B, 3, T, H, W]."""
    p, tub = cfg["patch_size"], cfg["tubelet_size"]
    B, _, T, H, W = x.shape
    Tp, Hp, Wp = T // tub, H // p, W // p
    t = F.conv3d(x, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], stride=(tub, p, p))
    t = t.flatten(2).transpose(1, 2)
    if not cfg["use_rope"]:
        t = t + sd["pos_embed"]
    ids = None
    if masks is not None:
        if not isinstance(masks, list):
            masks = [masks]
        t = apply_masks(t, masks)
        ids = torch.cat(masks, 0)
    kw = dict(ids=ids, tokens_per_frame=Hp * Wp, tokens_per_row=Wp, use_rope=cfg["use_rope"])
    for i in range(cfg["depth"]):
        t = block(t, sd, f"blocks.{i}.", cfg["num_heads"], eps=eps, **kw)
    if final_norm:
        t = F.layer_norm(t, (t.shape[-1],), sd["norm.weight"], sd["norm.bias"], eps)
    return t


# src/models/predictor.py:166-246 (RoPE or sincos, mask tokens)
def predictor_forward(z, masks_x, masks_y, sd, cfg, mask_index=1, eps=1e-6):
    """cfg: dict(num_heads, depth, use_rope, grid_size, num_mask_tokens, num_patches)."""
    if not isinstance(masks_x, list):
        masks_x = [masks_x]
    if not isinstance(masks_y, list):
        masks_y = [masks_y]
    B = len(z) // len(masks_x)
    x = F.linear(z, sd["predictor_embed.weight"], sd["predictor_embed.bias"])
    _, Nc, Dp = x.shape
    if not cfg["use_rope"]:
        x = x + apply_masks(sd["predictor_pos_embed"].repeat(B, 1, 1), masks_x)
    tok = sd[f"mask_tokens.{mask_index % cfg['num_mask_tokens']}"]
    pred = apply_masks(tok.repeat(B, cfg["num_patches"], 1), masks_y)
    if not cfg["use_rope"]:
        pe = apply_masks(sd["predictor_pos_embed"].repeat(B, 1, 1), masks_y)
        pe = torch.cat([torch.cat([pe[i * B:(i + 1) * B] for _ in range(len(masks_x))], 0)
                        for i in range(len(pe) // B)], 0)
        pred = pred + pe
    x = x.repeat(len(masks_x), 1, 1)
    x = torch.cat([x, pred], 1)
    mx = torch.cat(masks_x, 0)
    my = torch.cat(masks_y, 0)
    m = torch.cat([mx, my], 1)
    order = torch.argsort(m, dim=1)
    m = torch.gather(m, 1, order)
    x = torch.gather(x, 1, order[..., None].expand(-1, -1, Dp))
    g = cfg["grid_size"]
    kw = dict(ids=m, tokens_per_frame=g * g, tokens_per_row=g, use_rope=cfg["use_rope"])
    for i in range(cfg["depth"]):
        x = block(x, sd, f"predictor_blocks.{i}.", cfg["num_heads"], eps=eps, **kw)
    x = F.layer_norm(x, (Dp,), sd["predictor_norm.weight"], sd["predictor_norm.bias"], eps)
    rev = torch.argsort(order, dim=1)
    x = torch.gather(x, 1, rev[..., None].expand(-1, -1, Dp))[:, Nc:]
    return F.linear(x, sd["predictor_proj.weight"], sd["predictor_proj.bias"])


# ------------------------------------------------------------------------------------------------
# app/vjepa/train.py:414-435
def jepa_loss(z_list, h, masks_pred, loss_exp=1.0):
    """z_list: predictor outputs per mask; h: target features [B, N, D] (already layer-normed)."""
    hs = apply_masks(h, masks_pred, concat=False)
    loss, n = 0.0, 0
    for zi, hi in zip(z_list, hs):
        loss = loss + torch.mean(torch.abs(zi - hi) ** loss_exp) / loss_exp
        n += 1
    return loss / n


def forward_target(x, sd_target, cfg):
    """train.py:414-418: target encoder (all tokens) + F.layer_norm (no affine, eps 1e-5)."""
    h = encoder_forward(x, sd_target, cfg)
    return F.layer_norm(h, (h.size(-1),))


# ------------------------------------------------------------------------------------------------
# src/utils/schedulers.py:41-93
class WarmupCosine:
    def __init__(self, warmup_steps, start_lr, ref_lr, T_max, final_lr=0.0):
        self.start_lr, self.ref_lr, self.final_lr = start_lr, ref_lr, final_lr
        self.warmup_steps, self.T_max, self._step = warmup_steps, T_max - warmup_steps, 0.0

    def step(self):
        self._step += 1
        if self._step < self.warmup_steps:
            return self.start_lr + float(self._step) / float(max(1, self.warmup_steps)) * (self.ref_lr - self.start_lr)
        progress = float(self._step - self.warmup_steps) / float(max(1, self.T_max))
        return max(self.final_lr,
                   self.final_lr + (self.ref_lr - self.final_lr) * 0.5 * (1.0 + math.cos(math.pi * progress)))


class CosineWD:
    def __init__(self, ref_wd, T_max, final_wd=0.0):
        self.ref_wd, self.final_wd, self.T_max, self._step = ref_wd, final_wd, T_max, 0.0

    def step(self):
        self._step += 1
        progress = self._step / self.T_max
        wd = self.final_wd + (self.ref_wd - self.final_wd) * 0.5 * (1.0 + math.cos(math.pi * progress))
        return max(self.final_wd, wd) if self.final_wd <= self.ref_wd else min(self.final_wd, wd)


# torch.optim.AdamW (foreach math) as configured by app/vjepa/utils.py:207-255
def adamw_step(p, g, m, v, step, lr, wd, beta1=0.9, beta2=0.999, eps=1e-8):
    p.mul_(1 - lr * wd)
    m.lerp_(g, 1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-(lr / bc1))


# app/vjepa/train.py:456-465
def ema_update(target, online, m):
    target.mul_(m)
    target.add_(online, alpha=1 - m)


# ------------------------------------------------------------------------------------------------
class OracleTrainer:
    """app/vjepa/train.py:409-471 restated on CPU fp32: per-mask encoder/predictor calls
    (wrappers.py:20-43), L1 loss, autograd backward, AdamW over the 4 param groups of
    app/vjepa/utils.py:224-237 (params with no gradient are skipped, as torch.optim does), EMA."""

    def __init__(self, enc_sd, pred_sd, enc_cfg, pred_cfg, betas=(0.9, 0.999), eps=1e-8, loss_exp=1.0):
        self.enc = {k: v.detach().clone().float().requires_grad_(k != "pos_embed") for k, v in enc_sd.items()}
        self.pred = {k: v.detach().clone().float().requires_grad_(k != "predictor_pos_embed")
                     for k, v in pred_sd.items()}
        self.tgt = {k: v.detach().clone().float() for k, v in enc_sd.items()}
        self.enc_cfg, self.pred_cfg = enc_cfg, pred_cfg
        self.betas, self.eps, self.loss_exp = betas, eps, loss_exp
        self.state = {}

    def loss(self, clips, masks_enc, masks_pred):
        with torch.no_grad():
            h = forward_target(clips, self.tgt, self.enc_cfg)
        z = [encoder_forward(clips, self.enc, self.enc_cfg, masks=m) for m in masks_enc]
        z = [predictor_forward(zi, mx, my, self.pred, self.pred_cfg, mask_index=0)
             for zi, mx, my in zip(z, masks_enc, masks_pred)]
        return jepa_loss(z, h, masks_pred, self.loss_exp)

    def loss_groups(self, groups):
        """train.py:414-435 with several frames-per-clip groups [(clips, masks_enc, masks_pred), ...]:
        group i's predictor uses mask token i (wrappers.py:36-43, mask_index = i) and the loss is the
        mean over every (group, mask) pair (train.py:429-434)."""
        tot, n = 0.0, 0
        for i, (clips, me, mp) in enumerate(groups):
            with torch.no_grad():
                h = forward_target(clips, self.tgt, self.enc_cfg)
            z = [encoder_forward(clips, self.enc, self.enc_cfg, masks=m) for m in me]
            z = [predictor_forward(zi, mx, my, self.pred, self.pred_cfg, mask_index=i)
                 for zi, mx, my in zip(z, me, mp)]
            tot = tot + jepa_loss(z, h, mp, self.loss_exp) * len(me)
            n += len(me)
        return tot / n

    def step_groups(self, groups, lr, wd, momentum):
        return self._update(self.loss_groups(groups), lr, wd, momentum)

    def step(self, clips, masks_enc, masks_pred, lr, wd, momentum):
        return self._update(self.loss(clips, masks_enc, masks_pred), lr, wd, momentum)

    def _update(self, loss, lr, wd, momentum):
        loss.backward()
        with torch.no_grad():
            for sd in (self.enc, self.pred):
                for k, p in sd.items():
                    if not p.requires_grad or p.grad is None:
                        continue
                    st = self.state.setdefault(id(p), dict(m=torch.zeros_like(p), v=torch.zeros_like(p), t=0))
                    st["t"] += 1
                    decay = 0.0 if ("bias" in k or p.dim() == 1) else wd
                    adamw_step(p, p.grad, st["m"], st["v"], st["t"], lr, decay, *self.betas, self.eps)
                    p.grad = None
            for k in self.tgt:
                ema_update(self.tgt[k], self.enc[k].detach(), momentum)
        return loss.item()


# app/vjepa/transforms.py:98-112 with src/datasets/utils/video/transforms.py:510-542 (crop + bilinear
# resize), :149-170 (flip) and transforms.py:139-152 (normalisation), for given draws
def video_transform(buffer, params, crop, mean, std):
    """buffer uint8 [T, H, W, C]; params (top, left, h, w, flip); mean / std per channel (0-1 units)."""
    i, j, h, w, flip = params
    x = buffer.to(torch.float32).permute(3, 0, 1, 2)  # C T H W
    x = x[:, :, i:i + h, j:j + w]
    x = F.interpolate(x, size=(crop, crop), mode="bilinear", align_corners=False)
    if flip:
        x = x.flip(-1)
    m = torch.tensor(mean, dtype=torch.float32) * 255.0
    s = torch.tensor(std, dtype=torch.float32) * 255.0
    C, T, H, W = x.shape
    x = x.reshape(C, -1).permute(1, 0)
    x = (x - m) / s
    return x.permute(1, 0).reshape(C, T, H, W)


# ------------------------------------------------------------------------------------------------
# Frozen-encoder consumers


# src/models/utils/modules.py:566-594 (CrossAttention: q / kv Linears, SDPA, no output projection)
def cross_attention(q, x, sd, prefix, num_heads):
    B, n, C = q.shape
    N = x.shape[1]
    hd = C // num_heads
    qh = F.linear(q, sd[prefix + "q.weight"], sd.get(prefix + "q.bias"))
    qh = qh.reshape(B, n, num_heads, hd).permute(0, 2, 1, 3)
    kv = F.linear(x, sd[prefix + "kv.weight"], sd.get(prefix + "kv.bias"))
    kv = kv.reshape(B, N, 2, num_heads, hd).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(qh, kv[0], kv[1])
    return o.transpose(1, 2).reshape(B, n, C)


# src/models/utils/modules.py:597-610 (CrossAttentionBlock: norm1 is applied to the KEYS' input x)
def cross_attention_block(q, x, sd, prefix, num_heads, eps=1e-5):
    D = q.shape[-1]
    xn = F.layer_norm(x, (D,), sd[prefix + "norm1.weight"], sd[prefix + "norm1.bias"], eps)
    q = q + cross_attention(q, xn, sd, prefix + "xattn.", num_heads)
    y = F.layer_norm(q, (D,), sd[prefix + "norm2.weight"], sd[prefix + "norm2.bias"], eps)
    y = F.gelu(F.linear(y, sd[prefix + "mlp.fc1.weight"], sd[prefix + "mlp.fc1.bias"]))
    return q + F.linear(y, sd[prefix + "mlp.fc2.weight"], sd[prefix + "mlp.fc2.bias"])


# src/models/attentive_pooler.py:91-100 (depth-1 self-attention Blocks without RoPE, then the queries)
def attentive_pooler(x, sd, prefix, num_heads, depth, complete_block=True, eps=1e-5):
    for i in range(depth - 1):
        x = block(x, sd, f"{prefix}blocks.{i}.", num_heads, eps=eps, use_rope=False)
    q = sd[prefix + "query_tokens"].repeat(len(x), 1, 1)
    if complete_block:
        return cross_attention_block(q, x, sd, prefix + "cross_attention_block.", num_heads, eps)
    return cross_attention(q, x, sd, prefix + "cross_attention_block.", num_heads)


# src/models/attentive_pooler.py:134-137
def attentive_classifier(x, sd, num_heads, depth, complete_block=True, eps=1e-5):
    x = attentive_pooler(x, sd, "pooler.", num_heads, depth, complete_block, eps).squeeze(1)
    return F.linear(x, sd["linear.weight"], sd["linear.bias"])


# evals/video_classification_frozen/modelcustom/vit_encoder_multiclip.py:117-162 (ClipAggregation)
def clip_aggregation(x, encode, tubelet_size, pos_embed=None, clip_indices=None):
    """x: list (clips) of lists (views) of [B, C, F, H, W]; encode: clips -> [*, N, D] tokens;
    pos_embed [1, max_T, D] or None. Returns a list (views) of [B, clips*T*S, D]."""
    num_clips, num_views = len(x), len(x[0])
    B, C, Fr, H, W = x[0][0].size()
    outputs = encode(torch.cat([torch.cat(xi, dim=0) for xi in x], dim=0))
    _, N, D = outputs.size()
    T = Fr // tubelet_size
    S = N // T
    eff_B = B * num_views
    views = [[] for _ in range(num_views)]
    for i in range(num_clips):
        o = outputs[i * eff_B:(i + 1) * eff_B]
        for j in range(num_views):
            views[j].append(o[j * B:(j + 1) * B])
    res = []
    for outs in views:
        out = torch.cat([o.reshape(B, T, S, D) for o in outs], dim=1).flatten(1, 2)
        if pos_embed is not None and clip_indices is not None:
            idx = [c[:, ::tubelet_size] for c in clip_indices]
            pe = pos_embed.repeat(B, 1, 1)
            pe = torch.cat([apply_masks(pe, [i], concat=False)[0] for i in idx], dim=1)
            out = out + pe.unsqueeze(2).repeat(1, 1, S, 1).flatten(1, 2)
        res.append(out)
    return res


# ------------------------------------------------------------------------------------------------
# V-JEPA 2-AC action-conditioned predictor


# src/models/utils/modules.py:12-23
def action_block_causal_mask(T, H, W, add_tokens=1):
    n_t = add_tokens + H * W
    mask = torch.zeros(T * n_t, T * n_t, dtype=torch.bool)
    for t1 in range(T):
        for t2 in range(0, t1 + 1):
            mask[t1 * n_t:(t1 + 1) * n_t, t2 * n_t:(t2 + 1) * n_t] = True
    return mask


# src/models/utils/modules.py:163-258 (ACRoPEAttention.forward, mask=None)
def ac_rope_attention(x, sd, prefix, num_heads, T, H, W, action_tokens, attn_mask, grid_size):
    B, N, C = x.shape
    hd = C // num_heads
    sw = 2 * ((hd // 3) // 2)
    ids = torch.arange(T * H * W)
    d, h, w = (p.float() for p in separate_positions(ids, H * W, W))
    h = h * (grid_size / H)
    w = w * (grid_size / W)

    def qkv_of(t):
        return F.linear(t, sd[prefix + "qkv.weight"], sd[prefix + "qkv.bias"]).unflatten(
            -1, (3, num_heads, hd)).permute(2, 0, 3, 1, 4)

    xv = x.view(B, T, action_tokens + H * W, C)
    aq, ak, av = [], [], []
    for i in range(action_tokens):  # :183-200: depth slice rotated by the frame index, the rest as is
        q, k, v = qkv_of(xv[:, :, i])
        pos = torch.arange(T).float()
        aq.append(torch.cat([rotate_queries_or_keys(q[..., :sw], pos), q[..., sw:]], -1))
        ak.append(torch.cat([rotate_queries_or_keys(k[..., :sw], pos), k[..., sw:]], -1))
        av.append(v)
    q, k, v = qkv_of(xv[:, :, action_tokens:].flatten(1, 2))
    qs, ks = [], []
    for ax, pos in enumerate((d, h, w)):
        qs.append(rotate_queries_or_keys(q[..., ax * sw:(ax + 1) * sw], pos))
        ks.append(rotate_queries_or_keys(k[..., ax * sw:(ax + 1) * sw], pos))
    q = torch.cat(qs + [q[..., 3 * sw:]], -1)
    k = torch.cat(ks + [k[..., 3 * sw:]], -1)

    def merge(tx, ta):  # :233-241: per frame, the action tokens first
        tx = tx.reshape(B, num_heads, T, H * W, hd)
        ta = torch.stack(ta, dim=3)  # [B, heads, T, A, hd]
        return torch.cat([ta, tx], dim=3).flatten(2, 3)

    if action_tokens > 0:
        q, k, v = merge(q, aq), merge(k, ak), merge(v, av)
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask)
    o = o.transpose(1, 2).reshape(B, N, C)
    return F.linear(o, sd[prefix + "proj.weight"], sd[prefix + "proj.bias"])


# src/models/utils/modules.py:488-497 (ACBlock with ACRoPEAttention; GELU MLP or SwiGLUFFN; draws =
# the drop_path per-sample scales of the attention and MLP branches, or None)
def ac_block(x, sd, prefix, num_heads, T, H, W, action_tokens, attn_mask, grid_size, eps=1e-6, draws=None):
    D = x.shape[-1]
    y = F.layer_norm(x, (D,), sd[prefix + "norm1.weight"], sd[prefix + "norm1.bias"], eps)
    y = ac_rope_attention(y, sd, prefix + "attn.", num_heads, T, H, W, action_tokens, attn_mask, grid_size)
    x = x + (y if draws is None else y * draws[0].view(-1, 1, 1))
    y = F.layer_norm(x, (D,), sd[prefix + "norm2.weight"], sd[prefix + "norm2.bias"], eps)
    y = mlp(y, sd, prefix + "mlp.")
    return x + (y if draws is None else y * draws[1].view(-1, 1, 1))


# src/models/ac_predictor.py:141-190
def ac_predictor_forward(x, actions, states, sd, cfg, extrinsics=None, eps=1e-6, block_draws=None):
    gh = gw = cfg["grid"]
    x = F.linear(x, sd["predictor_embed.weight"], sd["predictor_embed.bias"])
    B, N_ctxt, D = x.shape
    T = N_ctxt // (gh * gw)
    s = F.linear(states, sd["state_encoder.weight"], sd["state_encoder.bias"]).unsqueeze(2)
    a = F.linear(actions, sd["action_encoder.weight"], sd["action_encoder.bias"]).unsqueeze(2)
    x = x.view(B, T, gh * gw, D)
    if cfg["use_extrinsics"]:
        e = F.linear(extrinsics, sd["extrinsics_encoder.weight"], sd["extrinsics_encoder.bias"]).unsqueeze(2)
        x = torch.cat([a, s, e, x], dim=2).flatten(1, 2)
    else:
        x = torch.cat([a, s, x], dim=2).flatten(1, 2)
    cond = 3 if cfg["use_extrinsics"] else 2
    mask = None
    if cfg["is_frame_causal"]:
        mask = action_block_causal_mask(cfg["num_frames"] // cfg["tubelet_size"], gh, gw, cond)
        mask = mask[:x.size(1), :x.size(1)]
    for i in range(cfg["depth"]):
        x = ac_block(x, sd, f"predictor_blocks.{i}.", cfg["num_heads"], T, gh, gw, cond, mask, gh, eps,
                     draws=block_draws[i] if block_draws else None)
    x = x.view(B, T, cond + gh * gw, D)[:, :, cond:].flatten(1, 2)
    x = F.layer_norm(x, (D,), sd["predictor_norm.weight"], sd["predictor_norm.bias"], eps)
    return F.linear(x, sd["predictor_proj.weight"], sd["predictor_proj.bias"])
