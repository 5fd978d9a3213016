"""Tensor-level wrappers over the HIP kernels (libvjepa_hip.so).

Every function validates shapes/dtypes/devices on the host (so a kernel never sees an operand it
was not written for), then enqueues the kernel on torch's current HIP stream. No CPU fallback.
"""

import os

import torch

from ._lib import call, int_array

EPI_BF16, EPI_F32, EPI_F32_RESID, EPI_GELU, EPI_GELU_BWD = 0, 1, 2, 3, 4
EPI_ROPE, EPI_PARTIAL = 5, 6  # internal to the library (vj_qkv_rope_gemm / split-K slabs): not for vj_gemm_bf16
EPI_BF16_RESID = 7  # bf16 residual in, bf16 out (no-grad target encoder: the reference's autocast precision)
EPI_NAMES = ["EPI_BF16", "EPI_F32", "EPI_F32_RESID", "EPI_GELU", "EPI_GELU_BWD", "EPI_ROPE", "EPI_PARTIAL", "EPI_BF16_RESID"]
BF16 = torch.bfloat16
F32 = torch.float32


_SHAPE_LABELS = bool(int(__import__("os").environ.get("VJ_SHAPE_LABELS", "0")))
# A/B knob: VJ_WGRAD_BIAS=0 computes the bias gradients by a separate column-sum pass (the pre-round-6 path)
_WGRAD_BIAS = os.environ.get("VJ_WGRAD_BIAS", "1") != "0"


class KernelEvents:
    """Per-launch HIP-event timing of the library's kernels on the launching (current) stream,
    with the algorithmic FLOPs of each launch (bench.py roofline). Active only between start/stop."""

    active = None

    def __init__(self, only=None):
        self.rec = []
        self.only = only  # None: every launch; else the set of labels to time (cheap enough for a timed region)

    def start(self):
        KernelEvents.active = self

    def stop(self):
        KernelEvents.active = None
        torch.cuda.synchronize()

    def summary(self):
        out = {}
        for name, flops, s, e in self.rec:
            d = out.setdefault(name, dict(count=0, total_ms=0.0, flops=0.0))
            d["count"] += 1
            d["total_ms"] += s.elapsed_time(e)
            d["flops"] += flops
        return out


def _call(fn, *args, label=None, flops=0):
    prof = KernelEvents.active
    if prof is None or (prof.only is not None and (label or fn) not in prof.only):
        return call(fn, *args)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    rc = call(fn, *args)
    e.record()
    prof.rec.append((label or fn, flops, s, e))
    return rc


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("vjepa2_amd ops require device (HIP) tensors; there is no CPU path")


def _rowmajor(t, name):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a 2-D row-major tensor (stride(1)==1), got {tuple(t.shape)} {t.stride()}")
    return t.stride(0)


# ------------------------------------------------------------------------------------------------
# GEMMs (nn.Linear forward / dgrad / wgrad)
def gemm(M, N, K, a, lda, a_kmajor, b, ldb, b_kmajor, epi, out=None, ldc=0, out2=None, ldc2=0, bias=None, aux=None,
         ldaux=0, splitk=1):
    _dev(a, b, out, out2, bias, aux)
    if a.dtype != BF16 or b.dtype != BF16:
        raise TypeError("gemm operands must be bf16")
    if bias is not None and (bias.dtype != F32 or bias.numel() < N):
        raise TypeError("gemm bias must be f32 [N]")
    label = f"k_gemm<{int(a_kmajor)},{int(b_kmajor)},{EPI_NAMES[epi]}>"
    if _SHAPE_LABELS:  # diagnostics (VJ_SHAPE_LABELS=1): per-shape kernel-event labels
        label += f"[{M}x{N}x{K}]"
    splitk = _effective_splitk(K, splitk)
    if splitk > 1:
        ws = torch.empty(splitk * M * N, dtype=F32, device=a.device)
        _call("vj_gemm_bf16_splitk", M, N, K, _p(a), lda, int(a_kmajor), _p(b), ldb, int(b_kmajor), epi, _p(bias),
              _p(aux), ldaux, _p(out), ldc, _p(out2), ldc2, splitk, _p(ws), ws.numel(), _stream(),
              label=label + "[splitk]", flops=2.0 * M * N * K)
        return
    _call("vj_gemm_bf16", M, N, K, _p(a), lda, int(a_kmajor), _p(b), ldb, int(b_kmajor), epi, _p(bias), _p(aux), ldaux,
          _p(out), ldc, _p(out2), ldc2, _stream(), label=label, flops=2.0 * M * N * K)


def _effective_splitk(K, splitk):
    """The library's slicing: kslice = ceil(ceil(K / splitk) / 64) * 64, splitk = ceil(K / kslice)."""
    if splitk <= 1:
        return 1
    kslice = (K + splitk - 1) // splitk
    kslice = (kslice + 63) // 64 * 64
    return (K + kslice - 1) // kslice


def wgrad_splitk(M, N, K, cus=None):
    """Split K (tokens) of a weight-gradient GEMM [M, N] += A[M, K] B[K, N]. Tiles are 256 x (256 or
    128) when M >= 256 and N >= 128 (the C side's choice), else 128 x 128. Picks the split that
    minimises (waves of tiles on the CUs) x (work per tile) + the f32 partial-slab traffic, keeping
    >= 512 of K per slice. `cus`: the CUs the GEMM is sized for — the whole chip. With the weight
    gradients on their own stream (functions.wgrad_stream) sizing for half the chip measured the same
    step time (round 5: 222.6 vs 222.7 clips/s; round 4 had read +0.3 % for it, inside the noise),
    for 64 / 32 CUs 5 / 8 % slower (profiles/r05_wgrad_experiments_step_ab.txt); run alone (the
    serialised profile) the half-chip split left half the CUs idle. The split does not depend on the
    stream setting: it fixes the summation order, so the gradients are bitwise independent of the
    stream configuration (tests/test_gpu_production.py)."""
    if cus is None:
        cus = 256
    if M >= 256 and N >= 128:  # the C side's column-tile rule (vj_gemm256.hip wide_tile_ok)
        wide = N % 256 == 0 or (N > 256 and -(-N // 256) * 256 * 100 <= 115 * N)
        tm, tn, per_cu = 256, (256 if wide else 128), 1
    else:
        tm, tn, per_cu = 128, 128, 2
    tiles = -(-M // tm) * -(-N // tn)
    best, best_t = 1, None
    for s in range(1, max(1, K // 512) + 1):
        waves = -(-tiles * s // (cus * per_cu))
        # ~1 PF/s over 256 CUs for the MFMA work, ~5 TB/s for writing + re-reading the slabs
        t = waves * (K / s) * tm * tn * 2 / 3.9e12 + (s * M * N * 8 / 5.0e12 if s > 1 else 0.0)
        if best_t is None or t < best_t * 0.98:
            best, best_t = s, t
    return best


def linear_fwd(x, w, bias=None, epi=EPI_BF16, out=None, out2=None, resid=None):
    """Y = X W^T + b.  x bf16 [M,K] row-major, w bf16 [N,K].  Returns the output tensor(s).
    EPI_GELU: (out, out2) = (GELU'(pre) bf16 if `out` is given (saved for the backward, EPI_GELU_BWD)
    else None, GELU(pre) bf16), pre = the bf16-rounded X W^T + b."""
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K, (tuple(x.shape), tuple(w.shape))
    if K % 8:  # 16-B operand rows: zero-pad the reduction dim (e.g. the 7-wide action / state encoders)
        x, w = _pad_cols(x), _pad_cols(w)
        K = x.shape[1]
    lda = _rowmajor(x, "x")
    ldb = _rowmajor(w, "w")
    if epi == EPI_BF16:
        out = out if out is not None else torch.empty(M, N, dtype=BF16, device=x.device)
    elif epi in (EPI_F32, EPI_F32_RESID):
        out = out if out is not None else torch.empty(M, N, dtype=F32, device=x.device)
        if epi == EPI_F32_RESID:
            assert resid is not None and resid.dtype == F32 and resid.shape == (M, N)
    elif epi == EPI_GELU:
        out2 = out2 if out2 is not None else torch.empty(M, N, dtype=BF16, device=x.device)
    elif epi == EPI_BF16_RESID:
        assert resid is not None and resid.dtype == BF16 and resid.shape == (M, N)
        out = out if out is not None else torch.empty(M, N, dtype=BF16, device=x.device)
    ldc = out.stride(0) if out is not None else 0
    ldc2 = out2.stride(0) if out2 is not None else 0
    gemm(M, N, K, x, lda, True, w, ldb, True, epi, out=out, ldc=ldc, out2=out2, ldc2=ldc2, bias=bias,
         aux=resid, ldaux=resid.stride(0) if resid is not None else 0)
    return (out, out2) if epi == EPI_GELU else out


def linear_dgrad(dy, w, out=None, gelu_grad=None, wt=None, resid=None):
    """dX = dY W (bf16 out); with gelu_grad (the GELU derivative the forward's EPI_GELU saved): dX = (dY W) * gelu_grad. `wt` = W^T [K, N] contiguous (the
    K-major B operand the paired GEMM reads); without it W is read MN-major (256-row kernel).
    resid (bf16 [M, K], needs wt): dX = resid + dY W (the gradient of an input read by two Linears)."""
    if resid is not None:
        M, K = dy.shape[0], w.shape[1]
        assert gelu_grad is None and wt is not None and resid.dtype == BF16 and resid.shape == (M, K)
        assert dy.shape[1] % 8 == 0 and K % 8 == 0
        out = out if out is not None else torch.empty(M, K, dtype=BF16, device=dy.device)
        gemm(M, K, dy.shape[1], dy, _rowmajor(dy, "dy"), True, wt, _rowmajor(wt, "wt"), True, EPI_BF16_RESID, out=out,
             ldc=out.stride(0), aux=resid, ldaux=_rowmajor(resid, "resid"))
        return out
    M, N = dy.shape
    K = w.shape[1]
    assert w.shape[0] == N
    if N % 8:  # the GEMM's K (= N here) must be a multiple of 8 (16-B DMA rows): zero-pad dY's columns
        dy, w, wt = _pad_cols(dy), _pad_rows(w), None  # and W's rows (a classifier head's num_classes)
        N = dy.shape[1]
    if K % 8:  # output width not a multiple of 8: compute into padded columns, return the view
        assert gelu_grad is None and out is None
        return linear_dgrad(dy, _pad_cols(w))[:, :K]
    out = out if out is not None else torch.empty(M, K, dtype=BF16, device=dy.device)
    epi = EPI_GELU_BWD if gelu_grad is not None else EPI_BF16
    aux = dict(aux=gelu_grad, ldaux=gelu_grad.stride(0) if gelu_grad is not None else 0)
    if wt is not None:
        assert wt.shape == (K, N), (tuple(wt.shape), (K, N))
        gemm(M, K, N, dy, _rowmajor(dy, "dy"), True, wt, _rowmajor(wt, "wt"), True, epi, out=out, ldc=out.stride(0),
             **aux)
    else:
        gemm(M, K, N, dy, _rowmajor(dy, "dy"), True, w, _rowmajor(w, "w"), False, epi, out=out, ldc=out.stride(0),
             **aux)
    return out


def transpose_bf16(x, out=None):
    """out[c, r] = x[r, c] (bf16, HIP kernel)."""
    _dev(x)
    assert x.dtype == BF16 and x.dim() == 2
    R, C = x.shape
    out = out if out is not None else torch.empty(C, R, dtype=BF16, device=x.device)
    _call("vj_transpose_bf16", R, C, _p(x), _rowmajor(x, "x"), _p(out), _rowmajor(out, "out"), _stream())
    return out


def transpose_batch_desc(pairs):
    """Device descriptor table of vj_transpose_bf16_batch for [(src [R, C], dst [C, R]), ...]:
    int64 [n][8] = {src, dst, R, C, ld_src, ld_dst, first 64x64 tile, tiles across}. Returns (table,
    total tiles). Built once per weight set (the pointers stay fixed)."""
    rows, tiles = [], 0
    for src, dst in pairs:
        _dev(src, dst)
        R, C = src.shape
        assert src.dtype == BF16 and dst.dtype == BF16 and dst.shape == (C, R), (tuple(src.shape), tuple(dst.shape))
        lds, ldd = _rowmajor(src, "src"), _rowmajor(dst, "dst")
        if R % 8 or C % 8 or lds % 8 or ldd % 8 or (src.data_ptr() | dst.data_ptr()) & 15:
            raise ValueError("transpose_batch_desc: rows, cols, strides must be multiples of 8, pointers 16-B aligned")
        tx, ty = -(-C // 64), -(-R // 64)
        rows.append([src.data_ptr(), dst.data_ptr(), R, C, lds, ldd, tiles, tx])
        tiles += tx * ty
    return torch.tensor(rows, dtype=torch.int64).to(pairs[0][0].device), tiles


def transpose_bf16_batch(desc, n, tiles):
    """One launch of n transposes described by transpose_batch_desc's table."""
    _call("vj_transpose_bf16_batch", n, _p(desc), tiles, _stream())


def _pad_cols(t):
    """[R, C] -> [R, C rounded up to 8], zero columns appended (GEMM operand rows are 16-B chunks)."""
    out = torch.zeros(t.shape[0], (t.shape[1] + 7) // 8 * 8, dtype=t.dtype, device=t.device)
    out[:, :t.shape[1]] = t
    return out


def _pad_rows(t):
    out = torch.zeros((t.shape[0] + 7) // 8 * 8, t.shape[1], dtype=t.dtype, device=t.device)
    out[:t.shape[0]] = t
    return out


def linear_wgrad(dy, x, dw, accumulate=True, db=None):
    """dW[N,K] += dY^T X  (f32 accumulate into dw); accumulate=False: dW = dY^T X (overwrite).
    db (f32 [N] or None): db += dY.sum(0), the bias gradient, from the same GEMM (vj_gemm_bf16_wgrad)."""
    M, N = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dw.shape == (N, K) and dw.dtype == F32
    if db is not None and (N % 8 or K % 8 or not _WGRAD_BIAS):
        linear_wgrad(dy, x, dw, accumulate)
        return colsum(dy, db)
    if db is not None:
        _dev(dy, x, dw, db)
        assert db.dtype == F32 and db.numel() == N and db.is_contiguous()
        s = wgrad_splitk(N, K, M)
        s = _effective_splitk(M, s)
        nws = max(s * (N * K + N) if s > 1 else 0, min(256, max(1, (M + 63) // 64)) * N)
        ws = torch.empty(nws, dtype=F32, device=dy.device)
        _call("vj_gemm_bf16_wgrad", N, K, M, _p(dy), _rowmajor(dy, "dy"), _p(x), _rowmajor(x, "x"), _p(dw),
              _rowmajor(dw, "dw"), int(accumulate), _p(db), 1, s, _p(ws), ws.numel(), _stream(),
              label="k_gemm<0,0,wgrad+bias>", flops=2.0 * M * N * K)
        return dw
    if N % 8:  # dY^T is the MN-major A operand: its contiguous dim N must be a multiple of 8
        tmp = torch.zeros((N + 7) // 8 * 8, K, dtype=F32, device=dw.device)
        linear_wgrad(_pad_cols(dy), x, tmp)
        if accumulate:
            dw += tmp[:N]
        else:
            dw.copy_(tmp[:N])
        return dw
    if K % 8:  # X is the MN-major B operand: same for its width K
        tmp = torch.zeros(N, (K + 7) // 8 * 8, dtype=F32, device=dw.device)
        linear_wgrad(dy, _pad_cols(x), tmp)
        if accumulate:
            dw += tmp[:, :K]
        else:
            dw.copy_(tmp[:, :K])
        return dw
    if accumulate:
        gemm(N, K, M, dy, _rowmajor(dy, "dy"), False, x, _rowmajor(x, "x"), False, EPI_F32_RESID, out=dw,
             ldc=dw.stride(0), aux=dw, ldaux=dw.stride(0), splitk=wgrad_splitk(N, K, M))
    else:
        gemm(N, K, M, dy, _rowmajor(dy, "dy"), False, x, _rowmajor(x, "x"), False, EPI_F32, out=dw,
             ldc=dw.stride(0), splitk=wgrad_splitk(N, K, M))
    return dw


# ------------------------------------------------------------------------------------------------
# Block variants (vj_variants.hip): SwiGLU gate and drop_path row scaling
def swiglu_fwd(x12, out=None):
    """x12 bf16 [M, 2h] = fc1(x) | fc2(x) -> bf16 [M, h] = silu(x1) * x2 (SwiGLUFFN, modules.py:102-106)."""
    _dev(x12, out)
    assert x12.dtype == BF16 and x12.shape[1] % 2 == 0
    M, h = x12.shape[0], x12.shape[1] // 2
    out = out if out is not None else torch.empty(M, h, dtype=BF16, device=x12.device)
    _call("vj_swiglu_fwd", M, h, _p(x12), _rowmajor(x12, "x12"), _p(out), _rowmajor(out, "out"), _stream())
    return out


def swiglu_bwd(dh, x12, out=None):
    """dh bf16 [M, h], x12 (the forward's fc1 | fc2 outputs) -> dx12 bf16 [M, 2h] = dx1 | dx2."""
    _dev(dh, x12, out)
    M, h = dh.shape
    assert dh.dtype == BF16 and x12.dtype == BF16 and x12.shape == (M, 2 * h)
    out = out if out is not None else torch.empty(M, 2 * h, dtype=BF16, device=dh.device)
    _call("vj_swiglu_bwd", M, h, _p(dh), _rowmajor(dh, "dh"), _p(x12), _rowmajor(x12, "x12"), _p(out),
          _rowmajor(out, "out"), _stream())
    return out


def rowscale_add(y, scale, resid, out=None):
    """resid + bf16(bf16(y) * scale[row]) (drop_path on a residual branch): y f32 [M, N], scale f32 [M],
    resid f32 or bf16 [M, N] (out in resid's dtype)."""
    _dev(y, scale, resid, out)
    M, N = y.shape
    assert y.dtype == F32 and scale.dtype == F32 and scale.numel() == M and resid.shape == (M, N)
    out = out if out is not None else torch.empty_like(resid)
    _call("vj_rowscale_add", M, N, _p(y), _rowmajor(y, "y"), _p(scale), _p(resid), _rowmajor(resid, "resid"), _p(out),
          _rowmajor(out, "out"), int(resid.dtype == BF16), _stream())
    return out


def rowscale_bf16(dx, scale, out=None):
    """bf16(bf16(dx) * scale[row]): dx f32 [M, N] -> bf16 [M, N] (drop_path's backward)."""
    _dev(dx, scale, out)
    M, N = dx.shape
    assert dx.dtype == F32 and scale.dtype == F32 and scale.numel() == M
    out = out if out is not None else torch.empty(M, N, dtype=BF16, device=dx.device)
    _call("vj_rowscale_bf16", M, N, _p(dx), _rowmajor(dx, "dx"), _p(scale), _p(out), _rowmajor(out, "out"), _stream())
    return out


# ------------------------------------------------------------------------------------------------
def colsum(x, out, accumulate=True):
    """out[n] (+)= sum_m x[m, n]; x bf16 or f32 [M,N]."""
    _dev(x, out)
    M, N = x.shape
    if N % 8:  # 16-B row chunks: zero-pad the columns (a classifier head's bias gradient)
        tmp = torch.zeros((N + 7) // 8 * 8, dtype=F32, device=x.device)
        colsum(_pad_cols(x), tmp, accumulate=False)
        if accumulate:
            out += tmp[:N]
        else:
            out.copy_(tmp[:N])
        return out
    S = min(256, max(1, (M + 63) // 64))
    ws = torch.empty(S * N, dtype=F32, device=x.device)
    _call("vj_colsum_f32", M, N, _p(x), int(x.dtype == BF16), _rowmajor(x, "x"), _p(out), int(accumulate), _p(ws),
         ws.numel(), _stream())
    return out


def layernorm_fwd(x, weight, bias, eps, out_dtype=BF16, want_stats=True):
    _dev(x)
    M, D = x.shape
    y = torch.empty(M, D, dtype=out_dtype, device=x.device)
    mean = torch.empty(M, dtype=F32, device=x.device) if want_stats else None
    rstd = torch.empty(M, dtype=F32, device=x.device) if want_stats else None
    _call("vj_layernorm_fwd", M, D, _p(x), int(x.dtype == BF16), _rowmajor(x, "x"), _p(weight), _p(bias), float(eps),
         _p(y), int(out_dtype == F32), D, _p(mean), _p(rstd), _stream())
    return y, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, weight, dres_in=None, dweight=None, dbias=None, want_bf16=False, sum_in=None,
                  sum_out=None):
    """Returns (dres f32 = dres_in + dLN/dx, optional bf16 copy). Accumulates dweight/dbias and the
    column sums of dres_in / dres into sum_in / sum_out (fused bias gradients).
    x bf16 (the bf16 residual stream): dres_in bf16 (or None) and dres is bf16 only -> (dres, dres)."""
    _dev(dy, x)
    M, D = x.shape
    assert dy.dtype == BF16 and dy.shape == (M, D)
    assert sum_in is None or dres_in is not None
    if x.dtype == BF16:
        assert dres_in is None or (dres_in.dtype == BF16 and dres_in.shape == (M, D))
        dres = torch.empty(M, D, dtype=BF16, device=x.device)
        nsum = 4 if (sum_in is not None or sum_out is not None) else (2 if (dweight is not None or dbias is not None) else 0)
        ws, nws = None, 0
        if nsum:
            from ._lib import load

            nws = load().vj_layernorm_bwd_blocks(M) * nsum * D
            ws = torch.empty(nws, dtype=F32, device=x.device)
        _call("vj_layernorm_bwd_bf16", M, D, _p(dy), _rowmajor(dy, "dy"), _p(x), _rowmajor(x, "x"), _p(mean),
              _p(rstd), _p(weight), _p(dres_in), _rowmajor(dres_in, "dres_in") if dres_in is not None else 0, _p(dres),
              D, _p(dweight), _p(dbias), _p(sum_in), _p(sum_out), _p(ws), nws, _stream())
        return dres, dres
    dres = torch.empty(M, D, dtype=F32, device=x.device)
    dres_bf = torch.empty(M, D, dtype=BF16, device=x.device) if want_bf16 else None
    nsum = 4 if (sum_in is not None or sum_out is not None) else (2 if (dweight is not None or dbias is not None) else 0)
    ws = None
    nws = 0
    if nsum:
        from ._lib import load

        nws = load().vj_layernorm_bwd_blocks(M) * nsum * D
        ws = torch.empty(nws, dtype=F32, device=x.device)
    _call("vj_layernorm_bwd", M, D, _p(dy), _rowmajor(dy, "dy"), _p(x), _rowmajor(x, "x"), _p(mean), _p(rstd),
          _p(weight), _p(dres_in), dres_in.stride(0) if dres_in is not None else 0, _p(dres), D, _p(dres_bf), D,
          _p(dweight), _p(dbias), _p(sum_in), _p(sum_out), _p(ws), nws, _stream())
    return dres, dres_bf


# ------------------------------------------------------------------------------------------------
# fp8 (OCP e4m3) with per-row power-of-two scales: (bytes uint8 [M, K], exponents int32 [M])
FP8 = torch.uint8


def quant_rows_fp8(x, out=None, exps=None):
    """Per-row scaled e4m3 of x f32 / bf16 [M, K] -> (uint8 [M, K], int32 [M])."""
    _dev(x)
    M, K = x.shape
    out = out if out is not None else torch.empty(M, K, dtype=FP8, device=x.device)
    exps = exps if exps is not None else torch.empty(M, dtype=torch.int32, device=x.device)
    _call("vj_quant_rows_fp8", M, K, _p(x), int(x.dtype == BF16), _rowmajor(x, "x"), _p(out), _rowmajor(out, "out"),
          _p(exps), _stream())
    return out, exps


def layernorm_fwd_fp8(x, weight, bias, eps):
    """LayerNorm with a per-row scaled e4m3 output -> (uint8 [M, D], int32 [M])."""
    _dev(x)
    M, D = x.shape
    y = torch.empty(M, D, dtype=FP8, device=x.device)
    e = torch.empty(M, dtype=torch.int32, device=x.device)
    _call("vj_layernorm_fwd_fp8", M, D, _p(x), int(x.dtype == BF16), _rowmajor(x, "x"), _p(weight), _p(bias),
          float(eps), _p(y), D, _p(e), None, None, _stream())
    return y, e


def linear_fwd_fp8(x8, ex, w8, ew, bias=None, epi=EPI_BF16, out=None, out2=None, resid=None):
    """Y = (x8 * 2^ex) (w8 * 2^ew)^T + b on the fp8 MFMA; epilogues as linear_fwd."""
    _dev(x8, w8, bias, resid)
    assert x8.dtype == FP8 and w8.dtype == FP8 and ex.dtype == torch.int32 and ew.dtype == torch.int32
    M, K = x8.shape
    N = w8.shape[0]
    assert w8.shape[1] == K
    if epi == EPI_BF16:
        out = out if out is not None else torch.empty(M, N, dtype=BF16, device=x8.device)
    elif epi in (EPI_F32, EPI_F32_RESID):
        out = out if out is not None else torch.empty(M, N, dtype=F32, device=x8.device)
    elif epi == EPI_GELU:
        out2 = out2 if out2 is not None else torch.empty(M, N, dtype=BF16, device=x8.device)
    _call("vj_gemm_fp8", M, N, K, _p(x8), _rowmajor(x8, "x8"), _p(ex), _p(w8), _rowmajor(w8, "w8"), _p(ew), epi,
          _p(bias), _p(resid), resid.stride(0) if resid is not None else 0, _p(out),
          out.stride(0) if out is not None else 0, _p(out2), out2.stride(0) if out2 is not None else 0, _stream(),
          label=f"k_gemm_fp8<{EPI_NAMES[epi]}>", flops=2.0 * M * N * K)
    return (out, out2) if epi == EPI_GELU else out


def qkv_rope_fp8(x8, ex, w8, ew, bias, H, hd, ids, ids_mod, tpf, tpr, cos_tab, sin_tab):
    _dev(x8, w8, bias, ids, cos_tab, sin_tab)
    M, K = x8.shape
    N = 3 * H * hd
    assert w8.shape == (N, K) and x8.dtype == FP8 and w8.dtype == FP8
    out = torch.empty(M, N, dtype=BF16, device=x8.device)
    _call("vj_qkv_rope_gemm_fp8", M, K, _p(x8), _rowmajor(x8, "x8"), _p(ex), _p(w8), _rowmajor(w8, "w8"), _p(ew),
          _p(bias), _p(out), N, H, hd, _p(ids), int(ids_mod), int(tpf), int(tpr), _p(cos_tab), _p(sin_tab),
          cos_tab.shape[0], _stream(), label="k_gemm_fp8<EPI_ROPE>", flops=2.0 * M * N * K)
    return out


def rope_(qkv, H, hd, q_off, k_off, ids, ids_mod, tpf, tpr, cos_tab, sin_tab, inverse=False):
    _dev(qkv, ids, cos_tab, sin_tab)
    T = qkv.shape[0]
    if ids is not None:
        assert ids.dtype == torch.int32 and ids.numel() == T
    half = (hd // 3) // 2
    _call("vj_rope", T, H, hd, _p(qkv), _rowmajor(qkv, "qkv"), q_off, k_off, _p(ids), int(ids_mod), int(tpf), int(tpr),
         _p(cos_tab), _p(sin_tab), half, int(inverse), _stream())


def attn_fwd(qkv, H, hd, groups, scale, q_off=None, k_off=None, v_off=None, fblk=0, dropout_p=0.0, seed=0):
    """groups: list of (nseq, len). Returns (O bf16 [T, H*hd], stats f32 [2, H, T]). fblk > 0: frame-causal
    mask (token i sees key j iff j // fblk <= i // fblk). dropout_p > 0: SDPA's attention dropout with the
    mask of `seed` (vj_attn_fwd_ex; the backward needs the same p and seed)."""
    _dev(qkv)
    T = qkv.shape[0]
    D = H * hd
    q_off = 0 if q_off is None else q_off
    k_off = D if k_off is None else k_off
    v_off = 2 * D if v_off is None else v_off
    o = torch.empty(T, D, dtype=BF16, device=qkv.device)
    stats = torch.empty(2, H, T, dtype=F32, device=qkv.device)
    ns, ln = [g[0] for g in groups], [g[1] for g in groups]
    _call("vj_attn_fwd_ex", T, H, hd, _p(qkv), _rowmajor(qkv, "qkv"), q_off, k_off, v_off, _p(o), D, _p(stats),
          float(scale), len(groups), int_array(ns), int_array(ln), int(fblk), float(dropout_p), int(seed) & 0xFFFFFFFF,
          _stream(),
          label=f"attn_fwd<hd{hd}>", flops=sum(4.0 * n * l * l * D for n, l in groups))
    return o, stats


def attn_bwd(qkv, o, do, stats, H, hd, groups, scale, dqkv=None, rope=None, fblk=0, dropout_p=0.0, seed=0):
    """rope = (ids, ids_mod, tpf, tpr, cos_tab, sin_tab) -> dq, dk returned w.r.t. the un-rotated q, k.
    dropout_p, seed: those of the forward (attention dropout)."""
    _dev(qkv, o, do, stats)
    T = qkv.shape[0]
    D = H * hd
    dqkv = dqkv if dqkv is not None else torch.empty(T, 3 * D, dtype=BF16, device=qkv.device)
    ns, ln = [g[0] for g in groups], [g[1] for g in groups]
    ids, mod, tpf, tpr, ct, st = rope if rope is not None else (None, 0, 0, 0, None, None)
    _call("vj_attn_bwd_ex", T, H, hd, _p(qkv), _rowmajor(qkv, "qkv"), 0, D, 2 * D, _p(o), _rowmajor(o, "o"), _p(do),
          _rowmajor(do, "do"), _p(stats), _p(dqkv), _rowmajor(dqkv, "dqkv"), float(scale), len(groups), int_array(ns),
          int_array(ln), _p(ids), int(mod), int(tpf), int(tpr), _p(ct), _p(st), int(fblk), float(dropout_p),
          int(seed) & 0xFFFFFFFF, _stream(), label=f"attn_bwd<hd{hd}>",
          flops=sum(10.0 * n * l * l * D for n, l in groups))  # FA2 convention: 5 matmuls = 2.5 x forward
    return dqkv


def dropout(x, p, seed, resid=None, aux=None, out=None):
    """nn.Dropout's forward (or, on a gradient with the forward's seed, its backward) on a row-major
    [M, N] tensor (vj_dropout): bf16(bf16(x) * z), z = 1 / (1 - p) on kept elements. x f32 or bf16;
    resid (f32 / bf16): returns resid + that, in resid's dtype; aux (bf16): returns bf16(that * aux)."""
    _dev(x)
    M, N = x.shape
    if resid is not None:
        assert resid.shape == x.shape and resid.dtype in (F32, BF16)
        out = out if out is not None else torch.empty(M, N, dtype=resid.dtype, device=x.device)
    else:
        out = out if out is not None else torch.empty(M, N, dtype=BF16, device=x.device)
    if aux is not None:
        assert aux.shape == x.shape and aux.dtype == BF16
    _call("vj_dropout", M, N, _p(x), _rowmajor(x, "x"), int(x.dtype == F32), _p(aux),
          _rowmajor(aux, "aux") if aux is not None else 0, _p(resid), _rowmajor(resid, "resid") if resid is not None else 0,
          int(resid is not None and resid.dtype == F32), _p(out), _rowmajor(out, "out"), float(p), int(seed) & 0xFFFFFFFF,
          _stream(), label="vj_dropout")
    return out


def _xattn_ws(B, nq, N, H, hd, device):
    import ctypes

    n = ctypes.c_long(0)
    call("vj_xattn_ws_floats", B, nq, N, H, hd, ctypes.byref(n))
    return torch.empty(max(1, n.value), dtype=F32, device=device)


def xattn_fwd(q, kv, B, nq, N, H, hd, scale):
    """Cross-attention (CrossAttention.forward's SDPA, modules.py:585-587): q bf16 [B*nq, H*hd],
    kv bf16 [B*N, 2*H*hd] -> (O bf16 [B*nq, H*hd], lse2 f32 [B*H, nq])."""
    _dev(q, kv)
    assert q.dtype == BF16 and kv.dtype == BF16 and q.shape == (B * nq, H * hd) and kv.shape == (B * N, 2 * H * hd)
    o = torch.empty(B * nq, H * hd, dtype=BF16, device=q.device)
    lse2 = torch.empty(B * H, nq, dtype=F32, device=q.device)
    ws = _xattn_ws(B, nq, N, H, hd, q.device)
    _call("vj_xattn_fwd", B, nq, N, H, hd, _p(q), _rowmajor(q, "q"), _p(kv), _rowmajor(kv, "kv"), _p(o), H * hd,
          _p(lse2), float(scale), _p(ws), ws.numel(), _stream(), label="xattn_fwd", flops=4.0 * B * nq * N * H * hd)
    return o, lse2


def xattn_bwd(q, kv, o, do, lse2, B, nq, N, H, hd, scale):
    """Backward of xattn_fwd -> (dq bf16 [B*nq, H*hd], dkv bf16 [B*N, 2*H*hd])."""
    _dev(q, kv, o, do, lse2)
    assert do.dtype == BF16 and do.shape == o.shape
    dq = torch.empty(B * nq, H * hd, dtype=BF16, device=q.device)
    dkv = torch.empty(B * N, 2 * H * hd, dtype=BF16, device=q.device)
    ws = _xattn_ws(B, nq, N, H, hd, q.device)
    _call("vj_xattn_bwd", B, nq, N, H, hd, _p(q), _rowmajor(q, "q"), _p(kv), _rowmajor(kv, "kv"), _p(o),
          _rowmajor(o, "o"), _p(do), _rowmajor(do, "do"), _p(lse2), float(scale), _p(dq), H * hd, _p(dkv), 2 * H * hd,
          _p(ws), ws.numel(), _stream(), label="xattn_bwd", flops=10.0 * B * nq * N * H * hd)
    return dq, dkv


def qkv_rope(x, w, bias, H, hd, ids, ids_mod, tpf, tpr, cos_tab, sin_tab):
    """Fused QKV projection + RoPE of q, k: bf16 [M, 3*H*hd]."""
    _dev(x, w, bias, ids, cos_tab, sin_tab)
    M, K = x.shape
    N = 3 * H * hd
    assert w.shape == (N, K) and x.dtype == BF16 and w.dtype == BF16
    out = torch.empty(M, N, dtype=BF16, device=x.device)
    _call("vj_qkv_rope_gemm", M, K, _p(x), _rowmajor(x, "x"), _p(w), _rowmajor(w, "w"), _p(bias), _p(out), N, H, hd,
          _p(ids), int(ids_mod), int(tpf), int(tpr), _p(cos_tab), _p(sin_tab), cos_tab.shape[0], _stream(),
          label="k_gemm<1,1,EPI_ROPE>", flops=2.0 * M * N * K)
    return out


def im2col(clip, patch, tub, idx=None, out=None):
    """clip f32 [B,C,T,H,W] -> bf16 [R, C*tub*p*p]; idx int64 [B,K] kept tokens (or all tokens)."""
    _dev(clip, idx)
    assert clip.dtype == F32 and clip.is_contiguous()
    B, C, Tf, Hf, Wf = clip.shape
    N = (Tf // tub) * (Hf // patch) * (Wf // patch)
    if idx is not None:
        assert idx.dtype == torch.int64 and idx.is_contiguous() and idx.shape[0] == B
        assert int(idx.shape[1]) <= N
        K = idx.shape[1]
    else:
        K = N
    R = B * K
    kdim = C * tub * patch * patch
    if out is None:
        out = torch.empty(R, kdim, dtype=BF16, device=clip.device)
    assert out.shape == (R, kdim) and out.is_contiguous() and out.dtype == BF16
    _call("vj_im2col_tubelet", R, K, _p(idx), B, C, Tf, Hf, Wf, tub, patch, _p(clip), _p(out), _stream())
    return out


def ids_to_int32(mask_list):
    """Concatenate int64 [B, K_m] masks (row-major) into one int32 id vector (RoPE positions)."""
    n = sum(m.numel() for m in mask_list)
    out = torch.empty(n, dtype=torch.int32, device=mask_list[0].device)
    o = 0
    for m in mask_list:
        ids64to32(m.contiguous(), out=out[o:o + m.numel()])
        o += m.numel()
    return out


def gather_rows(src, idx, out=None, nrows=None):
    """out[r] = src[idx[r]] (bit-exact)."""
    _dev(src, idx)
    R = idx.numel()
    out = out if out is not None else torch.empty(R, src.shape[1], dtype=src.dtype, device=src.device)
    es = src.element_size()
    _call("vj_gather_rows", R, src.shape[1] * es, _p(src), _rowmajor(src, "src") * es, _p(idx), _p(out),
         _rowmajor(out, "out") * es, 0, _stream())
    return out


def scatter_rows(src, idx, out):
    """out[idx[r]] = src[r] (bit-exact)."""
    _dev(src, idx, out)
    R = idx.numel()
    es = src.element_size()
    _call("vj_gather_rows", R, src.shape[1] * es, _p(src), _rowmajor(src, "src") * es, _p(idx), _p(out),
         _rowmajor(out, "out") * es, 1, _stream())
    return out


def fill_rows(dst, idx, vec):
    _dev(dst, idx, vec)
    _call("vj_fill_rows", idx.numel(), dst.shape[1], _p(dst), _rowmajor(dst, "dst"), _p(idx), _p(vec), _stream())


def add_rows(dst, table, idx=None, idx_mod=0):
    _dev(dst, table, idx)
    _call("vj_add_rows", dst.shape[0], dst.shape[1], _p(dst), _rowmajor(dst, "dst"), _p(table),
         _rowmajor(table, "table"), table.shape[0], _p(idx), int(idx_mod), _stream())


def pred_index(mx, my, row0, N, pos, ctx_dst, tgt_rows, loss_rows=None):
    _dev(mx, my)
    B, K = mx.shape
    Kp = my.shape[1]
    assert mx.dtype == torch.int64 and my.dtype == torch.int64 and mx.is_contiguous() and my.is_contiguous()
    _call("vj_pred_index", B, K, Kp, _p(mx), _p(my), int(row0), B, int(N), _p(pos), _p(ctx_dst), _p(tgt_rows),
         _p(loss_rows), _stream())


def ids64to32(x, out=None):
    _dev(x)
    assert x.dtype == torch.int64 and x.is_contiguous()
    out = out if out is not None else torch.empty(x.numel(), dtype=torch.int32, device=x.device)
    _call("vj_ids64to32", x.numel(), _p(x), _p(out), _stream())
    return out


def jepa_loss(z, tgt, loss_rows, gamma, beta, group_rows, eps1=1e-6, eps2=1e-5, loss_exp=1.0, npairs=None):
    """Returns (loss f32 [1], dz bf16 [R, D], row_loss f32 [R]). z bf16 or f32 [R, D]; the loss is the
    mean over `npairs` (default len(group_rows)) of each mask group's mean |z - h|^p / p."""
    _dev(z, tgt, loss_rows)
    assert z.dtype in (F32, BF16) and tgt.dtype in (F32, BF16)
    R, D = z.shape
    npairs = len(group_rows) if npairs is None else npairs
    dz = torch.empty(R, D, dtype=BF16, device=z.device)
    row_loss = torch.empty(R, dtype=F32, device=z.device)
    loss = torch.empty(1, dtype=F32, device=z.device)
    _call("vj_jepa_loss", R, D, _p(z), int(z.dtype == BF16), _rowmajor(z, "z"), _p(tgt), int(tgt.dtype == BF16), _rowmajor(tgt, "tgt"),
         _p(loss_rows), _p(gamma), _p(beta), float(eps1), float(eps2), float(loss_exp), len(group_rows),
         int_array(group_rows), 1.0 / npairs, _p(dz), D, _p(row_loss), _p(loss), _stream())
    return loss, dz, row_loss


def check_finite(g, found_inf):
    _dev(g, found_inf)
    _call("vj_check_finite", g.numel(), _p(g), _p(found_inf), _stream())


def adamw(p, g, m, v, p_bf16, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0, found_inf=None):
    _dev(p, g, m, v, p_bf16, found_inf)
    _call("vj_adamw", p.numel(), _p(p), _p(g), _p(m), _p(v), _p(p_bf16), float(lr), float(beta1), float(beta2),
         float(eps), float(weight_decay), int(step), float(grad_scale), _p(found_inf), _stream())


def adamw_ema(p, g, m, v, p_bf16, lr, beta1, beta2, eps, weight_decay, step, target, target_bf16, momentum,
              grad_scale=1.0, found_inf=None):
    """adamw() followed by ema(target, p, momentum, target_bf16) in one pass over the arena slice."""
    _dev(p, g, m, v, p_bf16, found_inf, target, target_bf16)
    assert target.shape == p.shape and target.dtype == F32
    _call("vj_adamw_ema", p.numel(), _p(p), _p(g), _p(m), _p(v), _p(p_bf16), float(lr), float(beta1), float(beta2),
          float(eps), float(weight_decay), int(step), float(grad_scale), _p(found_inf), _p(target), _p(target_bf16),
          float(momentum), _stream(), label="vj_adamw")


def ema(target, online, momentum, target_bf16=None):
    _dev(target, online, target_bf16)
    _call("vj_ema", target.numel(), _p(target), _p(online), float(momentum), _p(target_bf16), _stream())


def gelu_eval(x):
    """(GELU(x), GELU'(x)) bf16 of bf16 x by the GEMM epilogues' exact evaluation (vj_gelu_eval)."""
    _dev(x)
    assert x.dtype == BF16 and x.is_contiguous()
    y, dy = torch.empty_like(x), torch.empty_like(x)
    _call("vj_gelu_eval", x.numel(), _p(x), _p(y), _p(dy), _stream())
    return y, dy


def cast_bf16(x, out=None):
    _dev(x)
    assert x.dtype == F32 and x.is_contiguous()
    out = out if out is not None else torch.empty(x.shape, dtype=BF16, device=x.device)
    _call("vj_cast_bf16", x.numel(), _p(x), _p(out), _stream())
    return out


def set_reserved_cus(n):
    """Persistent GEMM grids launched from now on leave n CUs free (vj_set_reserved_cus)."""
    call("vj_set_reserved_cus", int(n))


def proxy_copy(dst, src, blocks, mode=0):
    """Diagnostic: copy src into dst (same bytes) with `blocks` persistent workgroups (vj_proxy_copy;
    mode 1: non-temporal, 2: hold the CUs for the copy's time without moving bytes)."""
    _dev(dst, src)
    assert dst.is_contiguous() and src.is_contiguous() and dst.numel() * dst.element_size() == src.numel() * src.element_size()
    _call("vj_proxy_copy", _p(dst), _p(src), src.numel() * src.element_size(), blocks, mode, _stream())
    return dst


# ------------------------------------------------------------------------------------------------
# fp32-operand parity mode (vj_f32.hip): f32 operands throughout, off the training path.


def linear_fwd_f32(x, w, bias=None, epi=EPI_F32, resid=None):
    """Y = X W^T + b on the f32 MFMA; x f32 [M, K], w f32 [N, K]. EPI_GELU -> (pre, act)."""
    _dev(x, w, bias, resid)
    assert x.dtype == F32 and w.dtype == F32
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K
    y = torch.empty(M, N, dtype=F32, device=x.device)
    y2 = torch.empty(M, N, dtype=F32, device=x.device) if epi == EPI_GELU else None
    if epi == EPI_F32_RESID:
        assert resid is not None and resid.dtype == F32 and resid.shape == (M, N)
    _call("vj_gemm_f32", M, N, K, _p(x), _rowmajor(x, "x"), _p(w), _rowmajor(w, "w"), epi, _p(bias), _p(resid),
          resid.stride(0) if resid is not None else 0, _p(y), N, _p(y2), N if y2 is not None else 0, _stream(),
          label="k_gemm_f32", flops=2.0 * M * N * K)
    return (y, y2) if epi == EPI_GELU else y


def attn_fwd_f32(qkv, H, hd, groups, scale):
    """Exact-softmax attention on f32 qkv [T, 3*H*hd] -> (O f32 [T, H*hd], lse f32 [H, T] natural log)."""
    _dev(qkv)
    assert qkv.dtype == F32
    T = qkv.shape[0]
    D = H * hd
    o = torch.empty(T, D, dtype=F32, device=qkv.device)
    lse = torch.empty(H, T, dtype=F32, device=qkv.device)
    ns, ln = [g[0] for g in groups], [g[1] for g in groups]
    _call("vj_attn_fwd_f32", T, H, hd, _p(qkv), _rowmajor(qkv, "qkv"), 0, D, 2 * D, _p(o), D, _p(lse), float(scale),
          len(groups), int_array(ns), int_array(ln), _stream())
    return o, lse


def rope_f32_(qkv, H, hd, ids, ids_mod, tpf, tpr, cos_tab, sin_tab):
    """In-place 3-axis RoPE of the q and k columns of an f32 qkv buffer."""
    _dev(qkv, ids, cos_tab, sin_tab)
    assert qkv.dtype == F32
    T = qkv.shape[0]
    _call("vj_rope_f32", T, H, hd, _p(qkv), _rowmajor(qkv, "qkv"), 0, H * hd, _p(ids), int(ids_mod), int(tpf),
          int(tpr), _p(cos_tab), _p(sin_tab), (hd // 3) // 2, _stream())


def im2col_f32(clip, patch, tub, idx=None):
    """im2col with f32 rows: clip f32 [B,C,T,H,W] -> f32 [B*K, C*tub*p*p]."""
    _dev(clip, idx)
    assert clip.dtype == F32 and clip.is_contiguous()
    B, C, Tf, Hf, Wf = clip.shape
    N = (Tf // tub) * (Hf // patch) * (Wf // patch)
    K = idx.shape[1] if idx is not None else N
    if idx is not None:
        assert idx.dtype == torch.int64 and idx.is_contiguous() and idx.shape[0] == B and int(K) <= N
    out = torch.empty(B * K, C * tub * patch * patch, dtype=F32, device=clip.device)
    _call("vj_im2col_tubelet_f32", B * K, K, _p(idx), B, C, Tf, Hf, Wf, tub, patch, _p(clip), _p(out), _stream())
    return out


# ------------------------------------------------------------------------------------------------
# JEPA masks on the device (masks.MaskSpec.build)


def mask_count(B, duration, height, width, npred, boxes, t, h, w, max_ctx, counts):
    _dev(boxes, counts)
    assert boxes.dtype == torch.int32 and boxes.is_contiguous() and boxes.shape == (B, npred, 3)
    _call("vj_mask_count", B, duration, height, width, npred, _p(boxes), t, h, w, max_ctx, _p(counts), _stream())


def mask_emit(B, duration, height, width, npred, boxes, t, h, w, max_ctx, mode, k_enc, k_pred, enc, pred):
    _dev(boxes, enc, pred)
    assert enc.dtype == torch.int64 and pred.dtype == torch.int64 and enc.is_contiguous() and pred.is_contiguous()
    _call("vj_mask_emit", B, duration, height, width, npred, _p(boxes), t, h, w, max_ctx, mode, k_enc, k_pred,
          _p(enc), _p(pred), _stream())


def video_transform(frames, params, crop, mean, std, out):
    """uint8 frames [B, T, H, W, C] + per-clip (top, left, h, w, flip) int32 [B, 5] -> out f32 [B, C, T, S, S]."""
    _dev(frames, params, mean, std, out)
    assert frames.dtype == torch.uint8 and frames.is_contiguous() and frames.dim() == 5
    B, T, H, W, C = frames.shape
    assert params.dtype == torch.int32 and params.shape == (B, 5) and params.is_contiguous()
    assert out.shape == (B, C, T, crop, crop) and out.dtype == F32 and out.is_contiguous()
    p = params.cpu()
    assert bool(((p[:, 2] > 0) & (p[:, 3] > 0) & (p[:, 0] >= 0) & (p[:, 1] >= 0) & (p[:, 0] + p[:, 2] <= H)
                 & (p[:, 1] + p[:, 3] <= W)).all()), "crop boxes must lie inside the frames"
    _call("vj_video_transform", B, T, H, W, C, crop, _p(frames), _p(params), _p(mean), _p(std), _p(out), _stream())
