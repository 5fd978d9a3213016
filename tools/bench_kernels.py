"""A/B timing of GEMM / attention kernel builds in ONE process (interleaved rounds, median).

usage: python tools/bench_kernels.py [COL ...]   COL = lib.so | lib.so@ENV=V[,ENV2=V2] | @ENV=V
(default: vjepa2_amd/libvjepa_hip.so). Builds come from `python -m vjepa2_amd.build --variant NAME
-DMACRO=...`; an @ENV column times a build under host-side knobs (VJ_GEMM_GROUP, VJ_GEMM_PXCD), set
only while that column runs. Random operands (uniform [-1, 1) scaled), shapes of the ViT-L/16 B=24
train step.
"""
import contextlib
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vjepa2_amd._lib import SIGNATURES  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    lib = ctypes.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:  # an older build (A/B against a previous source tree)
            continue
        fn.argtypes = args
        fn.restype = ctypes.c_int
    return lib


# (name, M, N, K, a_kmajor, b_kmajor, epi, splitk); epi 7 = GELU with GELU' saved, 8 = bf16 residual
GEMMS = [
    ("square4096", 4096, 4096, 4096, 1, 1, 1, 1),
    ("qkv  ctx", 11712, 3072, 1024, 1, 1, 0, 1),
    ("proj ctx", 11712, 1024, 1024, 1, 1, 2, 1),
    ("fc1  ctx", 11712, 4096, 1024, 1, 1, 3, 1),
    ("fc2  ctx", 11712, 1024, 4096, 1, 1, 2, 1),
    ("fc1  tgt", 49152, 4096, 1024, 1, 1, 3, 1),
    ("fc1  ctx save", 11712, 4096, 1024, 1, 1, 7, 1),  # 7: GELU with the derivative saved (training path)
    ("qkv  tgt", 49152, 3072, 1024, 1, 1, 0, 1),
    ("proj tgt", 49152, 1024, 1024, 1, 1, 2, 1),
    ("proj tgt f32", 49152, 1024, 1024, 1, 1, 1, 1),
    ("proj tgt bf16", 49152, 1024, 1024, 1, 1, 0, 1),
    ("fc2  tgt", 49152, 1024, 4096, 1, 1, 2, 1),
    ("fc2  tgt bf16", 49152, 1024, 4096, 1, 1, 0, 1),
    ("proj tgt bres", 49152, 1024, 1024, 1, 1, 8, 1),  # 8: bf16 residual (the step's proj / fc2)
    ("fc2  tgt bres", 49152, 1024, 4096, 1, 1, 8, 1),
    ("proj ctx bres", 11712, 1024, 1024, 1, 1, 8, 1),
    ("fc2  ctx bres", 11712, 1024, 4096, 1, 1, 8, 1),
    ("dgrad fc2 Wt", 11712, 4096, 1024, 1, 1, 0, 1),
    ("dgrad fc2 GELU_BWD Wt", 11712, 4096, 1024, 1, 1, 4, 1),
    ("pred dgrad fc2 GELU_BWD Wt", 71232, 1536, 384, 1, 1, 4, 1),
    ("dgrad fc2", 11712, 4096, 1024, 1, 0, 0, 1),
    ("dgrad fc1", 11712, 1024, 4096, 1, 0, 0, 1),
    ("dgrad fc2 GELU_BWD", 11712, 4096, 1024, 1, 0, 4, 1),
    ("pred dgrad fc2 GELU_BWD", 71232, 1536, 384, 1, 0, 4, 1),
    ("wgrad fc1", 4096, 1024, 11712, 0, 0, 2, 4),
    ("wgrad qkv", 3072, 1024, 11712, 0, 0, 2, 5),
    ("wgrad proj", 1024, 1024, 11712, 0, 0, 2, 15),
    # 9: weight + bias gradient (vj_gemm_bf16_wgrad: the bias sums fused; a library without it runs
    # the split-K GEMM + vj_colsum_f32, the pre-fusion path)
    ("wgrad+b fc1", 4096, 1024, 11712, 0, 0, 9, 4),
    ("wgrad+b qkv", 3072, 1024, 11712, 0, 0, 9, 5),
    ("pred wgrad+b fc1", 1536, 384, 71232, 0, 0, 9, 14),
    ("pred wgrad+b qkv", 1152, 384, 71232, 0, 0, 9, 14),
    # ViT-g (D = 1408) weight gradients, K = 34304 context tokens: split 4 / 5 / 6 (the 128- and
    # 256-wide column-tile sizings pick different splits)
    ("g wgrad qkv s4", 4224, 1408, 34304, 0, 0, 2, 4),
    ("g wgrad qkv s5", 4224, 1408, 34304, 0, 0, 2, 5),
    ("g wgrad fc1 s6", 6144, 1408, 34304, 0, 0, 2, 6),
    ("g wgrad fc1 s5", 6144, 1408, 34304, 0, 0, 2, 5),
    ("g wgrad proj s7", 1408, 1408, 34304, 0, 0, 2, 7),
    ("pred qkv", 71232, 1152, 384, 1, 1, 0, 1),
    ("pred dgrad fc1", 71232, 384, 1536, 1, 0, 0, 1),
    ("pred wgrad fc1", 1536, 384, 71232, 0, 0, 2, 14),
    ("pred fc1", 71232, 1536, 384, 1, 1, 3, 1),
    ("pred fc1 save", 71232, 1536, 384, 1, 1, 7, 1),
    ("pred fc2", 71232, 384, 1536, 1, 1, 2, 1),
    ("pred proj", 71232, 384, 384, 1, 1, 2, 1),
    ("pred dgrad proj", 71232, 384, 384, 1, 1, 0, 1),
    ("pred dgrad qkv", 71232, 384, 1152, 1, 1, 0, 1),
]


ATTN = [("attn fwd hd64 ctx", 64, 16, [(24, 424), (24, 64)], False),
        ("attn fwd hd64 tgt", 64, 16, [(24, 2048)], False),
        ("attn bwd hd64 ctx", 64, 16, [(24, 424), (24, 64)], True),
        ("attn fwd hd32 pred", 32, 12, [(24, 1464), (24, 1504)], False),
        ("attn bwd hd32 pred", 32, 12, [(24, 1464), (24, 1504)], True),
        ("attn bwd hd64 ctx rope", 64, 16, [(24, 424), (24, 64)], "rope"),
        ("attn bwd hd32 pred rope", 32, 12, [(24, 1464), (24, 1504)], "rope"),
        ("attn fwd hd64 N2048", 64, 16, [(8, 2048)], False),
        ("attn bwd hd64 N2048", 64, 16, [(8, 2048)], True),
        ("attn bwd hd64 N4608", 64, 16, [(2, 4608)], True),
        ("attn bwd hd32 N4608", 32, 12, [(4, 4608)], True),
        ("attn fwd hd64 N8192", 64, 22, [(2, 8192)], False)]


def gemm_case(lib, case, dev, stream):
    name, M, N, K, akm, bkm, epi, sk = case
    rowsum = epi == 9
    epi = 2 if rowsum else epi
    save_d = epi == 7
    epi = 3 if save_d else (7 if epi == 8 else epi)  # 8: EPI_BF16_RESID (7 in the library)
    g = torch.Generator(device="cpu").manual_seed(0)
    A = ((torch.rand(M, K, generator=g) * 2 - 1) if akm else (torch.rand(K, M, generator=g) * 2 - 1)).to(dev).bfloat16()
    B = ((torch.rand(N, K, generator=g) * 2 - 1) if bkm else (torch.rand(K, N, generator=g) * 2 - 1)).to(dev).bfloat16()
    lda = K if akm else M
    ldb = K if bkm else N
    bias = torch.zeros(N, device=dev)
    if epi in (1, 2):
        C = torch.zeros(M, N, device=dev)
    else:
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    C2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if epi == 3 else None
    aux = C if epi in (2, 7) else ((torch.rand(M, N, generator=g) * 4 - 2).to(dev).bfloat16() if epi == 4 else None)
    ws = torch.empty(max(1, sk * M * N if sk > 1 else 1), device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    if rowsum:
        db = torch.zeros(M, device=dev)
        ws = torch.empty(max(sk * (M * N + M), 256 * M), device=dev)
        fused = hasattr(lib, "vj_gemm_bf16_wgrad")

        def run_rs():
            if fused:
                rc = lib.vj_gemm_bf16_wgrad(M, N, K, p(A), lda, p(B), ldb, p(C), N, 1, p(db), 1, sk, p(ws), ws.numel(),
                                            stream)
            else:
                rc = lib.vj_gemm_bf16_splitk(M, N, K, p(A), lda, akm, p(B), ldb, bkm, 2, None, p(C), N, p(C), N, None, 0,
                                             sk, p(ws), ws.numel(), stream)
                rc = rc or lib.vj_colsum_f32(K, M, p(A), 1, lda, p(db), 1, p(ws), ws.numel(), stream)
            assert rc == 0, rc
        return run_rs, 2.0 * M * N * K

    def run():
        rc = lib.vj_gemm_bf16_splitk(M, N, K, p(A), lda, akm, p(B), ldb, bkm, epi, p(bias), p(aux), N if aux is not None else 0,
                                     p(C) if epi != 3 or save_d else None, N if epi != 3 or save_d else 0, p(C2),
                                     N if C2 is not None else 0,
                                     sk, p(ws), ws.numel(), stream)
        assert rc == 0, rc
    return run, 2.0 * M * N * K


# (name, M, ids_mod): fused QKV + RoPE GEMM (vj_qkv_rope_gemm) at the ViT-L target / context sizes,
# 16 heads of 64, K = 1024; tokens by position (row % ids_mod: 8 frames x 16 x 16)
ROPE = [("qkv rope tgt", 49152, 2048), ("qkv rope ctx", 11712, 2048)]


def rope_case(lib, M, ids_mod, dev, stream):
    import math
    H, hd, K = 16, 64, 1024
    N = 3 * H * hd
    g = torch.Generator(device="cpu").manual_seed(1)
    x = ((torch.rand(M, K, generator=g) * 2 - 1)).to(dev).bfloat16()
    w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to(dev).bfloat16()
    b = torch.zeros(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    half = (hd // 3) // 2
    npos = 16
    pos = torch.arange(npos, dtype=torch.float64)[:, None]
    om = 1.0 / 10000 ** (torch.arange(half, dtype=torch.float64) / half)
    cos_t = torch.cos(pos * om).float().to(dev).contiguous()
    sin_t = torch.sin(pos * om).float().to(dev).contiguous()
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run():
        rc = lib.vj_qkv_rope_gemm(M, K, p(x), K, p(w), K, p(b), p(out), N, H, hd, None, ids_mod, 256, 16, p(cos_t),
                                  p(sin_t), npos, stream)
        assert rc == 0, rc
    return run, 2.0 * M * N * K


def attn_case(lib, hd, H, groups, dev, stream, bwd):
    T = sum(n * l for n, l in groups)
    D = H * hd
    qkv = (torch.randn(T, 3 * D, device=dev)).bfloat16()
    o = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(2, H, T, device=dev)
    do = torch.randn(T, D, device=dev).bfloat16()
    dqkv = torch.empty(T, 3 * D, device=dev, dtype=torch.bfloat16)
    ns = (ctypes.c_int * len(groups))(*[g[0] for g in groups])
    ln = (ctypes.c_int * len(groups))(*[g[1] for g in groups])
    sc = hd ** -0.5
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def fwd():
        assert lib.vj_attn_fwd(T, H, hd, P(qkv), 3 * D, 0, D, 2 * D, P(o), D, P(stats), sc, len(groups), ns, ln, stream) == 0
    fwd()

    # bwd == "rope": with the inverse 3-axis RoPE fused into the dq / dk stores (as the step runs it)
    half = (hd // 3) // 2
    tab = torch.rand(256 * half, device=dev) * 6.0
    cos_t, sin_t = tab.cos(), tab.sin()
    rope = (None, max(g[1] for g in groups), 64, 8, P(cos_t), P(sin_t)) if bwd == "rope" else (None, 0, 0, 0, None, None)

    def bwdf():
        assert lib.vj_attn_bwd(T, H, hd, P(qkv), 3 * D, 0, D, 2 * D, P(o), D, P(do), D, P(stats), P(dqkv), 3 * D,
                               sc, len(groups), ns, ln, *rope, stream) == 0
    bwdf.keep = (cos_t, sin_t)  # the tables stay allocated while the case runs
    fl = sum(4.0 * n * l * l * D for n, l in groups)
    return (bwdf, 2.5 * fl) if bwd else (fwd, fl)  # backward: FA2 convention, 5 matmuls


# (name, M, D, with dres_in): LayerNorm backward of the block's norm1 / norm2 (dres out f32 + bf16
# copy, dgamma / dbeta partials); the "TF" column is TB/s of algorithmic bytes for these
LNB = [("ln bwd ctx", 11712, 1024, True), ("ln bwd tgt-size", 49152, 1024, True), ("ln bwd pred", 71232, 384, True)]


def ln_bwd_case(lib, M, D, acc, dev, stream):
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, D, generator=g).to(dev)
    dy = torch.randn(M, D, generator=g).to(dev).bfloat16()
    mean = x.mean(1).contiguous()
    rstd = (x.var(1, unbiased=False) + 1e-6).rsqrt().contiguous()
    gamma = torch.rand(D, generator=g).to(dev)
    dres_in = torch.randn(M, D, generator=g).to(dev) if acc else None
    dres = torch.empty(M, D, device=dev)
    dres_bf = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    dgamma = torch.empty(D, device=dev)
    dbeta = torch.empty(D, device=dev)
    nb = lib.vj_layernorm_bwd_blocks(M)
    ws = torch.empty(nb * 2 * D, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    if rowsum:
        db = torch.zeros(M, device=dev)
        ws = torch.empty(max(sk * (M * N + M), 256 * M), device=dev)
        fused = hasattr(lib, "vj_gemm_bf16_wgrad")

        def run_rs():
            if fused:
                rc = lib.vj_gemm_bf16_wgrad(M, N, K, p(A), lda, p(B), ldb, p(C), N, 1, p(db), 1, sk, p(ws), ws.numel(),
                                            stream)
            else:
                rc = lib.vj_gemm_bf16_splitk(M, N, K, p(A), lda, akm, p(B), ldb, bkm, 2, None, p(C), N, p(C), N, None, 0,
                                             sk, p(ws), ws.numel(), stream)
                rc = rc or lib.vj_colsum_f32(K, M, p(A), 1, lda, p(db), 1, p(ws), ws.numel(), stream)
            assert rc == 0, rc
        return run_rs, 2.0 * M * N * K

    def run():
        rc = lib.vj_layernorm_bwd(M, D, p(dy), D, p(x), D, p(mean), p(rstd), p(gamma), p(dres_in), D, p(dres), D,
                                  p(dres_bf), D, p(dgamma), p(dbeta), None, None, p(ws), ws.numel(), stream)
        assert rc == 0, rc
    byt = M * D * (4 + 2 + 4 + 2 + (4 if acc else 0))
    return run, byt * 1e3


# (name, M, D, x bf16): LayerNorm forward of the block's norm1 / norm2 (bf16 out + mean / rstd); TB/s
LNF = [("ln fwd tgt bf16", 49152, 1024, True), ("ln fwd ctx f32", 15432, 1024, False),
       ("ln fwd pred f32", 73104, 384, False)]


def ln_fwd_case(lib, M, D, xbf, dev, stream):
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, D, generator=g).to(dev)
    if xbf:
        x = x.bfloat16()
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    gamma = torch.rand(D, generator=g).to(dev)
    beta = torch.rand(D, generator=g).to(dev)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run():
        rc = lib.vj_layernorm_fwd(M, D, p(x), int(xbf), D, p(gamma), p(beta), 1e-6, p(y), 0, D, p(mean), p(rstd), stream)
        assert rc == 0, rc
    return run, M * D * ((2 if xbf else 4) + 2) * 1e3


# (name, M, N): bias-gradient column sums of a bf16 [M, N] gradient (qkv / fc1 of the context and
# predictor blocks); TB/s of the bytes read
CSUM = [("colsum ctx fc1", 11712, 4096), ("colsum ctx qkv", 11712, 3072), ("colsum pred fc1", 71232, 1536)]


def colsum_case(lib, M, N, dev, stream):
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, N, generator=g).to(dev).bfloat16()
    out = torch.zeros(N, device=dev)
    ws = torch.empty(256 * N, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run():
        rc = lib.vj_colsum_f32(M, N, p(x), 1, N, p(out), 0, p(ws), ws.numel(), stream)
        assert rc == 0, rc
    return run, M * N * 2 * 1e3


def time_fn(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def parse_col(arg):
    path, _, env = arg.partition("@")
    envs = dict(kv.split("=", 1) for kv in env.split(",") if kv)
    return (path or os.path.join(HERE, "vjepa2_amd", "libvjepa_hip.so")), envs


@contextlib.contextmanager
def env_set(envs):
    old = {k: os.environ.get(k) for k in envs}
    os.environ.update(envs)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    cols = [parse_col(a) for a in sys.argv[1:]] or [parse_col("")]
    paths = [p for p, _ in cols]
    rounds = int(os.environ.get("VJ_BENCH_ROUNDS", "7"))
    dev = torch.device("cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    libs = [load(pth) for pth in paths]
    cases = []
    only = os.environ.get("VJ_BENCH_ONLY", "")
    kind = os.environ.get("VJ_BENCH_KIND", "")  # gemm | attn | ln: one family only
    for c in GEMMS:
        if (only and only not in c[0]) or kind not in ("", "gemm"):
            continue
        cases.append((c[0], [gemm_case(lib, c, dev, stream) for lib in libs]))
    for name, M, mod in ROPE:
        if (only and only not in name) or kind not in ("", "gemm", "rope"):
            continue
        cases.append((name, [rope_case(lib, M, mod, dev, stream) for lib in libs]))
    for name, hd, H, groups, bwd in ATTN:
        if (only and only not in name) or kind not in ("", "attn"):
            continue
        cases.append((name, [attn_case(lib, hd, H, groups, dev, stream, bwd) for lib in libs]))
    for name, M, D, xbf in LNF:
        if (only and only not in name) or kind not in ("", "ln"):
            continue
        cases.append((name, [ln_fwd_case(lib, M, D, xbf, dev, stream) for lib in libs]))
    for name, M, N in CSUM:
        if (only and only not in name) or kind not in ("", "ln", "mem"):
            continue
        cases.append((name, [colsum_case(lib, M, N, dev, stream) for lib in libs]))
    for name, M, D, acc in LNB:
        if (only and only not in name) or kind not in ("", "ln"):
            continue
        cases.append((name, [ln_bwd_case(lib, M, D, acc, dev, stream) for lib in libs]))
    names = [os.path.basename(p).replace("libvjepa_hip", "lib")[:14] + ("@" + ",".join(f"{k[7:] if k.startswith('VJ_GEMM_') else k}={v}" for k, v in e.items()) if e else "") for p, e in cols]
    print(f"{'case':22s} " + " ".join(f"{n[:26]:>26s}" for n in names), flush=True)
    for name, runs in cases:
        res = [[] for _ in libs]
        for _ in range(rounds):
            for i, (fn, fl) in enumerate(runs):
                with env_set(cols[i][1]):
                    res[i].append(time_fn(fn))
        out = []
        for i, (fn, fl) in enumerate(runs):
            ms = statistics.median(res[i])
            out.append(f"{ms * 1e3:9.1f}us {fl / ms / 1e9:7.1f}TF")
        print(f"{name:22s} " + " ".join(f"{c:>26s}" for c in out), flush=True)


if __name__ == "__main__":
    main()
