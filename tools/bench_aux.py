"""Timing of the §8f row 3 / row 4 kernels at eval / V-JEPA 2-AC shapes (HIP events, median of rounds).

    python tools/bench_aux.py            (prints one line per case; JSON with --json)

* cross-attention (vj_xattn_fwd / _bwd): the ViT-L probe (16 heads, hd 64) over 2 clips' tokens
  (N = 4096), nq = 1 (classifier) and 3 (action anticipation), B = 32; HBM-bound on the K/V read:
  algorithmic bytes = B·N·2D·2 (K and V) + small, reported as GB/s against 8 TB/s.
* frame-causal attention (vj_attn_fwd_fc / _bwd_fc): the AC predictor at 256² (16×16 patches + 2
  conditioning tokens per frame, fblk = 258), 8 frames after tubelets (L = 2064), 16 heads, hd 64,
  B = 8; MFMA-bound, algorithmic flops of the visible (block-lower-triangular) score blocks.
"""
import json
import statistics
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from vjepa2_amd import ops  # noqa: E402


def timed(fn, iters=10, rounds=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters)
    return statistics.median(res)


def main():
    dev = "cuda"
    out = []
    g = torch.Generator(device=dev).manual_seed(0)
    B, N, H, hd = 32, 4096, 16, 64
    D = H * hd
    kv = torch.randn(B * N, 2 * D, device=dev, generator=g).to(torch.bfloat16)
    for nq in (1, 3):
        q = torch.randn(B * nq, D, device=dev, generator=g).to(torch.bfloat16)
        do = torch.randn(B * nq, D, device=dev, generator=g).to(torch.bfloat16)
        o, lse = ops.xattn_fwd(q, kv, B, nq, N, H, hd, hd**-0.5)
        ms = timed(lambda: ops.xattn_fwd(q, kv, B, nq, N, H, hd, hd**-0.5))
        byt = B * N * 2 * D * 2
        out.append(dict(case=f"xattn fwd B{B} N{N} nq{nq} hd{hd}", us=round(ms * 1e3, 1),
                        GBps=round(byt / ms / 1e6, 1), frac_hbm=round(byt / ms / 1e6 / 8000.0, 3)))
        ms = timed(lambda: ops.xattn_bwd(q, kv, o, do, lse, B, nq, N, H, hd, hd**-0.5))
        byt = B * N * 2 * D * 2 * 2  # read K, V; write dK, dV
        out.append(dict(case=f"xattn bwd B{B} N{N} nq{nq} hd{hd}", us=round(ms * 1e3, 1),
                        GBps=round(byt / ms / 1e6, 1), frac_hbm=round(byt / ms / 1e6 / 8000.0, 3)))
    Bf, T, fblk = 8, 8, 258
    L = T * fblk
    qkv = torch.randn(Bf * L, 3 * D, device=dev, generator=g).to(torch.bfloat16)
    dout = torch.randn(Bf * L, D, device=dev, generator=g).to(torch.bfloat16)
    groups = [(Bf, L)]
    visible = sum((t + 1) * fblk * fblk for t in range(T))  # score entries per (sequence, head)
    fl = 4.0 * visible * D * Bf
    o, st = ops.attn_fwd(qkv, H, hd, groups, hd**-0.5, fblk=fblk)
    ms = timed(lambda: ops.attn_fwd(qkv, H, hd, groups, hd**-0.5, fblk=fblk))
    out.append(dict(case=f"frame-causal attn fwd B{Bf} L{L} fblk{fblk}", us=round(ms * 1e3, 1),
                    TFs=round(fl / ms / 1e9, 1), frac_mfma=round(fl / ms / 1e9 / 2500.0, 3)))
    ms = timed(lambda: ops.attn_bwd(qkv, o, dout, st, H, hd, groups, hd**-0.5, fblk=fblk))
    out.append(dict(case=f"frame-causal attn bwd B{Bf} L{L} fblk{fblk}", us=round(ms * 1e3, 1),
                    TFs=round(2.5 * fl / ms / 1e9, 1), frac_mfma=round(2.5 * fl / ms / 1e9 / 2500.0, 3)))
    ms = timed(lambda: ops.attn_fwd(qkv, H, hd, groups, hd**-0.5))
    out.append(dict(case=f"full attn fwd B{Bf} L{L} (same shape, no mask)", us=round(ms * 1e3, 1),
                    TFs=round(4.0 * L * L * D * Bf / ms / 1e9, 1)))
    if "--json" in sys.argv:
        print(json.dumps(out))
    else:
        for r in out:
            print(r)


if __name__ == "__main__":
    main()
