"""Bitwise comparison of two attention builds (e.g. a restructured epilogue that must not change a bit):
O, lse and dQKV (with and without the fused inverse RoPE) on the step's shapes.

usage: python tools/attn_libcmp.py libA.so libB.so
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import load  # noqa: E402

CASES = [(64, 16, [(24, 424), (24, 64)]), (64, 4, [(3, 2048)]), (32, 12, [(4, 1464), (4, 1504)]),
         (64, 2, [(3, 70), (2, 130)]), (32, 3, [(2, 257), (1, 5)]), (80, 2, [(2, 150), (1, 33)]),
         (88, 2, [(1, 200), (3, 31)])]


def run(lib, hd, H, groups, rope, seed):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(seed)
    T = sum(n * l for n, l in groups)
    D = H * hd
    qkv = torch.randn(T, 3 * D, generator=g).to(dev).bfloat16()
    do = torch.randn(T, D, generator=g).to(dev).bfloat16()
    half = (hd // 3) // 2
    ang = torch.rand(256 * max(half, 1), generator=g).to(dev) * 6.0
    cos_t, sin_t = ang.cos().contiguous(), ang.sin().contiguous()
    o = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(2, H, T, device=dev)
    dqkv = torch.zeros(T, 3 * D, device=dev, dtype=torch.bfloat16)
    ns = (ctypes.c_int * len(groups))(*[x[0] for x in groups])
    ln = (ctypes.c_int * len(groups))(*[x[1] for x in groups])
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    sc = hd ** -0.5
    assert lib.vj_attn_fwd(T, H, hd, P(qkv), 3 * D, 0, D, 2 * D, P(o), D, P(stats), sc, len(groups), ns, ln, None) == 0
    lse = stats[0].clone()
    mod = max(x[1] for x in groups)
    r = (None, mod, 64, 8, P(cos_t), P(sin_t)) if rope else (None, 0, 0, 0, None, None)
    assert lib.vj_attn_bwd(T, H, hd, P(qkv), 3 * D, 0, D, 2 * D, P(o), D, P(do), D, P(stats), P(dqkv), 3 * D, sc,
                           len(groups), ns, ln, *r, None) == 0
    torch.cuda.synchronize()
    return o, lse, dqkv


def main(a, b):
    la, lb = load(a), load(b)
    bad = 0
    for hd, H, groups in CASES:
        for rope in (False, True):
            x = run(la, hd, H, groups, rope, hd + H)
            y = run(lb, hd, H, groups, rope, hd + H)
            same = [torch.equal(p, q) for p, q in zip(x, y)]
            bad += not all(same)
            print(f"hd={hd} H={H} groups={groups} rope={rope}: o/lse/dqkv equal {same}", flush=True)
    print("ALL EQUAL" if not bad else f"{bad} MISMATCHES")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
