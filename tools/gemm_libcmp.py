"""Bitwise comparison of two GEMM builds (a change of LDS layout or schedule must not change a bit): every
tools/bench_kernels.GEMMS case (and the RoPE QKV GEMM) run through both libraries on the same operands.

usage: python tools/gemm_libcmp.py libA.so libB.so
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import GEMMS, load  # noqa: E402


def run(lib, case, dev, stream):
    name, M, N, K, akm, bkm, epi, sk = case
    save_d = epi == 7
    epi = 3 if save_d else (7 if epi == 8 else epi)  # 8: EPI_BF16_RESID (7 in the library)
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = ((torch.rand(M, K, generator=g) * 2 - 1) if akm else (torch.rand(K, M, generator=g) * 2 - 1)).to(dev).bfloat16()
    B = ((torch.rand(N, K, generator=g) * 2 - 1) if bkm else (torch.rand(K, N, generator=g) * 2 - 1)).to(dev).bfloat16()
    bias = (torch.rand(N, generator=g) - 0.5).to(dev)
    f32 = epi in (1, 2)
    C = (torch.rand(M, N, generator=g) - 0.5).to(dev) if f32 else torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    C2 = torch.zeros(M, N, device=dev, dtype=torch.bfloat16) if epi == 3 else None
    if epi == 7:
        C = (torch.rand(M, N, generator=g) * 4 - 2).to(dev).bfloat16()
    aux = C if epi in (2, 7) else ((torch.rand(M, N, generator=g) * 4 - 2).to(dev).bfloat16() if epi == 4 else None)
    ws = torch.empty(max(1, sk * M * N if sk > 1 else 1), device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    rc = lib.vj_gemm_bf16_splitk(M, N, K, p(A), K if akm else M, akm, p(B), K if bkm else N, bkm, epi, p(bias), p(aux),
                                 N if aux is not None else 0, p(C) if epi != 3 or save_d else None,
                                 N if epi != 3 or save_d else 0, p(C2), N if C2 is not None else 0, sk, p(ws),
                                 ws.numel(), stream)
    assert rc == 0, rc
    torch.cuda.synchronize()
    return [t for t in (C, C2) if t is not None]


def main(a, b):
    la, lb = load(a), load(b)
    dev = torch.device("cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    bad = 0
    for case in GEMMS:
        x, y = run(la, case, dev, stream), run(lb, case, dev, stream)
        same = all(torch.equal(u, v) for u, v in zip(x, y))
        bad += not same
        print(f"{case[0]:28s} equal={same}", flush=True)
    print("ALL EQUAL" if not bad else f"{bad} MISMATCHES")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
