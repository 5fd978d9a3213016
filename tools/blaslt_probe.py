"""The library GEMM (torch.mm -> hipBLASLt on ROCm) against this repo's k_gemm256 on the train step's
plain shapes, in one process: is any of them worth handing to the library?

usage: python tools/blaslt_probe.py [lib.so]
"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import gemm_case, load, time_fn  # noqa: E402

# (name, M, N, K, a_kmajor, b_kmajor, epi, splitk) as tools/bench_kernels.GEMMS; epi 0 = bf16 out,
# 1 = f32 out (split-K for the weight gradients)
CASES = [
    ("qkv  tgt (bf16 out)", 49152, 3072, 1024, 1, 1, 0, 1),
    ("fc2  tgt (bf16 out)", 49152, 1024, 4096, 1, 1, 0, 1),
    ("proj tgt (bf16 out)", 49152, 1024, 1024, 1, 1, 0, 1),
    ("dgrad fc2 Wt", 11712, 4096, 1024, 1, 1, 0, 1),
    ("dgrad fc1", 11712, 1024, 4096, 1, 0, 0, 1),
    ("pred dgrad qkv", 71232, 384, 1152, 1, 1, 0, 1),
    ("wgrad fc1 (f32)", 4096, 1024, 11712, 0, 0, 1, 4),
    ("wgrad qkv (f32)", 3072, 1024, 11712, 0, 0, 1, 5),
    ("wgrad proj (f32)", 1024, 1024, 11712, 0, 0, 1, 15),
    ("pred wgrad fc1 (f32)", 1536, 384, 71232, 0, 0, 1, 14),
    ("square4096", 4096, 4096, 4096, 1, 1, 0, 1),
]


def torch_case(M, N, K, akm, bkm, f32out, dev):
    g = torch.Generator(device="cpu").manual_seed(0)
    A = ((torch.rand(M, K, generator=g) * 2 - 1) if akm else (torch.rand(K, M, generator=g) * 2 - 1)).to(dev).bfloat16()
    B = ((torch.rand(N, K, generator=g) * 2 - 1) if bkm else (torch.rand(K, N, generator=g) * 2 - 1)).to(dev).bfloat16()
    a = A if akm else A.t()  # [M, K]
    b = B.t() if bkm else B  # [K, N]
    out = torch.empty(M, N, device=dev, dtype=torch.float32 if f32out else torch.bfloat16)

    def run():
        if f32out:
            torch.mm(a, b, out_dtype=torch.float32, out=out)
        else:
            torch.mm(a, b, out=out)
    return run


# residual GEMMs: out(bf16) = resid(bf16) + A W^T + bias; ours EPI_BF16_RESID (7), the library's
# addmm(resid, A, W^T) (beta = 1; its bias would be one more epilogue term)
RESID = [("fc2  tgt + resid", 49152, 1024, 4096), ("proj tgt + resid", 49152, 1024, 1024),
         ("fc2  ctx + resid", 11712, 1024, 4096), ("proj ctx + resid", 11712, 1024, 1024)]


def resid_cases(lib, M, N, K, dev, stream):
    g = torch.Generator(device="cpu").manual_seed(0)
    A = (torch.rand(M, K, generator=g) * 2 - 1).to(dev).bfloat16()
    W = (torch.rand(N, K, generator=g) * 2 - 1).to(dev).bfloat16()
    R = (torch.rand(M, N, generator=g) * 2 - 1).to(dev).bfloat16()
    bias = torch.zeros(N, device=dev)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731

    def ours():
        assert lib.vj_gemm_bf16_splitk(M, N, K, p(A), K, 1, p(W), K, 1, 7, p(bias), p(R), N, p(C), N, None, 0, 1,
                                       None, 0, stream) == 0

    def lt():
        torch.addmm(R, A, W.t(), out=C)
    return ours, lt, 2.0 * M * N * K


def _pair(name, ours, lt, fl, rounds=5):
    to, tl = [], []
    for _ in range(rounds):  # interleaved, median: the clock drifts with the load (DVFS)
        to.append(time_fn(ours))
        tl.append(time_fn(lt))
    t_o, t_l = statistics.median(to), statistics.median(tl)
    print(f"{name:28s} {t_o * 1e3:8.1f}us {fl / t_o / 1e9:7.1f}TF   {t_l * 1e3:8.1f}us {fl / t_l / 1e9:7.1f}TF",
          flush=True)


def main():
    lib = load(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "vjepa2_amd",
                                                                   "libvjepa_hip.so"))
    dev = torch.device("cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    print(f"{'case':28s} {'k_gemm256':>20s} {'torch.mm (hipBLASLt)':>24s}")
    for c in CASES:
        name, M, N, K, akm, bkm, epi, sk = c
        ours, fl = gemm_case(lib, (name, M, N, K, akm, bkm, epi, sk), dev, stream)
        _pair(name, ours, torch_case(M, N, K, akm, bkm, epi == 1, dev), fl)
    for name, M, N, K in RESID:
        _pair(name, *resid_cases(lib, M, N, K, dev, stream))


if __name__ == "__main__":
    main()
