"""Library GEMM reference points on the box: torch.matmul (hipBLASLt on ROCm) for the ViT-L step's
GEMM shapes, bf16 in / bf16 out, no epilogue. Calibration only (what a tuned library reaches on a
plain GEMM of the same shape); the product path uses its own fused kernels.

    python tools/blaslt_probe.py
"""
import torch

SHAPES = [  # (name, M, N, K, a_transposed, b_transposed): C[M,N] = A[M,K] B[K,N]
    ("square 4096", 4096, 4096, 4096, False, True),
    ("fc1 tgt  X W^T", 49152, 4096, 1024, False, True),
    ("qkv tgt  X W^T", 49152, 3072, 1024, False, True),
    ("fc2 tgt  X W^T", 49152, 1024, 4096, False, True),
    ("fc1 ctx  X W^T", 11712, 4096, 1024, False, True),
    ("wgrad fc1 dY^T X", 4096, 1024, 11712, True, False),
    ("wgrad qkv dY^T X", 3072, 1024, 11712, True, False),
    ("pred wgrad fc1", 1536, 384, 71232, True, False),
    ("pred fc1 X W^T", 71232, 1536, 384, False, True),
    ("wgrad fc2 dY^T X", 1024, 4096, 11712, True, False),
    ("wgrad proj dY^T X", 1024, 1024, 11712, True, False),
    ("pred wgrad qkv", 1152, 384, 71232, True, False),
]


def main():
    dev = torch.device("cuda")
    print(f"{'shape':22s} {'us':>9s} {'TF/s':>8s}")
    for name, M, N, K, at, bt in SHAPES:
        a = (torch.randn(K, M, device=dev).bfloat16().t() if at else torch.randn(M, K, device=dev).bfloat16())
        b = (torch.randn(N, K, device=dev).bfloat16().t() if bt else torch.randn(K, N, device=dev).bfloat16())
        for _ in range(3):
            torch.matmul(a, b)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        s.record()
        for _ in range(n):
            torch.matmul(a, b)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / n
        print(f"{name:22s} {ms * 1e3:9.1f} {2.0 * M * N * K / ms / 1e9:8.1f}", flush=True)


if __name__ == "__main__":
    main()
