"""Run ONE kernel case of tools/bench_kernels.py a fixed number of times (for rocprofv3 --pmc passes).

    python tools/kernel_one.py "<case name>" [iters] [lib.so]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_kernels as bk  # noqa: E402


def main():
    name = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(bk.HERE, "vjepa2_amd", "libvjepa_hip.so")
    lib = bk.load(path)
    dev = torch.device("cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    fn = None
    for c in bk.GEMMS:
        if c[0] == name:
            fn, fl = bk.gemm_case(lib, c, dev, stream)
    for n, hd, H, groups, bwd in bk.ATTN:
        if n == name:
            fn, fl = bk.attn_case(lib, hd, H, groups, dev, stream, bwd)
    assert fn is not None, f"unknown case {name!r}"
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {iters} launches, {fl / 1e9:.1f} GFLOP each")


if __name__ == "__main__":
    main()
