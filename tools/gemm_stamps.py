"""Diagnostic: per-tile s_memtime stamps of k_gemm256 (build variant 'stamps', -DVJ_GEMM_STAMPS=1):
main-loop and epilogue cycles per tile and how synchronised the CUs' epilogues are.
usage: python tools/gemm_stamps.py [case-substring]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_kernels as bk  # noqa: E402

lib = bk.load(os.environ.get("VJ_STAMPS_LIB") or os.path.join(bk.HERE, "vjepa2_amd", "libvjepa_hip_stamps.so"))
dev = torch.device("cuda")
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
only = sys.argv[1] if len(sys.argv) > 1 else "tgt"
for case in bk.GEMMS:
    if only not in case[0]:
        continue
    run, fl = bk.gemm_case(lib, case, dev, stream)
    run()
    torch.cuda.synchronize()
    lib.vj_debug_gemm_stamps_clear()
    run()
    torch.cuda.synchronize()
    buf = np.zeros(2048 * 16 * 4, dtype=np.int64)
    lib.vj_debug_gemm_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_long(buf.nbytes))
    st = buf.reshape(2048, 16, 4)
    valid = st[:, :, 0] != 0
    main = (st[:, :, 1] - st[:, :, 0])[valid]
    epi = (st[:, :, 2] - st[:, :, 1])[valid]
    t0 = st[:, :, 0][valid].min()
    end = st[:, :, 2][valid].max()
    ntile = valid.sum(1)
    k1 = st[:, :, 3][valid]
    if (k1 != 0).all():  # staggered builds: first 64-deep K step vs the rest of the main loop
        nks = case[3] // 64
        first = (k1 - st[:, :, 0][valid])
        rest = (st[:, :, 1][valid] - k1) / max(1, nks - 1)
        print(f"{case[0]:22s} first K step {np.median(first):8.0f} cyc (p90 {np.percentile(first, 90):.0f})  "
              f"later steps {np.median(rest):7.0f} cyc each", flush=True)
    print(f"{case[0]:22s} tiles/block {ntile[ntile > 0].min()}-{ntile.max()}  main {np.median(main):8.0f} cyc  "
          f"epi {np.median(epi):8.0f} cyc (p10 {np.percentile(epi, 10):.0f} p90 {np.percentile(epi, 90):.0f})  "
          f"span {end - t0} cyc", flush=True)
    # epilogue start spread across blocks for tile 0 and 1
    for it in range(2):
        e1 = st[:, it, 1][st[:, it, 1] != 0]
        if len(e1):
            print(f"   tile {it}: epilogue starts spread {np.percentile(e1, 90) - np.percentile(e1, 10):.0f} cyc")

    # S64 interval stamps (K steps 1-4 of each block's second tile; waves 0 and 4): cycles of each
    # interval between barriers, median over blocks
    if hasattr(lib, "vj_debug_gemm_istamps"):
        ib = np.zeros(2048 * 2 * 16, dtype=np.int64)
        lib.vj_debug_gemm_istamps(ctypes.c_void_p(ib.ctypes.data), ctypes.c_long(ib.nbytes))
        ib = ib.reshape(2048, 2, 16)
        ok = (ib[:, 0, :] != 0).all(1)
        if ok.any():
            d = np.diff(ib[ok][:, 0, :], axis=1)  # wave 0: intervals after barrier k -> k + 1
            print(f"   wave 0 intervals (M0, L1, M1, L0', ...) median cycles: {np.median(d, axis=0).astype(int).tolist()}")
            d4 = np.diff(ib[ok][:, 1, :], axis=1)
            print(f"   wave 4 intervals median cycles: {np.median(d4, axis=0).astype(int).tolist()}")
