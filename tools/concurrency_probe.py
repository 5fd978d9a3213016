"""Do two kernels of the step gain from running at once? One process: each kernel alone, then the pair
issued back to back on ONE stream (serial) and on TWO streams (concurrent), N_REP launches each,
timed with HIP events; prints T_alone, T_serial, T_concurrent and the concurrent / serial ratio
(1.0 = zero-sum, < 1 = the pair overlaps). Shapes: bench_kernels' ViT-L/16 B=24 cases.

usage: python tools/concurrency_probe.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_kernels as bk  # noqa: E402

N_REP = 6


def main():
    dev = torch.device("cuda:0")
    lib = bk.load(os.path.join(bk.HERE, "vjepa2_amd", "libvjepa_hip.so"))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    h1, h2 = s1.cuda_stream, s2.cuda_stream

    def attn(hd, H, groups, bwd, st):
        return bk.attn_case(lib, hd, H, groups, dev, st, bwd)[0]

    def gemm(name, st):
        c = next(c for c in bk.GEMMS if c[0] == name)
        return bk.gemm_case(lib, c, dev, st)[0]

    pred = [(24, 1464), (24, 1504)]
    kernels = {
        "attn bwd hd32 pred": lambda st: attn(32, 12, pred, True, st),
        "attn fwd hd32 pred": lambda st: attn(32, 12, pred, False, st),
        "attn fwd hd64 tgt": lambda st: attn(64, 16, [(24, 2048)], False, st),
        "fc2 tgt bres": lambda st: gemm("fc2  tgt bres", st),
        "fc1 tgt": lambda st: gemm("fc1  tgt", st),
        "wgrad fc1": lambda st: gemm("wgrad fc1", st),
    }
    pairs = [("attn bwd hd32 pred", "fc2 tgt bres"), ("attn bwd hd32 pred", "wgrad fc1"),
             ("attn fwd hd32 pred", "fc1 tgt"), ("attn fwd hd64 tgt", "fc2 tgt bres"),
             ("fc1 tgt", "fc2 tgt bres"), ("attn bwd hd32 pred", "attn fwd hd32 pred")]

    def timed(fn, reps=5):
        out = []
        for _ in range(reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) * 1e3)
        return statistics.median(out)

    print(f"{'pair':48s} {'T_a':>9s} {'T_b':>9s} {'serial':>9s} {'concur':>9s} {'c/s':>6s}  (us per pair, {N_REP} reps)")
    for a, b in pairs:
        ka1, kb1 = kernels[a](h1), kernels[b](h1)
        ka2 = kernels[a](h1)
        kb2 = kernels[b](h2)
        for f in (ka1, kb1, ka2, kb2):
            f()  # warm

        def bracket(body):
            def f():
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                s2.wait_stream(cur)
                body()
                cur.wait_stream(s1)
                cur.wait_stream(s2)
            return f

        def rep(*fns):
            def body():
                for _ in range(N_REP):
                    for fn in fns:
                        fn()
            return body

        alone_a, alone_b = bracket(rep(ka1)), bracket(rep(kb1))
        serial, concur = bracket(rep(ka1, kb1)), bracket(rep(ka2, kb2))

        ta, tb, ts, tc = (timed(f) / N_REP for f in (alone_a, alone_b, serial, concur))
        print(f"{a + ' || ' + b:48s} {ta:9.1f} {tb:9.1f} {ts:9.1f} {tc:9.1f} {tc / ts:6.3f}", flush=True)


if __name__ == "__main__":
    main()
