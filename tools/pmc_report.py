"""Per-kernel summary of the rocprofv3 PMC passes of tools/pmc_bench.sh.

MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of the
             dispatch's SIMD-cycles the matrix pipes were busy (GRBM_GUI_ACTIVE is summed over the 8
             XCDs; SQ_VALU_MFMA_BUSY_CYCLES counts MFMA cycles, 32 per 32x32x16 / 16 per 16x16x32 bf16).
clock      = GRBM_GUI_ACTIVE / 8 / dispatch duration (MI355X_MICROARCH.md, DVFS give-back).
HBM bytes  = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; gfx950 FETCH_SIZE counts half of 16-B/lane
             streaming reads, MI355X_MICROARCH.md HBM section). Durations are those of the profiled
             (serialised) dispatches of the MFMA pass.
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("_GLOBAL__N_1::", "")
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:  # drop the parameter list (the first top-level parenthesis)
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:70]


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            did = r["Dispatch_Id"]
            if did not in seen:
                seen.add(did)
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return per, durs


def main(root):
    p1, d1 = load(os.path.join(root, "p1"))
    p2, _ = load(os.path.join(root, "p2"))
    p3, _ = load(os.path.join(root, "p3"))
    rows = []
    for k, cs in p1.items():
        n = len(d1[k])
        t = sum(d1[k])
        grbm = cs.get("GRBM_GUI_ACTIVE", 0.0)
        busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        mf = busy / (1024 * grbm / 8) if grbm else 0.0
        clk = grbm / 8 / t / 1e9 if t else 0.0
        fetch = 2 * p2.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 / n
        write = p3.get(k, {}).get("WRITE_SIZE", 0.0) * 1024 / n
        rows.append((t, k, n, t / n * 1e6, mf, clk, fetch, write, (fetch + write) / (t / n) / 1e9 if t else 0.0))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"{'kernel':70s} {'launch':>6s} {'avg_us':>8s} {'%time':>6s} {'MFMA%':>6s} {'GHz':>5s} "
          f"{'fetch_MB':>9s} {'write_MB':>9s} {'HBM_GB/s':>9s}")
    for t, k, n, avg, mf, clk, fe, wr, bw in rows[:30]:
        print(f"{k:70s} {n:6d} {avg:8.1f} {100 * t / tot:6.1f} {100 * mf:6.1f} {clk:5.2f} {fe / 1e6:9.1f} "
              f"{wr / 1e6:9.1f} {bw:9.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
