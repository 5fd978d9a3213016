"""Summarise a rocprofv3 --stats kernel CSV per train step: python tools/prof_summary.py <csv> <steps> <out.txt>."""
import csv
import sys


def main(path, steps, out, cmd="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0"):
    rows = list(csv.DictReader(open(path)))
    lines = [f"# rocprofv3 --kernel-trace --stats -- {cmd}",
             f"# MI355X (gfx950), ViT-L/16 B=24 16x256^2; {steps} traced train steps (warmup + timed); per step = total / {steps}",
             f"{'ms/step':>9} {'calls/step':>10} {'avg_us':>9}  kernel"]
    tot = 0.0
    for r in rows:
        t = float(r["TotalDurationNs"])
        tot += t
        n = r["Name"].replace("(anonymous namespace)::", "")
        n = n[5:] if n.startswith("void ") else n
        n = n.split("(")[0]
        lines.append(f"{t / steps / 1e6:9.3f} {int(r['Calls']) / steps:10.1f} {float(r['AverageNs']) / 1e3:9.1f}  {n}")
    lines.append(f"{tot / steps / 1e6:9.3f} {'':10} {'':9}  TOTAL GPU kernel time per step")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
