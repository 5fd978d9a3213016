"""Summarise a rocprofv3 --kernel-trace run per train step.

    python tools/prof_summary.py <rocpd .db or --stats kernel CSV> <steps> <out.txt> [cmd]

ROCm 7.2's rocprofv3 writes a rocpd SQLite database by default (`<dir>/<name>_results.db`);
older runs wrote `*_kernel_stats.csv`. Both are read here (sqlite3 / csv from the stdlib).
"""
import csv
import sqlite3
import sys

DEFAULT_CMD = "python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0"


def _rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = ("select name, count(*), sum(duration), avg(duration) from kernels group by name "
             "order by sum(duration) desc")
        return [(n, int(k), float(t), float(a)) for n, k, t, a in c.execute(q)]
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]))
            for r in csv.DictReader(open(path))]


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = n[5:] if n.startswith("void ") else n
    return n.split("(")[0]


def main(path, steps, out, cmd=DEFAULT_CMD):
    lines = [f"# rocprofv3 --kernel-trace --stats -- {cmd}",
             f"# MI355X (gfx950), ViT-L/16 B=24 16x256^2; {steps} traced train steps (warmup + timed); "
             f"per step = total / {steps}",
             f"{'ms/step':>9} {'calls/step':>10} {'avg_us':>9}  kernel"]
    tot = 0.0
    for name, calls, total_ns, avg_ns in _rows(path):
        tot += total_ns
        lines.append(f"{total_ns / steps / 1e6:9.3f} {calls / steps:10.1f} {avg_ns / 1e3:9.1f}  {short(name)}")
    lines.append(f"{tot / steps / 1e6:9.3f} {'':10} {'':9}  TOTAL GPU kernel time per step")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], *(sys.argv[4:5] or []))
