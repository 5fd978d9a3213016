"""Summarise a rocprofv3 --kernel-trace run per train step.

    python tools/prof_summary.py <run_kernel_trace.csv | rocpd .db | --stats kernel CSV> <steps> <out.txt> [cmd]

With the kernel TRACE (timestamps), the per-step figures come from the steady state only: the window
from the second to the last k_jepa_loss launch (one per step, between a step's forward and its
backward) holds whole step cycles (backward + update of step k, forward of step k + 1), so the
first traced step's setup work (arena builds, weight loads: ~1300 runtime copy kernels, the init
fills) is not charged to the step. With only the --stats CSV or a rocpd .db,
totals are divided by `steps` (setup included), as before.
"""
import csv
import sqlite3
import sys

DEFAULT_CMD = "python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0"
STEP_MARK = "k_jepa_loss"


def _rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = ("select name, count(*), sum(duration), avg(duration) from kernels group by name "
             "order by sum(duration) desc")
        return [(n, int(k), float(t), float(a)) for n, k, t, a in c.execute(q)], None
    rows = list(csv.DictReader(open(path)))
    if rows and "Start_Timestamp" in rows[0]:  # kernel trace: steady-state window
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        marks = [int(r["Start_Timestamp"]) for r in rows if STEP_MARK in r["Kernel_Name"]]
        if len(marks) < 3:
            raise SystemExit(f"{path}: need >= 3 {STEP_MARK} launches for a steady-state window")
        t0, t1 = marks[1], marks[-1]
        agg = {}
        for r in rows:
            s = int(r["Start_Timestamp"])
            if t0 <= s < t1:
                d = agg.setdefault(r["Kernel_Name"], [0, 0.0])
                d[0] += 1
                d[1] += int(r["End_Timestamp"]) - s
        out = sorted(((n, k, t, t / k) for n, (k, t) in agg.items()), key=lambda x: -x[2])
        return out, len(marks) - 2
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"])) for r in rows], None


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = n[5:] if n.startswith("void ") else n
    return n.split("(")[0]


def main(path, steps, out, cmd=DEFAULT_CMD):
    rows, window = _rows(path)
    if window is not None:
        steps = window
        how = (f"steady state: {steps} step cycles between the 2nd and the last {STEP_MARK} launch "
               "(setup excluded); per step = window total / steps")
    else:
        how = f"{steps} traced train steps (warmup + timed); per step = total / {steps} (setup included)"
    lines = [f"# rocprofv3 --kernel-trace --stats -- {cmd}",
             f"# MI355X (gfx950), ViT-L/16 B=24 16x256^2; {how}",
             f"{'ms/step':>9} {'calls/step':>10} {'avg_us':>9}  kernel"]
    tot = 0.0
    for name, calls, total_ns, avg_ns in rows:
        tot += total_ns
        lines.append(f"{total_ns / steps / 1e6:9.3f} {calls / steps:10.1f} {avg_ns / 1e3:9.1f}  {short(name)}")
    lines.append(f"{tot / steps / 1e6:9.3f} {'':10} {'':9}  TOTAL GPU kernel time per step")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], *(sys.argv[4:5] or []))
