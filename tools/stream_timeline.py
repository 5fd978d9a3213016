"""Per-stream timeline of one steady-state train step from a rocprofv3 kernel trace taken with the side
streams ON (the bench's real configuration): for each phase of the step (forward up to the loss,
backward + update after it) the busy time of every queue, the time with 0 / 1 / 2+ kernels in flight,
and the kernels that run with nothing else in flight (where one stream alone holds the chip).

    python tools/stream_timeline.py <run_kernel_trace.csv> [out.txt]
"""
import csv
import re
import sys

STEP_MARK = "k_jepa_loss"


def _short(name):
    name = re.sub(r"^void\s+", "", name)
    return re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0][:70]


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if STEP_MARK in r["Kernel_Name"]]
    if len(marks) < 3:
        raise SystemExit("need >= 3 steps in the trace")
    t0, t1 = marks[-3], marks[-2]  # loss(k) .. loss(k+1): backward + update of step k, forward of k+1
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows
          if t0 <= int(r["Start_Timestamp"]) < t1]
    # the forward of step k+1 starts at its first patch-embedding GEMM after the update's last AdamW
    adam = [e for s, e, q, n in ks if "k_adamw" in n]
    tf = max(adam) if adam else t0
    lines = [f"# {path}: one step cycle, loss(k) -> loss(k+1), {(t1 - t0) / 1e6:.2f} ms"]
    for name, a, b in (("backward + update", t0, tf), ("forward", tf, t1)):
        ev = []
        per_q = {}
        for s, e, q, n in ks:
            s, e = max(s, a), min(e, b)
            if e <= s:
                continue
            ev += [(s, 1), (e, -1)]
            per_q[q] = per_q.get(q, 0) + (e - s)
        ev.sort()
        hist = {0: 0, 1: 0, 2: 0}
        cur, last = 0, a
        for t, d in ev:
            hist[min(cur, 2)] += t - last
            cur += d
            last = t
        hist[0] += b - last
        tot = b - a
        lines.append(f"{name}: {tot / 1e6:.2f} ms; idle {hist[0] / 1e6:.2f} ms, one kernel {hist[1] / 1e6:.2f} ms, "
                     f"2+ kernels {hist[2] / 1e6:.2f} ms")
        for q, t in sorted(per_q.items(), key=lambda x: -x[1]):
            lines.append(f"   queue {q}: kernels busy {t / 1e6:.2f} ms")
    # kernels that run with nothing else in flight (the step's exposed critical path), whole cycle
    ev = []
    for i, (s, e, q, n) in enumerate(ks):
        ev += [(s, 1, i), (e, -1, i)]
    ev.sort()
    active, last, alone = set(), t0, {}
    for t, d, i in ev:
        if len(active) == 1:
            k = _short(ks[next(iter(active))][3])
            alone[k] = alone.get(k, 0) + (t - last)
        last = t
        if d == 1:
            active.add(i)
        else:
            active.discard(i)
    lines.append(f"kernels alone in flight: {sum(alone.values()) / 1e6:.2f} ms; largest:")
    for k, v in sorted(alone.items(), key=lambda x: -x[1])[:12]:
        lines.append(f"   {v / 1e6:6.2f} ms  {k}")
    txt = "\n".join(lines)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))
