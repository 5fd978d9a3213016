"""Per-step GPU occupancy from a rocprofv3 kernel trace of bench.py (side streams on):

    rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 \
        --cpu-baseline 0 --kernel-events 0 --synced-steps 0
    python tools/step_trace.py <dir>/run_kernel_trace.csv

Steps are delimited by the last AdamW launch of each update (k_adamw: one per arena slice of each
stage of the staged update). Per step: wall time, union of kernel intervals (GPU busy), idle time,
the sum of kernel durations and their ratio to the union (kernels in flight on average), and the busy
time of each queue (HIP stream) on its own. profiles/r04_step_trace_busy.txt was made with this."""
import csv
import sys


def union(intervals):
    busy, cur_s, cur_e = 0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return busy + (cur_e - cur_s if cur_e is not None else 0)


def main(path):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"])
                for r in csv.DictReader(open(path)))
    adam = [e for e in ev if "k_adamw" in e[2]]
    # an update is a run of AdamW launches with no other kernel of its queue between them
    ends, last = [], None
    for s, e, _, q in adam:
        if last is not None and any(last < x[0] < s and x[3] == q and "k_adamw" not in x[2] and "k_check" not in x[2]
                                    for x in ev if last < x[0] < s):
            ends.append(last)
        last = e
    if last is not None:
        ends.append(last)
    for a, b in zip(ends[:-1], ends[1:]):
        seg = [(max(s, a), min(e, b), q) for s, e, _, q in ev if e > a and s < b]
        busy = union([(s, e) for s, e, _ in seg])
        tot = sum(e - s for s, e, _ in seg)
        per_q = {q: union([(s, e) for s, e, qq in seg if qq == q]) for q in sorted({q for _, _, q in seg})}
        qs = "  ".join(f"queue {q} {t / 1e6:.1f} ms" for q, t in per_q.items())
        print(f"step wall {(b - a) / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(b - a - busy) / 1e6:.2f} ms  "
              f"sum {tot / 1e6:.2f} ms  in flight {tot / max(busy, 1):.2f}  |  {qs}")


if __name__ == "__main__":
    main(sys.argv[1])
