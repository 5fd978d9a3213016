"""HBM traffic per launch of the bench's dominant kernel, from two rocprofv3 PMC passes over bench.py.

    python tools/traffic.py <fetch_pass_dir> <write_pass_dir> <label> <out.json> [workload]

`label` is bench.py's kernel label (e.g. "k_gemm<1,1,EPI_F32_RESID>"); it is matched against the
rocprofv3 kernel names (k_gemm256<true, true, 2, BN> for every tile width BN).
Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads (buffer_load ... lds, which is how
every GEMM operand arrives), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
The result is written for bench.py, which reports it as roofline.traffic (bytes per launch).
"""
import csv
import glob
import json
import os
import re
import sys

EPI = {"EPI_BF16": 0, "EPI_F32": 1, "EPI_F32_RESID": 2, "EPI_GELU": 3, "EPI_GELU_BWD": 4, "EPI_ROPE": 5,
       "EPI_PARTIAL": 6, "EPI_BF16_RESID": 7}


def name_regex(label):
    m = re.fullmatch(r"k_gemm<(\d),(\d),(\w+)>(\[splitk\])?", label)
    if m:
        b = {"1": "true", "0": "false"}
        epi = EPI["EPI_PARTIAL"] if m[4] else EPI[m[3]]  # split-K slices write f32 partial slabs
        # every tile width, the 8-wave, two-workgroups-per-CU (", false, 4"), 192-row and staggered
        # (trailing ", true") instantiations
        return re.compile(rf"k_gemm256<{b[m[1]]}, {b[m[2]]}, {epi}, \d+(, (?:true|false|\d+))*>")
    return re.compile(re.escape(label.split("<")[0]) + r"\b")


def per_launch(d, counter, rx):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and rx.search(r["Kernel_Name"]):
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fetch_dir, write_dir, label, out = sys.argv[1:5]
    workload = sys.argv[5] if len(sys.argv) > 5 else "vit_large 16x256^2 B=24"  # bench.py's default run
    rx = name_regex(label)
    fetch = per_launch(fetch_dir, "FETCH_SIZE", rx)
    write = per_launch(write_dir, "WRITE_SIZE", rx)
    assert fetch and write, f"no launches of {label} ({rx.pattern}) in the PMC passes"
    fkib = sum(fetch) / len(fetch)
    wkib = sum(write) / len(write)
    res = {"kernel": label, "workload": workload, "rocprof_regex": rx.pattern, "launches": [len(fetch), len(write)],
           "fetch_kib_per_launch": round(fkib, 1), "write_kib_per_launch": round(wkib, 1),
           "hbm_bytes_per_launch": round((2.0 * fkib + wkib) * 1024.0),
           "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (KiB units; gfx950 FETCH_SIZE "
                         "counts half of 16B/lane streaming reads)"}
    # profiles/traffic.json holds one entry per (kernel, workload): replace this one's, keep the others
    try:
        old = json.load(open(out))
        old = old if isinstance(old, list) else [old]
    except (OSError, ValueError):
        old = []
    keep = [e for e in old if (e.get("kernel"), e.get("workload")) != (label, workload)]
    json.dump(keep + [res], open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
