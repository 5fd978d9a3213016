"""GPU: the launcher (vjepa2_amd.main = app/main.py:35-84) and `bench.py --gpus N` run end to end.

* `python -m vjepa2_amd.main --fname <ViT-L pretrain yaml> --devices cuda:0` — the reference
  config (tests/launch_cfg.py restates configs/train/vitl16/pretrain-256px-16f.yaml) with batch,
  crop, frames and ipe shrunk to a micro size — trains 2 steps through a spawned rank process and
  writes its log, params-pretrain.yaml and latest.pt;
* the same with two ranks sharing the box's one GPU over gloo (RCCL needs one device per rank):
  both ranks run, their losses are logged per rank;
* with RCCL and more ranks than devices, both entry points exit non-zero with a clear message;
* `VJ_DIST_BACKEND=gloo python bench.py --gpus 2` starts two ranks itself and reports n_gpus 2,
  dp2 and a per-GPU value.
"""

import csv
import json
import os
import subprocess
import sys

import pytest
import yaml

from launch_cfg import micro

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT",
                                                           "VJ_DIST_BACKEND")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.update(kw)
    return env


def _run(cmd, env, timeout=240):
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    return r


def _rows(path):
    with open(path) as f:
        return list(csv.reader(f))


def test_main_single_rank_vitl_config(tmp_path):
    cfg = tmp_path / "vitl.yaml"
    cfg.write_text(yaml.dump(micro(tmp_path / "out")))
    r = _run([sys.executable, "-m", "vjepa2_amd.main", "--fname", str(cfg), "--devices", "cuda:0"], _env())
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = tmp_path / "out"
    rows = _rows(out / "log_r0.csv")
    assert len(rows) == 2, rows
    losses = [float(x[2]) for x in rows]
    assert all(0.0 < l < 10.0 for l in losses), losses
    assert (out / "params-pretrain.yaml").exists() and (out / "latest.pt").exists()
    print("losses", losses)


def test_main_two_ranks_gloo_one_device(tmp_path):
    cfg = tmp_path / "vitl.yaml"
    cfg.write_text(yaml.dump(micro(tmp_path / "out")))
    r = _run([sys.executable, "-m", "vjepa2_amd.main", "--fname", str(cfg), "--devices", "cuda:0", "cuda:0"],
             _env(VJ_DIST_BACKEND="gloo"), timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for rank in range(2):
        rows = _rows(tmp_path / "out" / f"log_r{rank}.csv")
        assert len(rows) == 2, (rank, rows)


def test_rccl_with_too_few_devices_fails_loudly(tmp_path):
    cfg = tmp_path / "vitl.yaml"
    cfg.write_text(yaml.dump(micro(tmp_path / "out")))
    import torch

    n = torch.cuda.device_count()
    devs = [f"cuda:{i}" for i in range(n + 1)]
    r = _run([sys.executable, "-m", "vjepa2_amd.main", "--fname", str(cfg), "--devices"] + devs, _env())
    assert r.returncode != 0 and "distinct devices" in (r.stdout + r.stderr)
    r = _run([sys.executable, "bench.py", "--gpus", str(n + 1), "--steps", "1"], _env())
    assert r.returncode != 0 and "RCCL needs one device per rank" in r.stderr


def test_bench_gpus2_spawns_two_ranks():
    r = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "2",
              "--crop", "64", "--frames", "8", "--model", "vit_small", "--cpu-baseline", "0", "--kernel-events", "0"],
             _env(VJ_DIST_BACKEND="gloo"), timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["dist_backend"] == "gloo"
    assert abs(out["clips_per_s_per_gpu"] * 2 - out["value"]) < 1e-2 * out["value"]
    assert out["ms_per_step_median"] > 0
    # the exposed all-reduce time (backward end -> GradReducer.finish() end, median, max over ranks)
    # and every rank's process-group report
    assert out["allreduce_exposed_ms"] >= 0
    assert out["synced_comparison"]["ms_per_step"] > 0
    for rk in (0, 1):
        assert f"[bench rank {rk}/2] backend=gloo" in r.stderr, r.stderr[-2000:]
    print(lines[0][:400])


def test_bench_one_gpu_armed_reducer_over_rccl():
    """`bench.py --arm-reducer 1` at one GPU: the bucketed gradient all-reduce armed over a one-rank
    RCCL ("nccl") process group, the collective path of a DP run on one device."""
    r = _run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--batch", "2", "--crop", "64", "--frames",
              "8", "--model", "vit_small", "--cpu-baseline", "0", "--kernel-events", "0", "--arm-reducer", "1"],
             _env(), timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["reducer_armed"] is True and out["dist_backend"] == "nccl"
    assert out["allreduce_exposed_ms"] > 0 and 0.0 < out["loss_last"] < 10.0
    assert "[bench rank 0/1] backend=nccl" in r.stderr, r.stderr[-2000:]
