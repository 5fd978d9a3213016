"""CPU: the launcher (vjepa2_amd.main, drop-in for app/main.py:16-84) and bench.py's rank spawning,
up to the point where a rank would touch a GPU."""

import os
import subprocess
import sys

import pytest
import yaml

from launch_cfg import VITL_PRETRAIN_256_16F, micro
from vjepa2_amd import main as vmain

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CFG = "/root/reference/configs/train/vitl16/pretrain-256px-16f.yaml"


def test_parser_matches_reference_flags():
    a = vmain.make_parser().parse_args([])
    assert a.fname == "configs.yaml" and a.devices == [f"cuda:{i}" for i in range(8)] and a.debugmode is False
    a = vmain.make_parser().parse_args(["--fname", "x.yaml", "--devices", "cuda:2", "cuda:5", "--debugmode", "true"])
    assert a.devices == ["cuda:2", "cuda:5"] and a.debugmode is True
    assert [vmain.device_index(d) for d in a.devices] == [2, 5]
    with pytest.raises(ValueError):
        vmain.device_index("cpu")


@pytest.mark.skipif(not os.path.exists(REF_CFG), reason="reference tree not present (GPU box)")
def test_restated_config_equals_reference_yaml():
    """tests/launch_cfg.py restates the reference config's training keys (not the SLURM sizing or the
    dataset paths); pin every restated value against the file itself here."""
    ref = vmain.load_params(REF_CFG)
    for k, v in VITL_PRETRAIN_256_16F.items():
        if isinstance(v, dict):
            assert {kk: ref[k][kk] for kk in v} == v, k
        else:
            assert ref[k] == v, k


def test_load_params_and_app_dispatch(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text(yaml.dump(micro(tmp_path)))
    params = vmain.load_params(str(p))
    assert params["app"] == "vjepa" and params["data"]["batch_size"] == 2
    with pytest.raises(NotImplementedError):
        vmain.app_main("vjepa_droid", params)
    (tmp_path / "bad.yaml").write_text("a: 1\n")
    with pytest.raises(ValueError):
        vmain.load_params(str(tmp_path / "bad.yaml"))


def test_rccl_needs_one_device_per_rank():
    # this container has no HIP device: any RCCL launch is refused up front, gloo is not checked
    with pytest.raises(SystemExit, match="distinct devices"):
        vmain.check_devices(["cuda:0", "cuda:1"], "nccl")
    with pytest.raises(SystemExit, match="distinct devices"):
        vmain.check_devices(["cuda:0", "cuda:0"], "nccl")
    vmain.check_devices(["cuda:0", "cuda:0"], "gloo")


def test_bench_gpus_n_refuses_without_devices():
    """`bench.py --gpus 2` with RCCL and fewer devices than ranks exits non-zero with a message,
    before any rank starts (no silent single-rank run)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "VJ_DIST_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr
    assert "RCCL needs one device per rank" in r.stderr
