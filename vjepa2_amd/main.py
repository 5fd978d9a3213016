"""Local multi-GPU launcher: drop-in for app/main.py:35-84 + app/scaffold.py:14-17.

    python -m vjepa2_amd.main --fname configs/train/vitl16/pretrain-256px-16f.yaml --devices cuda:0 ... cuda:7

One OS process per `--devices` entry (the reference's `mp.Process(process_main)` per device,
main.py:76-84). Each rank:
  * binds its GPU (the device index of its `--devices` entry) BEFORE the process group, so RCCL
    builds its communicator on that device (the reference does the same with CUDA_VISIBLE_DEVICES,
    main.py:38; here every rank keeps the whole node visible, like torchrun, and RCCL reaches its
    peers over xGMI);
  * loads the YAML (main.py:54-55); rank 0 prints it and writes `params-pretrain.yaml` into
    `folder` (main.py:59-66);
  * `init_distributed(rank_and_world_size=(rank, world))` (main.py:69; "nccl" = RCCL);
  * dispatches on `app:` (scaffold.py:17): `vjepa` -> vjepa2_amd.train.main(args).

The parent process imports nothing that touches the GPU (no HIP call before the children start),
waits for every rank, and exits with the first non-zero child exit code; if one rank fails the
others are terminated (by their own PIDs) instead of hanging in a collective.

Differences from the reference, all deliberate:
  * `--debugmode` runs rank 0 in this process (same as the reference) ;
  * a failed init_process_group with world > 1 raises (vjepa2_amd/distributed.py), where the
    reference silently falls back to one process;
  * `VJ_DIST_BACKEND=gloo` lets several ranks share one device (rehearsal on a 1-GPU box; RCCL
    refuses two ranks on one device). With "nccl" every rank needs its own device, checked up front.
"""

import argparse
import logging
import os
import pprint
import socket
import sys

import yaml

logger = logging.getLogger("vjepa2_amd.main")

APPS = {"vjepa": "vjepa2_amd.train"}


def make_parser():
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--fname", type=str, default="configs.yaml", help="name of config file to load")
    p.add_argument("--devices", type=str, nargs="+",
                   default=[f"cuda:{i}" for i in range(8)], help="which devices to use on local machine")
    p.add_argument("--debugmode", type=lambda s: str(s).lower() in ("1", "true", "yes"), default=False,
                   help="run rank 0 in this process (no spawn)")
    return p


def device_index(dev):
    """'cuda:3' -> 3 (main.py:38 takes the text after ':')."""
    tail = str(dev).split(":")[-1]
    if not tail.isdigit():
        raise ValueError(f"device {dev!r}: expected cuda:<index>")
    return int(tail)


def load_params(fname):
    # yaml.safe_load: the configs are plain mappings (the reference uses FullLoader; no tags are used)
    with open(fname, "r") as f:
        params = yaml.safe_load(f)
    if not isinstance(params, dict) or "app" not in params:
        raise ValueError(f"{fname}: not a V-JEPA config (no 'app' key)")
    return params


def app_main(app, args, resume_preempt=False):
    """app/scaffold.py:14-17."""
    import importlib

    if app not in APPS:
        raise NotImplementedError(f"app {app!r}: this build implements {sorted(APPS)}")
    logger.info("Running pre-training of app: %s", app)
    return importlib.import_module(APPS[app]).main(args=args, resume_preempt=resume_preempt)


def process_main(rank, fname, world_size, devices):
    """main.py:35-73, one rank."""
    logging.basicConfig(stream=sys.stdout, level=logging.INFO if rank == 0 else logging.ERROR,
                        format="[%(levelname)-8s][%(asctime)s][%(name)s] %(message)s", force=True)
    os.environ["LOCAL_RANK"] = str(device_index(devices[rank]))
    logger.info("called-params %s", fname)
    params = load_params(fname)
    if rank == 0:
        pprint.PrettyPrinter(indent=4).pprint(params)
        folder = params.get("folder", ".")
        os.makedirs(folder, exist_ok=True)
        with open(os.path.join(folder, "params-pretrain.yaml"), "w") as f:
            yaml.dump(params, f)

    import torch

    from .distributed import init_distributed

    torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
    world_size, rank = init_distributed(rank_and_world_size=(rank, world_size))
    logger.info("Running... (rank: %d/%d)", rank, world_size)
    return app_main(params["app"], args=params)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def check_devices(devices, backend):
    """With RCCL every rank needs a distinct, existing device. torch.cuda.device_count() does not
    initialise HIP on this image, so the parent stays GPU-free."""
    import torch

    idx = [device_index(d) for d in devices]
    if backend != "nccl":
        return
    n = torch.cuda.device_count()
    bad = [i for i in idx if i >= n]
    if bad or len(set(idx)) != len(idx):
        raise SystemExit(f"vjepa2_amd.main: {len(idx)} RCCL ranks need {len(idx)} distinct devices; "
                         f"--devices {' '.join(devices)} but this node has {n} visible HIP device(s). "
                         "Use fewer --devices, or VJ_DIST_BACKEND=gloo to rehearse on one device.")


def launch(fname, devices):
    """Start one spawned process per device (main.py:76-84) and wait for all of them."""
    import multiprocessing as mp

    world = len(devices)
    check_devices(devices, os.environ.get("VJ_DIST_BACKEND", "nccl"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    from . import rank_env

    rank_env(os.environ)  # the spawned ranks inherit it: 8 hardware queues before their first HIP call
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=process_main, args=(r, fname, world, devices), name=f"rank{r}") for r in range(world)]
    for p in procs:
        p.start()
    code = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            p.join(timeout=1.0)
            if p.exitcode is None:
                continue
            alive.remove(p)
            if p.exitcode != 0 and code == 0:
                code = p.exitcode if p.exitcode > 0 else 1
                logger.error("%s exited with %s: terminating the other ranks", p.name, p.exitcode)
                for q in alive:
                    q.terminate()
    return code


def main(argv=None):
    args = make_parser().parse_args(argv)
    logging.basicConfig(stream=sys.stdout, level=logging.INFO)
    if args.debugmode:
        process_main(rank=0, fname=args.fname, world_size=1, devices=[args.devices[0]])
        return 0
    return launch(args.fname, args.devices)


if __name__ == "__main__":
    sys.exit(main())
