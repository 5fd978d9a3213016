"""vjepa2_amd — MI355X-native (gfx950) V-JEPA 2 pre-training step.

Host side mirrors the reference's module API (VisionTransformer / VisionTransformerPredictor /
MaskCollator / app.vjepa train step); the hot path runs in libvjepa_hip.so (include/vjepa_hip.h).
"""

__version__ = "0.1.0"

import os as _os
import warnings as _warnings

# Hardware queues per process. The train step keeps three HIP streams busy at once (compute, target
# encoder, weight gradients) and a data-parallel run adds RCCL's own; with HIP's default of 4 queues
# the streams share queues once RCCL is initialised, and the step loses 3 % even at one rank
# (profiles/r05_hw_queues_ab.txt: 215.3 vs 221.2 clips/s; with 8 queues 221.0). The HIP runtime reads
# the variable once, when it starts, so it is set here only while HIP is not up yet, and only when the
# caller has not chosen a value: unset, or HIP's own default 4 (which some environments export). Any
# other explicit GPU_MAX_HW_QUEUES is kept; VJ_HW_QUEUES=0 turns this off.
# The launchers (vjepa2_amd.main, bench.py's rank spawner) also put it into every rank's environment.
# A process whose HIP runtime is already up with fewer queues gets a warning (an error under
# VJ_STRICT=1): it runs correctly, ~3 % slower at world > 1.
HW_QUEUES = 8


def _hw_queues_note(msg):
    if _os.environ.get("VJ_STRICT", "0") == "1":
        raise RuntimeError(msg)
    _warnings.warn(msg, RuntimeWarning, stacklevel=3)


def _set_hw_queues():
    if _os.environ.get("VJ_HW_QUEUES", "1") == "0":
        return
    q = _os.environ.get("GPU_MAX_HW_QUEUES", "")
    try:
        import torch as _torch
    except ImportError:  # pragma: no cover
        return
    if q in ("", "4"):
        if not _torch.cuda.is_initialized():
            _os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)
        else:
            _hw_queues_note(f"vjepa2_amd imported after the HIP runtime started: it runs on "
                            f"{q or 'the default 4'} hardware queues, not {HW_QUEUES}; the train step's streams and RCCL's then share "
                            f"queues (~3 % slower at world > 1). Import vjepa2_amd (or set "
                            f"GPU_MAX_HW_QUEUES={HW_QUEUES}) before the first GPU call.")
    elif q.isdigit() and int(q) < HW_QUEUES:
        _hw_queues_note(f"GPU_MAX_HW_QUEUES={q} (explicit) is below the {HW_QUEUES} the train step's streams plus "
                        f"RCCL's need (~3 % slower at world > 1); kept as set.")


def rank_env(env):
    """The environment of a rank process about to be started (vjepa2_amd.main, bench.py --gpus N): the
    hardware-queue setting above applied to it, so it holds whatever the child imports first."""
    if env.get("VJ_HW_QUEUES", "1") != "0" and env.get("GPU_MAX_HW_QUEUES", "") in ("", "4"):
        env["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)
    return env


_set_hw_queues()
