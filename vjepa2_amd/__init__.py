"""vjepa2_amd — MI355X-native (gfx950) V-JEPA 2 pre-training step.

Host side mirrors the reference's module API (VisionTransformer / VisionTransformerPredictor /
MaskCollator / app.vjepa train step); the hot path runs in libvjepa_hip.so (include/vjepa_hip.h).
"""

__version__ = "0.1.0"

import os as _os

# Hardware queues per process. The train step keeps three HIP streams busy at once (compute, target
# encoder, weight gradients) and a data-parallel run adds RCCL's own; with HIP's default of 4 queues
# the streams share queues once RCCL is initialised, and the step loses 3 % even at one rank
# (profiles/r05_hw_queues_ab.txt: 215.3 vs 221.2 clips/s; with 8 queues 221.0). Raised before the HIP
# runtime starts (it reads the variable once, at initialisation); a larger value is left alone.
_q = _os.environ.get("GPU_MAX_HW_QUEUES", "")
if not _q.isdigit() or int(_q) < 8:
    try:
        import torch as _torch

        if not _torch.cuda.is_initialized():
            _os.environ["GPU_MAX_HW_QUEUES"] = "8"
    except ImportError:  # pragma: no cover
        pass
