"""Load a checkpoint WRITTEN BY THIS BUILD into the REFERENCE's own app.vjepa.utils.load_checkpoint
(app/vjepa/utils.py:90-135) with the reference's models, DDP wraps (train.py:279-281) and AdamW param
groups (utils.py:207-239). Runs only in the build container (the reference is not on the GPU box):

    python tests/golden/check_reference_load.py <latest.pt written by the build>

The checkpoint comes from tests/test_gpu_app.py::test_checkpoint_loads_into_reference_layout run on
the GPU box with VJ_CKPT_OUT=<path> (micro encoder/predictor of make_golden.gen_resume). The
reference is imported read-only with the stubs of make_golden.py; nothing is written into it.
"""

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (stubs + reference import path)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import app.vjepa.utils as rutils  # noqa: E402
from src.utils.wrappers import MultiSeqWrapper, PredictorMultiSeqWrapper  # noqa: E402


def main(path):
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("gloo", rank=0, world_size=1)

    def vit_micro(**kw):
        return mg.vit.VisionTransformer(img_size=64, patch_size=16, num_frames=8, tubelet_size=2, embed_dim=64,
                                        depth=2, num_heads=1, mlp_ratio=4, qkv_bias=True, use_rope=True,
                                        uniform_power=True, norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6))

    enc = MultiSeqWrapper(vit_micro())
    pred = PredictorMultiSeqWrapper(mg.vpred.vit_predictor(img_size=64, use_mask_tokens=True, patch_size=16,
                                                           num_frames=8, tubelet_size=2, embed_dim=64,
                                                           predictor_embed_dim=64, depth=2, num_heads=2,
                                                           uniform_power=True, num_mask_tokens=2, use_rope=True))
    tgt = MultiSeqWrapper(vit_micro())
    opt, scaler, _, _ = rutils.init_opt(enc, pred, iterations_per_epoch=3, start_lr=1e-4, ref_lr=5e-4, warmup=1,
                                        num_epochs=1)
    DDP = torch.nn.parallel.DistributedDataParallel
    enc, pred, tgt = DDP(enc, static_graph=True), DDP(pred, find_unused_parameters=True), DDP(tgt)
    enc, pred, tgt, opt, scaler, epoch = rutils.load_checkpoint(path, enc, pred, tgt, opt, scaler)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    for k, v in enc.state_dict().items():
        assert torch.equal(v, ck["encoder"][k]), k
    n_state = sum(1 for st in opt.state.values() if st)
    assert n_state == len(ck["opt"]["state"]) and n_state > 0
    for g in opt.param_groups:
        for p in g["params"]:
            st = opt.state.get(p)
            if st:
                assert st["exp_avg"].shape == p.shape
    print(f"reference load_checkpoint OK: epoch {epoch}, {len(ck['encoder'])} encoder / {len(ck['predictor'])} "
          f"predictor tensors, {n_state} AdamW states on the reference's parameters")


if __name__ == "__main__":
    main(sys.argv[1])
