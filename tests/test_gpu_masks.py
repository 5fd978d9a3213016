"""GPU: JEPA masks built on the device (vj_mask_count / vj_mask_emit, masks.MaskSpec.build) from the
collate's RNG draws are bit-identical to the reference's masks: against the golden masks the
reference itself generated (tests/golden/masks.pt) and against the host collate over many draws
of the ViT-L / ViT-g configs (src/masks/multiseq_multiblock3d.py:16-239)."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from test_host_logic import VITL, gold  # noqa: E402

DEV = "cuda"


def _collate(mc, B, fpc):
    from vjepa2_amd.masks import materialize

    entry, = mc([(torch.zeros(1), 0, [torch.arange(fpc)]) for _ in range(B)])
    _, e, p = materialize(entry, DEV)
    return e, p


@pytest.mark.parametrize("tag", ["vitl", "small"])
def test_device_masks_match_golden(tag):
    from vjepa2_amd.masks import MaskCollator

    g = gold("masks.pt")[tag]
    torch.manual_seed(239)
    mc = MaskCollator(VITL, [g["fpc"]], crop_size=g["crop"], patch_size=16, tubelet_size=2, device_masks=True)
    for it in g["iters"]:
        e, p = _collate(mc, g["B"], g["fpc"])
        for a, b in zip(e + p, it["enc"] + it["pred"]):
            assert a.is_cuda and a.dtype == torch.int64 and torch.equal(a.cpu(), b)


def test_device_mask_options_match_golden():
    from vjepa2_amd.masks import MaskCollator

    for name, ex in gold("masks.pt")["extras"].items():
        torch.manual_seed(5)
        mc = MaskCollator([ex["cfg"]], [8], crop_size=64, patch_size=16, tubelet_size=2, device_masks=True)
        e, p = _collate(mc, 3, 8)
        assert torch.equal(e[0].cpu(), ex["enc"][0]) and torch.equal(p[0].cpu(), ex["pred"][0]), name


@pytest.mark.parametrize("fpc,crop,B,extra", [(16, 256, 24, {}), (16, 384, 8, {}), (64, 256, 6, {}),
                                              (16, 256, 24, dict(max_temporal_keep=0.5, temporal_scale=[0.5, 1.0])),
                                              (16, 256, 5, dict(full_complement=True)),
                                              (16, 256, 5, dict(pred_full_complement=True, max_keep=300))])
def test_device_masks_match_host_collate(fpc, crop, B, extra):
    """Same seed, same draws: host collate (pinned to the reference's fixtures) vs the device build,
    10 collates per config (N = 2048 / 4608 / 8192 tokens)."""
    from vjepa2_amd.masks import MaskCollator

    cfgs = [dict(c, **extra) for c in VITL]
    host = MaskCollator(cfgs, [fpc], crop_size=crop, patch_size=16, tubelet_size=2)
    dev = MaskCollator(cfgs, [fpc], crop_size=crop, patch_size=16, tubelet_size=2, device_masks=True)
    for i in range(10):
        torch.manual_seed(1000 + i)
        (_, he, hp), = host([(torch.zeros(1), 0, [torch.arange(fpc)]) for _ in range(B)])
        after_host = torch.rand(1)
        torch.manual_seed(1000 + i)
        de, dp = _collate(dev, B, fpc)
        assert torch.equal(torch.rand(1), after_host), "the draws consumed a different RNG stream"
        for a, b in zip(he + hp, de + dp):
            assert torch.equal(a, b.cpu())
