"""GPU: the video clip transform (vj_video_transform, vjepa2_amd.video.VideoTransform) against the
CPU restatement of app/vjepa/transforms.py:98-112 (oracle.video_transform: crop, F.interpolate
bilinear align_corners=False, flip, normalisation) on the same draws. The reference module itself
imports torchvision, which this image lacks, so the oracle restates it (parity is the same torch
interpolation call on the same crop box); tolerance: f32 interpolation order, 2e-5 in normalised
units."""

import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vjepa_oracle as orc  # noqa: E402

MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


@pytest.mark.parametrize("T,H,W,S", [(16, 256, 320, 256), (8, 360, 640, 224), (16, 128, 171, 256), (4, 64, 64, 64)])
def test_video_transform_matches_oracle(T, H, W, S):
    from vjepa2_amd.video import VideoTransform

    g = torch.Generator().manual_seed(T * H + W)
    frames = torch.randint(0, 256, (3, T, H, W, 3), generator=g, dtype=torch.uint8)
    vt = VideoTransform(crop_size=S)
    random.seed(5)
    np.random.seed(5)
    out = vt(frames).cpu()
    random.seed(5)
    np.random.seed(5)
    flips = 0
    for b in range(3):
        p = vt.draw(H, W)  # the same draws again, in the same order
        flips += p[4]
        exp = orc.video_transform(frames[b], p, S, MEAN, STD)
        err = (out[b] - exp).abs().max().item()
        assert err <= 2e-5, (b, p, err)
    assert out.shape == (3, 3, T, S, S)


def test_video_transform_flip_and_full_crop():
    """Forced boxes: the whole frame (identity resize: exact) and a flipped sub-box."""
    from vjepa2_amd import ops

    T, H, W, S = 2, 32, 32, 32
    frames = torch.randint(0, 256, (2, T, H, W, 3), generator=torch.Generator().manual_seed(3), dtype=torch.uint8)
    params = torch.tensor([[0, 0, H, W, 0], [3, 5, 20, 17, 1]], dtype=torch.int32)
    mean = torch.tensor(MEAN).cuda() * 255.0
    std = torch.tensor(STD).cuda() * 255.0
    out = torch.empty(2, 3, T, S, S, device="cuda")
    ops.video_transform(frames.cuda(), params.cuda(), S, mean, std, out)
    for b in range(2):
        exp = orc.video_transform(frames[b], params[b].tolist(), S, MEAN, STD)
        assert (out[b].cpu() - exp).abs().max().item() <= 2e-5
    ident = (frames[0].float().permute(3, 0, 1, 2) - mean.cpu()[:, None, None, None]) / std.cpu()[:, None, None, None]
    assert torch.equal(out[0].cpu(), ident)
