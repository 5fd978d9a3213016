"""Video clip transform on the GPU: app/vjepa/transforms.py:37-116 (VideoTransform, make_transforms)
for the training configuration the V-JEPA 2 configs use (no auto-augment, no motion shift, no
random erasing).

The host makes the reference's random draws in the reference's order (they define the stream):
the crop box of src/datasets/utils/video/transforms.py:470-507 (_get_param_spatial_crop: python
`random` for scale / log-ratio / offsets, plus one numpy draw per attempt for the switch_hw test,
which the reference evaluates before checking the flag) and the flip of :149-180 (numpy). The
device does the rest in one pass (vj_video_transform): crop, bilinear resize
(F.interpolate(align_corners=False), :537-542), horizontal flip and the (x - 255 mean) / (255 std)
normalisation (transforms.py:139-152), from uint8 frames to the f32 [C, T, S, S] clip the step
consumes, so the decoded video crosses PCIe as bytes.
"""

import math
import random

import numpy as np
import torch

from . import ops


def make_transforms(random_horizontal_flip=True, random_resize_aspect_ratio=(3 / 4, 4 / 3),
                    random_resize_scale=(0.3, 1.0), reprob=0.0, auto_augment=False, motion_shift=False, crop_size=224,
                    normalize=((0.485, 0.456, 0.406), (0.229, 0.224, 0.225))):
    """app/vjepa/transforms.py:13-34."""
    return VideoTransform(random_horizontal_flip=random_horizontal_flip,
                          random_resize_aspect_ratio=random_resize_aspect_ratio,
                          random_resize_scale=random_resize_scale, reprob=reprob, auto_augment=auto_augment,
                          motion_shift=motion_shift, crop_size=crop_size, normalize=normalize)


def crop_params(scale, ratio, height, width, num_repeat=10, log_scale=True, switch_hw=False):
    """video/transforms.py:470-507, the same draws in the same order."""
    for _ in range(num_repeat):
        area = height * width
        target_area = random.uniform(*scale) * area
        if log_scale:
            log_ratio = (math.log(ratio[0]), math.log(ratio[1]))
            aspect_ratio = math.exp(random.uniform(*log_ratio))
        else:
            aspect_ratio = random.uniform(*ratio)
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if np.random.uniform() < 0.5 and switch_hw:
            w, h = h, w
        if 0 < w <= width and 0 < h <= height:
            i = random.randint(0, height - h)
            j = random.randint(0, width - w)
            return i, j, h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


class VideoTransform:
    """transforms.py:37-116. __call__(buffer uint8 [T, H, W, C] or [B, T, H, W, C], host or device)
    -> f32 [C, T, S, S] (or [B, C, T, S, S]) on the device."""

    def __init__(self, random_horizontal_flip=True, random_resize_aspect_ratio=(3 / 4, 4 / 3),
                 random_resize_scale=(0.3, 1.0), reprob=0.0, auto_augment=False, motion_shift=False, crop_size=224,
                 normalize=((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)), device="cuda"):
        if auto_augment or motion_shift or reprob > 0:
            raise NotImplementedError("GPU VideoTransform: auto_augment, motion_shift and random erasing are not "
                                      "implemented (the V-JEPA 2 pre-training configs use none of them)")
        self.random_horizontal_flip = random_horizontal_flip
        self.scale = tuple(random_resize_scale)
        self.ratio = tuple(random_resize_aspect_ratio)
        self.crop_size = int(crop_size)
        self.device = torch.device(device)
        # the reference scales mean / std by 255 (uint8 space) when auto-augment is off
        self.mean = (torch.tensor(normalize[0], dtype=torch.float32) * 255.0).to(self.device)
        self.std = (torch.tensor(normalize[1], dtype=torch.float32) * 255.0).to(self.device)

    def draw(self, height, width):
        """One clip's draws: (top, left, height, width, flip)."""
        i, j, h, w = crop_params(self.scale, self.ratio, height, width)
        flip = bool(self.random_horizontal_flip and np.random.uniform() < 0.5)
        return i, j, h, w, int(flip)

    def __call__(self, buffer):
        frames = torch.as_tensor(buffer)
        single = frames.dim() == 4
        if single:
            frames = frames[None]
        if frames.dtype != torch.uint8:
            raise TypeError("GPU VideoTransform expects decoded uint8 frames [T, H, W, C]")
        B, T, H, W, C = frames.shape
        params = torch.tensor([self.draw(H, W) for _ in range(B)], dtype=torch.int32)
        frames = frames.to(self.device, non_blocking=True).contiguous()
        out = torch.empty(B, C, T, self.crop_size, self.crop_size, dtype=torch.float32, device=self.device)
        ops.video_transform(frames, params.to(self.device), self.crop_size, self.mean, self.std, out)
        return out[0] if single else out
