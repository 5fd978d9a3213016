"""Multi-sequence wrappers with the reference's call semantics (src/utils/wrappers.py:9-43).

They loop over (frames-per-clip group, mask) exactly like the reference (one encoder / predictor
call per mask). The train step does not use them on its hot path: it runs every mask of a group in
one ragged pass (VisionTransformer.forward_ragged / VisionTransformerPredictor.forward_ragged).
"""

import torch.nn as nn


class MultiSeqWrapper(nn.Module):
    def __init__(self, backbone):
        super().__init__()
        self.backbone = backbone

    def forward(self, x, masks=None):
        if masks is None:
            return [self.backbone(xi) for xi in x]
        return [[self.backbone(xi, masks=mij) for mij in mi] for xi, mi in zip(x, masks)]


class PredictorMultiSeqWrapper(nn.Module):
    def __init__(self, backbone):
        super().__init__()
        self.backbone = backbone

    def forward(self, x, masks_x, masks_y, has_cls=False):
        return [[self.backbone(xij, mxij, myij, mask_index=i, has_cls=has_cls)
                 for xij, mxij, myij in zip(xi, mxi, myi)]
                for i, (xi, mxi, myi) in enumerate(zip(x, masks_x, masks_y))]
