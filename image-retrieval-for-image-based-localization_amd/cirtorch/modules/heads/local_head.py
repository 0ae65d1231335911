"""localHead (reference ``cirtorch/modules/heads/local_head.py:19-71``).

forward(x [B, C, H, W], kpts [B, N, 2] normalised (x, y) grid coordinates)
-> descriptors [B, N, E]: bilinear ``grid_sample`` of the feature map at the
keypoints (zeros padding, align_corners=False), ``nn.Linear(dim, E)``
("whiten", state keys ``whiten.weight`` / ``whiten.bias``), then
``functional.normalize`` over E — one ``rr_local_head`` call (sample kernel,
exact-f32 MFMA Linear, normalisation).
"""

import torch.nn as nn

from ... import _ops
from ..abn import ABN


class localHead(nn.Module):
    def __init__(self, dim, embedding_size=None, norm_act=ABN):
        super().__init__()
        self.whiten = nn.Linear(dim, embedding_size, bias=True)
        self.reset_parameters()

    def reset_parameters(self):
        for _name, mod in self.named_modules():
            if isinstance(mod, nn.Linear):
                nn.init.xavier_normal_(mod.weight, 0.1)
            elif isinstance(mod, ABN):
                nn.init.constant_(mod.weight, 1.0)
            if hasattr(mod, "bias") and isinstance(getattr(mod, "bias"), nn.Parameter) and mod.bias is not None:
                nn.init.constant_(mod.bias, 0.0)

    def forward(self, x, kpts=None, img_size=None):
        return _ops.local_head(x, kpts, self.whiten.weight, self.whiten.bias)
