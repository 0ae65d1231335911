"""Deterministic random initialisation for benchmarking without checkpoints
(no pretrained weights are reachable offline).

He-normal convolutions; BN running statistics near (0, 1) with gamma ~1 on
activated BNs and ~0.3 on the residual-branch ends, so activations stay O(1)
through the deepest nets (bf16 MFMA clocks depend on operand values; the
benchmark must run on realistic, non-degenerate data)."""

import torch

from ..modules.abn import ABN


@torch.no_grad()
def random_init_(net, seed=0):
    g = torch.Generator().manual_seed(seed)
    for name, mod in net.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            fan_in = mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1]
            mod.weight.copy_(torch.randn(mod.weight.shape, generator=g) * (2.0 / fan_in) ** 0.5)
        elif isinstance(mod, ABN):
            c = mod.num_features
            branch_end = name.endswith("bn3") or (name.endswith("bn2") and mod.activation == "identity")
            lo, hi = (0.2, 0.4) if branch_end else (0.8, 1.2)
            mod.weight.copy_(torch.rand(c, generator=g) * (hi - lo) + lo)
            mod.bias.copy_((torch.rand(c, generator=g) - 0.5) * 0.04)
            mod.running_mean.copy_((torch.rand(c, generator=g) - 0.5) * 0.04)
            mod.running_var.copy_(torch.rand(c, generator=g) * 0.4 + 0.8)
        elif isinstance(mod, torch.nn.Linear):
            std = 0.1 * (2.0 / (mod.in_features + mod.out_features)) ** 0.5
            mod.weight.copy_(torch.randn(mod.weight.shape, generator=g) * std)
            if mod.bias is not None:
                mod.bias.zero_()
    for m in net.modules():
        if hasattr(m, "refresh_engine"):
            m.refresh_engine()
    return net
