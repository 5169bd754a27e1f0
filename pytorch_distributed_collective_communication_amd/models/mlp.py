"""A small MLP used to exercise data-parallel training on the backend
(the DP use case the reference's README motivates, README.md:5)."""
from __future__ import annotations

import torch
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self, d_in: int = 32, d_hidden: int = 64, d_out: int = 8, depth: int = 3):
        super().__init__()
        layers = [nn.Linear(d_in, d_hidden), nn.GELU()]
        for _ in range(depth - 2):
            layers += [nn.Linear(d_hidden, d_hidden), nn.GELU()]
        layers.append(nn.Linear(d_hidden, d_out))
        self.net = nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)


def synthetic_batch(n: int, d_in: int = 32, d_out: int = 8, seed: int = 0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d_in, generator=g)
    w = torch.randn(d_in, d_out, generator=g)
    y = x @ w + 0.1 * torch.randn(n, d_out, generator=g)
    return x.to(device), y.to(device)
