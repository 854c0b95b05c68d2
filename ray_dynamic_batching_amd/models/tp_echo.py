"""A minimal tensor-parallel servable: a row-parallel linear layer whose
partial products are summed with an all-reduce across the TP group.

Rank r holds the input columns [r*d/N, (r+1)*d/N) of one fixed weight W
[d_out, d]; y_r = x[:, shard] @ W[:, shard]^T, y = all_reduce(sum, y_r) =
x @ W^T for any N.  The last output column is all_reduce(sum, 1) = N, so a
response proves every rank of the group took part.  Runs on CPU (gloo) and on
GPU (RCCL) -- the plumbing test of Serve's TP replicas; Llama-3 (models/llama.py)
is the real one.
"""
from __future__ import annotations

from typing import Optional

import torch


class TPEcho:
    input_dtype = torch.float32
    output_dtype = torch.float32

    def __init__(self, d: int = 16, d_out: int = 8, tp_rank: int = 0, tp_size: int = 1,
                 group_name: Optional[str] = None, device="cpu", seed: int = 0):
        if d % tp_size:
            raise ValueError("d must be divisible by tp_size")
        self.d, self.d_out = d, d_out
        self.rank, self.tp, self.group = tp_rank, tp_size, group_name
        self.device = torch.device(device)
        g = torch.Generator().manual_seed(seed)
        w = torch.randn(d_out, d, generator=g)
        k = d // tp_size
        self.cols = (tp_rank * k, (tp_rank + 1) * k)
        self.w = w[:, self.cols[0]:self.cols[1]].contiguous().to(self.device)
        self.w_full = w          # the TP=1 reference (tests)

    @property
    def input_shape(self):
        return (self.d,)

    @property
    def output_shape(self):
        return (self.d_out + 1,)

    def example_input(self, batch: int, seed: int = 0, device=None) -> torch.Tensor:
        g = torch.Generator().manual_seed(seed)
        return torch.randn(batch, self.d, generator=g).to(device or self.device)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        a, b = self.cols
        y = torch.cat([x[:, a:b].float() @ self.w.t(), torch.ones(x.shape[0], 1, device=x.device)], dim=1)
        if self.tp > 1:
            from ..parallel import collective as col

            col.allreduce(y, self.group)
        return y

    __call__ = forward

    def reference(self, x: torch.Tensor) -> torch.Tensor:
        """TP = 1 result of the same weights (plus the world column)."""
        return torch.cat([x.float() @ self.w_full.t(), torch.full((x.shape[0], 1), float(self.tp))], dim=1)
