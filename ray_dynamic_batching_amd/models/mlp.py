"""2-layer MLP (BASELINE config 1: CPU plumbing model, Linear -> ReLU -> Linear)."""
from __future__ import annotations

import torch


class MLP:
    def __init__(self, d_in: int = 32, d_hidden: int = 64, d_out: int = 8, device="cpu", dtype=torch.float32,
                 seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.device = torch.device(device)
        self.w1 = (torch.randn(d_hidden, d_in, generator=g) * d_in ** -0.5).to(self.device, dtype)
        self.b1 = torch.zeros(d_hidden, device=self.device, dtype=dtype)
        self.w2 = (torch.randn(d_out, d_hidden, generator=g) * d_hidden ** -0.5).to(self.device, dtype)
        self.b2 = torch.zeros(d_out, device=self.device, dtype=dtype)
        self.input_shape, self.output_shape = (d_in,), (d_out,)
        self.input_dtype = self.output_dtype = dtype

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = torch.relu(x.to(self.w1.dtype) @ self.w1.t() + self.b1)
        return (h @ self.w2.t() + self.b2).contiguous()

    __call__ = forward

    def example_input(self, batch: int, seed: int = 0, device=None):
        g = torch.Generator(device="cpu").manual_seed(seed)
        return torch.randn(batch, *self.input_shape, generator=g).to(device or self.device)
