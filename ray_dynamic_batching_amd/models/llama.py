"""Llama-3 decoder (random init) with tensor parallelism for prefill serving
(BASELINE config 4: Llama-3-8B bf16, TP=8 replica, dyn-batch prefill <= 8 prompts).

Per rank (TP = t, MI355X-first layout):
  * token embedding REPLICATED (1 GB bf16 at 8B -- HBM is 288 GB, so no
    vocab-parallel gather + all-reduce is spent on the input side);
  * attention: column-parallel fused QKV (H/t q heads, Hkv/t kv heads, GQA),
    RoPE in place on the packed buffer, causal flash attention, row-parallel
    o_proj whose epilogue adds the residual on rank 0 only, then ONE all-reduce
    (RCCL over xGMI) yields x + attn(x) on every rank;
  * MLP: gate/up weights interleaved row-wise so a single GEMM with the fused
    SwiGLU epilogue produces silu(g)*u (F/t columns); row-parallel down proj
    (+residual on rank 0) then one all-reduce;
  * LM head vocab-parallel: each rank computes its vocab slice of the
    last-token logits, takes a local (max, argmax) and only 2 x B numbers are
    all-gathered to pick the global next token.
Two all-reduces of T x hidden bf16 per layer -- sized for the 7-link xGMI mesh
(see parallel.collective.xgmi_allreduce_time_model).  With the custom xGMI
all-reduce enabled on the group (parallel.xgmi, push-based one/two-shot over
peer memory) each all-reduce also applies the following RMSNorm.
"""
from __future__ import annotations

import zlib
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops


def gather_rows_for_sum(t: torch.Tensor, rank: int, world: int, dtype: torch.dtype) -> torch.Tensor:
    """An all-gather carried by a SUM all-reduce: rank ``rank``'s 4-byte tensor
    ``t`` as its raw bytes (integers 0..255, exact in bf16 / f16) in row ``rank``
    of an otherwise zero [world, D] block (D = bytes rounded up to 8, the xGMI
    kernel's row granularity).  Summing the blocks of all ranks (x + 0, f32
    accumulation) yields every rank's bytes; ``gathered_from_sum`` decodes."""
    if t.element_size() != 4:
        raise ValueError("gather_rows_for_sum: 4-byte elements")
    nb = t.numel() * 4
    buf = torch.zeros((world, -(-nb // 8) * 8), device=t.device, dtype=dtype)
    buf[rank, :nb] = t.contiguous().view(-1).view(torch.uint8).to(dtype)
    return buf


def gathered_from_sum(summed: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    """[world, D] summed byte rows -> [world, *like.shape] tensors of like's dtype."""
    nb = like.numel() * 4
    g = summed[:, :nb].to(torch.uint8).contiguous()
    return g.view(like.dtype).view((summed.shape[0],) + tuple(like.shape))


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    head_dim: int = 128
    intermediate: int = 14336
    rope_theta: float = 500000.0
    eps: float = 1e-5
    max_position: int = 8192
    seq_len: int = 512

    @staticmethod
    def llama3_8b(**kw) -> "LlamaConfig":
        return LlamaConfig(**kw)

    @staticmethod
    def tiny(**kw) -> "LlamaConfig":
        d = dict(vocab_size=1024, hidden=512, layers=2, heads=4, kv_heads=2, head_dim=128, intermediate=1024,
                 max_position=1024, seq_len=64)
        d.update(kw)
        return LlamaConfig(**d)


class LlamaTP:
    """Tensor-parallel shard of a Llama-3 model (tp_size=1 -> whole model)."""

    def __init__(self, cfg: LlamaConfig = None, tp_rank: int = 0, tp_size: int = 1, group_name: Optional[str] = None,
                 device="cuda", dtype=torch.bfloat16, backend: str = "hip", seed: int = 0,
                 init: str = "shard"):
        self.cfg = cfg = cfg or LlamaConfig()
        if cfg.heads % tp_size or cfg.kv_heads % tp_size or cfg.intermediate % tp_size or cfg.vocab_size % tp_size:
            raise ValueError("heads, kv_heads, intermediate and vocab must be divisible by tp_size")
        self.rank, self.tp = tp_rank, tp_size
        self.group = group_name
        self.use_xgmi = True          # custom xGMI all-reduce when the group has one (collective.enable_xgmi)
        # called before every xGMI all-reduce of an EAGER forward (tests that run
        # several TP ranks on ONE GPU: a rank spinning in the all-reduce kernel
        # can hold the CU slots a peer's GEMM needs, so they line up first)
        self.pre_collective = None
        self.device = torch.device(device)
        self.dtype = dtype
        self.backend = backend
        D, Dh = cfg.hidden, cfg.head_dim
        self.Hl, self.Hkvl = cfg.heads // tp_size, cfg.kv_heads // tp_size
        self.Fl = cfg.intermediate // tp_size
        self.Vl = cfg.vocab_size // tp_size
        r = tp_rank

        def gen(tag):  # process-independent seed (python's hash() is salted per process)
            return torch.Generator(device="cpu").manual_seed(zlib.crc32(repr((seed, tag)).encode()) & 0x7FFFFFFF)

        def full(tag, *shape, std=0.02):
            return torch.randn(*shape, generator=gen(tag)) * std

        def dev(t):
            return t.to(device=self.device, dtype=dtype).contiguous()

        # init="full": build full matrices on CPU and slice (identical model for any
        # tp_size -- used by the TP-equivalence tests); init="shard": generate each
        # shard directly (random init of an 8B model without 16 GB host tensors).
        def shard(tag, rows_full, cols, row_slices):
            if init == "full":
                w = full(tag, rows_full, cols)
                return dev(torch.cat([w[a:b] for a, b in row_slices]))
            n = sum(b - a for a, b in row_slices)
            return dev(full((tag, r), n, cols))

        def col_shard(tag, rows, cols_full, a, b):
            if init == "full":
                return dev(full(tag, rows, cols_full)[:, a:b])
            return dev(full((tag, r), rows, b - a))

        self.embed = dev(full("embed", cfg.vocab_size, D))
        self.layers = []
        q0, q1 = r * self.Hl * Dh, (r + 1) * self.Hl * Dh
        kvd = cfg.kv_heads * Dh
        k0, k1 = cfg.heads * Dh + r * self.Hkvl * Dh, cfg.heads * Dh + (r + 1) * self.Hkvl * Dh
        v0, v1 = k0 + kvd, k1 + kvd
        f0, f1 = r * self.Fl, (r + 1) * self.Fl
        for i in range(cfg.layers):
            qkv_rows = (cfg.heads + 2 * cfg.kv_heads) * Dh
            w_qkv = shard(("qkv", i), qkv_rows, D, [(q0, q1), (k0, k1), (v0, v1)])
            w_o = col_shard(("o", i), D, cfg.heads * Dh, q0, q1)
            if init == "full":
                g = full(("gate", i), cfg.intermediate, D)[f0:f1]
                u = full(("up", i), cfg.intermediate, D)[f0:f1]
            else:
                g = full(("gate", i, r), self.Fl, D)
                u = full(("up", i, r), self.Fl, D)
            w_gu = dev(torch.stack([g, u], dim=1).reshape(2 * self.Fl, D))   # rows: g0,u0,g1,u1,...
            w_down = col_shard(("down", i), D, cfg.intermediate, f0, f1)
            self.layers.append(dict(attn_norm=dev(torch.ones(D)), w_qkv=w_qkv, w_o=w_o,
                                    mlp_norm=dev(torch.ones(D)), w_gu=w_gu, w_down=w_down))
        self.final_norm = dev(torch.ones(D))
        self.lm_head = shard("lm_head", cfg.vocab_size, D, [(r * self.Vl, (r + 1) * self.Vl)])
        self.cos, self.sin = ops.rope_tables(cfg.max_position, Dh, cfg.rope_theta, device=self.device)

    # -- servable contract: one prompt of seq_len tokens -> next-token id
    @property
    def input_shape(self):
        return (self.cfg.seq_len,)

    input_dtype = torch.int32
    output_shape = (2,)            # (token id, as int32; logit bits as int32)
    output_dtype = torch.int32

    def _allreduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp > 1:
            from ..parallel import collective as col

            col.allreduce(t, self.group or "default")
        return t

    def _allgather(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp == 1:
            return t.unsqueeze(0)
        from ..parallel import collective as col

        xg = self._xgmi()
        if xg is not None and t.element_size() == 4:
            # over the xGMI all-reduce (graph-capturable on any host group, gloo
            # included): rank r writes its tensor's BYTES as bf16 integers 0..255
            # into row r of a zero [tp, D] block; the sum over ranks is then the
            # gather, exactly (x + 0 in f32, integers < 256 exact in bf16)
            buf = gather_rows_for_sum(t, self.rank, self.tp, xg.dtype)
            if self.pre_collective is not None:
                self.pre_collective()
            return gathered_from_sum(xg.all_reduce(buf), t)
        out = torch.empty((self.tp,) + tuple(t.shape), device=t.device, dtype=t.dtype)
        col.allgather_into(out.view(self.tp * t.shape[0], *t.shape[1:]) if t.dim() else out, t,
                           self.group or "default")
        return out

    @torch.no_grad()
    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, S] int32 -> [B, 2] int32: next-token id and its logit (f32 bits)."""
        x = self.hidden_states(ids)
        return self._next_token(x, ids.shape[0], ids.shape[1])

    __call__ = forward

    def hidden_states(self, ids: torch.Tensor) -> torch.Tensor:
        if self.backend == "hip":
            return self._layers_hip(ids)
        return self._layers_torch(ids)

    def _xgmi(self):
        if self.tp == 1 or not self.use_xgmi:
            return None
        from ..parallel import collective as col

        return col.get_xgmi(self.group or "default")

    def _layers_hip(self, ids):
        c = self.cfg
        B, S = ids.shape
        Dh = c.head_dim
        x = self.embed[ids.long().clamp_(0, c.vocab_size - 1)].reshape(B * S, c.hidden)
        first = self.rank == 0
        xg = self._xgmi()
        if xg is not None and B * S * c.hidden <= xg.max_elems:
            return self._layers_hip_xgmi(x, B, S, xg)
        for L in self.layers:
            h = ops.rms_norm(x, L["attn_norm"], c.eps)
            qkv = ops.linear(h, L["w_qkv"])
            ops.rope_(qkv, self.cos, self.sin, B, S, self.Hl, self.Hkvl, Dh)
            a = ops.attention(qkv, B, S, self.Hl, self.Hkvl, Dh, causal=True)
            x = self._allreduce(ops.linear(a, L["w_o"], residual=x if first else None))
            h = ops.rms_norm(x, L["mlp_norm"], c.eps)
            g = ops.linear(h, L["w_gu"], act="swiglu")
            x = self._allreduce(ops.linear(g, L["w_down"], residual=x if first else None))
        return x

    def _layers_hip_xgmi(self, x, B, S, xg):
        """TP layers with the custom xGMI all-reduce: each all-reduce also
        applies the NEXT RMSNorm (fused in the all-gather phase), so a layer is
        qkv GEMM -> RoPE -> attention -> o GEMM(+res) -> AR+norm -> gate/up
        GEMM(SwiGLU) -> down GEMM(+res) -> AR+norm; x lives in the
        communicator's gather buffer between the two all-reduces."""
        c = self.cfg
        Dh = c.head_dim
        first = self.rank == 0
        h = ops.rms_norm(x, self.layers[0]["attn_norm"], c.eps)
        n = len(self.layers)
        for i, L in enumerate(self.layers):
            qkv = ops.linear(h, L["w_qkv"])
            ops.rope_(qkv, self.cos, self.sin, B, S, self.Hl, self.Hkvl, Dh)
            a = ops.attention(qkv, B, S, self.Hl, self.Hkvl, Dh, causal=True)
            o = ops.linear(a, L["w_o"], residual=x if first else None)
            if self.pre_collective is not None:
                self.pre_collective()
            x, h = xg.all_reduce_rmsnorm(o, L["mlp_norm"], c.eps)
            g = ops.linear(h, L["w_gu"], act="swiglu")
            d = ops.linear(g, L["w_down"], residual=x if first else None)
            if self.pre_collective is not None:
                self.pre_collective()
            if i + 1 < n:
                x, h = xg.all_reduce_rmsnorm(d, self.layers[i + 1]["attn_norm"], c.eps)
            else:
                x = xg.all_reduce(d)
        return x

    def _layers_torch(self, ids):
        c = self.cfg
        B, S = ids.shape
        Dh = c.head_dim
        x = self.embed[ids.long().clamp(0, c.vocab_size - 1)].reshape(B * S, c.hidden)
        pos = torch.arange(S, device=x.device)
        cos, sin = self.cos[pos], self.sin[pos]

        def rope(t, n):
            t = t.view(B, S, n, Dh).float()
            t1, t2 = t[..., : Dh // 2], t[..., Dh // 2:]
            cc, ss = cos[None, :, None, :], sin[None, :, None, :]
            return torch.cat([t1 * cc - t2 * ss, t2 * cc + t1 * ss], -1).to(x.dtype)

        def rms(t, w):
            tf = t.float()
            return (tf * torch.rsqrt(tf.pow(2).mean(-1, keepdim=True) + c.eps) * w.float()).to(t.dtype)

        for L in self.layers:
            h = rms(x, L["attn_norm"])
            qkv = F.linear(h, L["w_qkv"])
            q = rope(qkv[:, : self.Hl * Dh], self.Hl).transpose(1, 2)
            k = rope(qkv[:, self.Hl * Dh:(self.Hl + self.Hkvl) * Dh], self.Hkvl).transpose(1, 2)
            v = qkv[:, (self.Hl + self.Hkvl) * Dh:].reshape(B, S, self.Hkvl, Dh).transpose(1, 2)
            if self.Hkvl != self.Hl:
                k = k.repeat_interleave(self.Hl // self.Hkvl, 1)
                v = v.repeat_interleave(self.Hl // self.Hkvl, 1)
            a = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B * S, self.Hl * Dh)
            o = F.linear(a, L["w_o"])
            if self.rank == 0:
                o = o + x
            x = self._allreduce(o)
            h = rms(x, L["mlp_norm"])
            gu = F.linear(h, L["w_gu"]).float()
            m = (F.silu(gu[:, 0::2]) * gu[:, 1::2]).to(x.dtype)
            d = F.linear(m, L["w_down"])
            if self.rank == 0:
                d = d + x
            x = self._allreduce(d)
        return x

    def _next_token(self, x: torch.Tensor, B: int, S: int) -> torch.Tensor:
        c = self.cfg
        last = x.view(B, S, c.hidden)[:, -1, :].contiguous()
        if self.backend == "hip":
            h = ops.rms_norm(last, self.final_norm, c.eps)
            logits = ops.linear(h, self.lm_head, out_dtype=torch.float32)
        else:
            lf = last.float()
            h = (lf * torch.rsqrt(lf.pow(2).mean(-1, keepdim=True) + c.eps) * self.final_norm.float()).to(x.dtype)
            logits = F.linear(h, self.lm_head).float()
        val, idx = logits.max(dim=-1)                             # local vocab slice
        loc = torch.stack([val, (idx + self.rank * self.Vl).float()], dim=-1)  # [B, 2]
        allv = self._allgather(loc)                               # [tp, B, 2]
        best = allv[..., 0].argmax(dim=0)                         # [B]
        bi = torch.arange(B, device=x.device)
        tok = allv[best, bi, 1].to(torch.int32)
        logit = allv[best, bi, 0].contiguous().view(torch.int32)
        return torch.stack([tok, logit], dim=-1).contiguous()

    def example_input(self, batch: int, seed: int = 0, device=None) -> torch.Tensor:
        g = torch.Generator(device="cpu").manual_seed(seed)
        return torch.randint(1, self.cfg.vocab_size, (batch, self.cfg.seq_len), generator=g,
                             dtype=torch.int32).to(device or self.device)

    def flops_per_prompt(self) -> float:
        c, S = self.cfg, self.cfg.seq_len
        per_tok = 2 * (c.hidden * (c.heads + 2 * c.kv_heads) * c.head_dim + c.heads * c.head_dim * c.hidden
                       + 3 * c.hidden * c.intermediate)
        attn = 2 * 2 * S * c.heads * c.head_dim / 2
        return c.layers * S * (per_tok + attn)
