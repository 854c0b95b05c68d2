"""BERT-base sequence classifier (random init) on the gfx950 kernels.

The north-star serving model (BASELINE.json: "BERT-base seq128 bf16").  The
``hip`` backend runs every op of the batched forward on the hand-written
kernels of :mod:`ray_dynamic_batching_amd.ops`:

  embed_ln (gather + LN fused) -> 12 x [ QKV GEMM(+bias) + attention in ONE
  kernel per layer (ops.qkv_attention: each (sequence, head) block projects
  its q/k/v tile and attends in LDS, key-padding mask from per-row lengths;
  S > 128 falls back to GEMM -> ops.attention) -> out GEMM
  (+bias +residual) -> LN -> FFN1 GEMM(+bias +GELU) -> FFN2 GEMM(+bias
  +residual) -> LN ] -> pooler GEMM(+tanh) on the strided CLS rows ->
  classifier GEMM (f32 logits)

so one layer is 6 kernel launches; it is captured
once per batch bucket into a hipGraph by the replica engine.  The ``torch``
backend is the eager PyTorch baseline (what the reference's serving path
runs: ``model(inputs)`` at scheduler.py:450).
"""
from __future__ import annotations

import os

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .. import ops


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    num_labels: int = 2
    seq_len: int = 128
    pad_token_id: int = 0

    @staticmethod
    def base(**kw) -> "BertConfig":
        return BertConfig(**kw)

    @staticmethod
    def tiny(**kw) -> "BertConfig":
        d = dict(vocab_size=1000, hidden=256, layers=2, heads=4, intermediate=512, max_position=128, seq_len=32)
        d.update(kw)
        return BertConfig(**d)


def bert_tile_signature(cfg: BertConfig, backend: str = "hip"):
    """Key of the shipped MI355X tile tables (runtime.engine.shipped_tile_table):
    only the BERT-base dims were tuned, only for the HIP kernels."""
    base = (cfg.hidden, cfg.heads, cfg.intermediate) == (768, 12, 3072)
    return f"bert_L{cfg.layers}_S{cfg.seq_len}" if base and backend == "hip" else None


class BertForSequenceClassification:
    """Weights are plain tensors (random N(0, 0.02) init, as BERT's initializer)."""

    def __init__(self, cfg: BertConfig = None, device="cuda", dtype=torch.bfloat16, backend: str = "hip",
                 seed: int = 0):
        self.cfg = cfg = cfg or BertConfig()
        self.device = torch.device(device)
        self.dtype = dtype
        if backend == "hip" and self.device.type != "cuda":
            raise ValueError("the hip backend needs a GPU device")
        self.backend = backend
        self.tile_signature = bert_tile_signature(cfg, backend)
        self.cls_only_last_layer = True
        # deferred LayerNorm (ops.linear_ln): the GEMMs around each LayerNorm
        # carry it, no LayerNorm kernel runs inside the layer stack
        # (RDB_BERT_FOLD_LN=1/0 forces it; by default a replica engine enables it
        # only with one compute stream -- see EngineRunner.build)
        # fused QKV projection + attention (ops.qkv_attention, S <= 128): the QKV
        # activation is never materialised; RDB_BERT_FUSED_ATTN=0 runs the
        # two-kernel path (GEMM -> ops.attention)
        self.fuse_qkv_attn = os.environ.get("RDB_BERT_FUSED_ATTN", "1") != "0"
        # RDB_BERT_LNOUT=1: o-proj / FFN-down with the residual add AND the
        # LayerNorm in the GEMM epilogue (ops.linear_residual_ln, row-panel
        # statistics through a workspace + arrival counter): no LayerNorm kernel
        # in the layer stack, but the panel wait (~2 memory round trips on the
        # critical path) costs more than the LayerNorm kernel it removes
        # (+11 us vs -5 us per GEMM, profiles/ab_r2.json) -- off by default
        self.fuse_residual_ln = os.environ.get("RDB_BERT_LNOUT", "0") == "1"
        # RDB_BERT_ROWLN: o-proj -> LN1 ("o"), FFN-down -> LN2 ("d") or both ("1")
        # on the full-row GEMM + LayerNorm kernel (ops.linear_rowln: 64-row blocks
        # own whole 768-wide rows, statistics block-local) for batches of at
        # least RDB_BERT_ROWLN_MIN_ROWS token rows; "0" = tiled GEMM + LayerNorm kernel
        rl = os.environ.get("RDB_BERT_ROWLN", "0")
        self.rowln_o = rl in ("1", "o")
        self.rowln_d = rl in ("1", "d")
        self.rowln_min_rows = int(os.environ.get("RDB_BERT_ROWLN_MIN_ROWS", "2048"))
        # RDB_ABLATE (profiling only -- WRONG outputs, never a measurement): comma
        # list of ops to skip in the hip forward ("ln": the in-stack LayerNorm
        # kernels, "gelu": FFN-up's activation) to bound what removing them can buy
        self.ablate = {a for a in os.environ.get("RDB_ABLATE", "").split(",") if a}
        # RDB_BERT_LN_PSTATS=1: no LayerNorm kernel in the stack and no statistics
        # work in any main loop -- o-proj / FFN-down write per-N-tile partial row
        # statistics from their staged epilogues, FFN-up / the next QKV+attention
        # run on the raw rows with the LayerNorm folded into their weights, residual
        # adds normalise on load (_forward_hip_pstats)
        self.ln_pstats = os.environ.get("RDB_BERT_LN_PSTATS", "0") == "1"
        if backend == "hip" and (self.fuse_residual_ln or self.rowln_o or self.rowln_d or self.ln_pstats):
            from .. import ops as _ops_mod

            if not _ops_mod.experimental_kernels_built():
                raise RuntimeError("RDB_BERT_LNOUT / RDB_BERT_ROWLN / RDB_BERT_LN_PSTATS run kernels that lost their "
                                   "A/Bs and are only in the opt-in RDB_EXPERIMENTAL_KERNELS build (ops/csrc/common.h)")
        env = os.environ.get("RDB_BERT_FOLD_LN", "")
        self.fold_ln_auto = env == ""
        self.fold_ln = env == "1" or (env == "" and self.auto_fold_ln(1))
        self._folded = None
        self._packed = None
        g = torch.Generator(device="cpu").manual_seed(seed)
        D, I = cfg.hidden, cfg.intermediate

        def w(*shape, std=0.02):
            return (torch.randn(*shape, generator=g) * std).to(device=self.device, dtype=dtype)

        def ones(n):
            return torch.ones(n, device=self.device, dtype=dtype)

        def zeros(n):
            return torch.zeros(n, device=self.device, dtype=dtype)

        self.word = w(cfg.vocab_size, D)
        self.pos = w(cfg.max_position, D)
        self.typ = w(cfg.type_vocab, D)
        self.emb_g, self.emb_b = ones(D), zeros(D)
        self.layers = []
        for _ in range(cfg.layers):
            self.layers.append(dict(
                w_qkv=w(3 * D, D), b_qkv=w(3 * D), w_o=w(D, D), b_o=w(D),
                ln1_g=ones(D), ln1_b=zeros(D), w_i=w(I, D), b_i=w(I), w_out=w(D, I), b_out=w(D),
                ln2_g=ones(D), ln2_b=zeros(D)))
        self.w_pool, self.b_pool = w(D, D), w(D)
        self.w_cls, self.b_cls = w(cfg.num_labels, D), w(cfg.num_labels)

    # -- serving contract (see runtime.engine.EngineRunner) --------------------
    @property
    def input_shape(self):
        return (self.cfg.seq_len,)

    input_dtype = torch.int32

    @property
    def output_shape(self):
        return (self.cfg.num_labels,)

    output_dtype = torch.float32

    def param_bytes(self) -> int:
        n = sum(t.numel() for t in [self.word, self.pos, self.typ, self.w_pool, self.w_cls])
        n += sum(t.numel() for L in self.layers for t in L.values())
        return n * torch.finfo(self.dtype).bits // 8

    def flops_per_sequence(self) -> float:
        c, S = self.cfg, self.cfg.seq_len
        per_tok = 2 * (4 * c.hidden * c.hidden + 2 * c.hidden * c.intermediate)
        attn = 2 * 2 * S * c.hidden
        return c.layers * S * (per_tok + attn)

    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        return self.forward(ids)

    @torch.no_grad()
    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if self.backend == "hip":
            return self._forward_hip(ids)
        return self._forward_torch(ids)

    def auto_fold_ln(self, compute_streams: int) -> bool:
        """Default for ``fold_ln``.  The deferred-LN forward shortens a lone
        batch's forward only against the two-kernel attention path (-1.5 % at
        bs32 seq128, bench/bert_breakdown.py); the fused projection+attention
        kernel (S <= 128) beats it by 12 %, and with several compute streams the
        LayerNorm kernels hide under the other stream's GEMMs anyway
        (profiles/bert_fold_ln_ab.json)."""
        c = self.cfg
        fused = self.fuse_qkv_attn and ops.qkv_attention_supported(c.seq_len, c.heads, c.hidden // c.heads, c.hidden)
        return compute_streams == 1 and not fused

    def refresh_folded_weights(self):
        """Recompute the LayerNorm-folded weights (call after changing weights)."""
        self._folded = None

    def _fold_key(self):
        """Identity + in-place version of every tensor the folded weights derive
        from: a weight swapped or modified after a warm-up forward re-folds."""
        return tuple((t.data_ptr(), t._version) for L in self.layers
                     for t in (L["w_qkv"], L["b_qkv"], L["w_i"], L["b_i"], L["ln1_g"], L["ln1_b"],
                               L["ln2_g"], L["ln2_b"]))

    def _packed_qkv(self):
        """Head-major QKV weights for ops.qkv_attention, rebuilt when a source
        tensor is swapped or modified in place."""
        key = tuple((t.data_ptr(), t._version) for L in self.layers for t in (L["w_qkv"], L["b_qkv"]))
        if self._packed is None or self._packed[0] != key:
            H = self.cfg.heads
            self._packed = (key, [ops.pack_qkv_heads(L["w_qkv"], L["b_qkv"], H) for L in self.layers])
        return self._packed[1]

    def _rowln_weights(self):
        """Per layer (w_o, w_out) packed for ops.linear_rowln, rebuilt when a
        source tensor is swapped or modified in place."""
        key = tuple((t.data_ptr(), t._version) for L in self.layers for t in (L["w_o"], L["w_out"]))
        if getattr(self, "_rowln", None) is None or self._rowln[0] != key:
            self._rowln = (key, [(ops.pack_rowln_weight(L["w_o"]), ops.pack_rowln_weight(L["w_out"]))
                                 for L in self.layers])
        return self._rowln[1]

    def _folded_weights(self):
        key = self._fold_key()
        if self._folded is not None and getattr(self, "_folded_key", None) != key:
            self._folded = None
        if self._folded is None:
            self._folded_key = key
            f = []
            for i, L in enumerate(self.layers):
                d = {}
                if i > 0:   # layer i's QKV consumes LN2 of layer i-1
                    P = self.layers[i - 1]
                    d["w_qkv"], d["cs_qkv"], d["b_qkv"] = ops.fold_ln_weights(L["w_qkv"], L["b_qkv"], P["ln2_g"],
                                                                              P["ln2_b"])
                d["w_i"], d["cs_i"], d["b_i"] = ops.fold_ln_weights(L["w_i"], L["b_i"], L["ln1_g"], L["ln1_b"])
                f.append(d)
            self._folded = f
        return self._folded

    def _deferred_weights(self):
        """Per layer, for _forward_hip_fused_deferred: the packed QKV weight with
        the previous layer's LN2 folded in (layer 0: plain) and FFN-up with LN1
        folded in; rebuilt when a source tensor is swapped or modified."""
        key = tuple((t.data_ptr(), t._version) for L in self.layers
                    for t in (L["w_qkv"], L["b_qkv"], L["w_i"], L["b_i"], L["ln1_g"], L["ln1_b"],
                              L["ln2_g"], L["ln2_b"]))
        if getattr(self, "_deferred", None) is None or self._deferred[0] != key:
            H = self.cfg.heads
            out = []
            for i, L in enumerate(self.layers):
                d = {}
                if i == 0:
                    d["wq"], d["bq"] = ops.pack_qkv_heads(L["w_qkv"], L["b_qkv"], H)
                else:
                    P = self.layers[i - 1]
                    w2, cs, bf = ops.fold_ln_weights(L["w_qkv"], L["b_qkv"], P["ln2_g"], P["ln2_b"])
                    d["wq"], d["bfq"] = ops.pack_qkv_heads(w2, bf, H)
                    d["csq"] = ops.pack_qkv_vec(cs, H)
                d["w_i"], d["cs_i"], d["b_i"] = ops.fold_ln_weights(L["w_i"], L["b_i"], L["ln1_g"], L["ln1_b"])
                out.append(d)
            self._deferred = (key, out)
        return self._deferred[1]

    def _forward_hip(self, ids: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        if (self.ln_pstats and self.dtype == torch.bfloat16 and c.hidden % 8 == 0 and c.intermediate % 8 == 0
                and self.fuse_qkv_attn and ops.qkv_attention_supported(ids.shape[1], c.heads, c.hidden // c.heads,
                                                                       c.hidden)):
            return self._forward_hip_pstats(ids)
        if self.fold_ln and self.dtype == torch.bfloat16 and c.hidden % 4 == 0:
            if self.fuse_qkv_attn and ops.qkv_attention_supported(ids.shape[1], c.heads, c.hidden // c.heads, c.hidden):
                return self._forward_hip_fused_deferred(ids)
            return self._forward_hip_folded(ids)
        c = self.cfg
        B, S = ids.shape
        D, H = c.hidden, c.heads
        fuse = self.fuse_qkv_attn and ops.qkv_attention_supported(S, H, D // H, D)
        # the fused kernel counts each sequence's key length from the ids itself
        kid = ((ids.contiguous(), c.pad_token_id) if fuse and ids.dtype == torch.int32
               and os.environ.get("RDB_BERT_KEY_IDS", "1") != "0" else None)
        lens = None if kid is not None else ops.seq_lens(ids, c.pad_token_id)
        n = len(self.layers)
        lnout = self.fuse_residual_ln and self.dtype == torch.bfloat16 and D % 8 == 0
        # row-panel LayerNorm workspaces, 2 per LNOUT GEMM: zeroed by the embedding kernel
        ws = torch.empty(4 * n, B * S, 2, device=ids.device, dtype=torch.float32) if lnout else None
        h = ops.embed_ln(ids, self.word, self.pos, self.typ, self.emb_g, self.emb_b, c.eps, zero_stats=ws)
        packed = self._packed_qkv() if fuse else None
        for i, L in enumerate(self.layers):
            if fuse:   # one kernel: projection tile of (sequence, head) -> attention in LDS
                ctx = ops.qkv_attention(h.reshape(B * S, D), packed[i][0], packed[i][1], B, S, H, lens=lens,
                                        key_ids=kid)
            else:
                qkv = ops.linear(h, L["w_qkv"], L["b_qkv"])
                ctx = ops.attention(qkv, B, S, H, H, D // H, lens=lens)
            if i == n - 1 and self.cls_only_last_layer:
                # Only the [CLS] row of the last layer reaches the pooler: its
                # keys/values need every token, but the o-proj, LN and FFN after
                # attention are row-wise, so they run on the B CLS rows (strided
                # views, no copy) instead of B*S -- the same logits, ~1/12 fewer FLOPs.
                ctx, h = ctx.view(B, S, D)[:, 0, :], h.view(B, S, D)[:, 0, :]
            elif lnout:
                h2 = h.reshape(B * S, D)
                h1 = ops.linear_residual_ln(ctx, L["w_o"], L["b_o"], h2, L["ln1_g"], L["ln1_b"], c.eps,
                                            ws[4 * i], ws[4 * i + 1].view(torch.int32))
                inter = ops.linear(h1, L["w_i"], L["b_i"], act="gelu")
                h = ops.linear_residual_ln(inter, L["w_out"], L["b_out"], h1, L["ln2_g"], L["ln2_b"], c.eps,
                                           ws[4 * i + 2], ws[4 * i + 3].view(torch.int32))
                continue
            rows = ctx.shape[0]
            cls_rows = i == n - 1 and self.cls_only_last_layer
            rowln = (not cls_rows and self.dtype == torch.bfloat16 and rows >= self.rowln_min_rows
                     and (self.rowln_o or self.rowln_d) and ops.linear_rowln_supported(rows, D, D)
                     and ops.linear_rowln_supported(rows, D, c.intermediate))
            rp = self._rowln_weights()[i] if rowln else None
            if rowln and self.rowln_o:
                h1 = ops.linear_rowln(ctx, rp[0], L["b_o"], h, L["ln1_g"], L["ln1_b"], c.eps)
            else:
                a = ops.linear(ctx, L["w_o"], L["b_o"], residual=h)
                h1 = a if "ln" in self.ablate and not cls_rows else ops.layer_norm(a, L["ln1_g"], L["ln1_b"], c.eps)
            inter = ops.linear(h1, L["w_i"], L["b_i"], act="none" if "gelu" in self.ablate else "gelu")
            if rowln and self.rowln_d:
                h = ops.linear_rowln(inter, rp[1], L["b_out"], h1, L["ln2_g"], L["ln2_b"], c.eps)
            else:
                o = ops.linear(inter, L["w_out"], L["b_out"], residual=h1)
                h = o if "ln" in self.ablate and not cls_rows else ops.layer_norm(o, L["ln2_g"], L["ln2_b"], c.eps)
        cls = h if self.cls_only_last_layer else h.view(B, S, D)[:, 0, :]
        pooled = ops.linear(cls, self.w_pool, self.b_pool, act="tanh")
        return ops.linear(pooled, self.w_cls, self.b_cls, out_dtype=torch.float32)

    def _forward_hip_fused_deferred(self, ids: torch.Tensor) -> torch.Tensor:
        """Four kernels per layer and no LayerNorm kernel inside the stack:
        fused QKV+attention reading the RAW residual stream with LN2 folded into
        its weights (row statistics computed in its own main loop, published by
        head 0), o-proj normalising that residual on load, FFN-up with LN1 folded
        in (statistics again computed in-loop, published by the first N tile),
        FFN-down normalising its residual on load.  No statistics pass, no atomics."""
        c = self.cfg
        B, S = ids.shape
        D, H, eps = c.hidden, c.heads, c.eps
        Wd = self._deferred_weights()
        lens = ops.seq_lens(ids, c.pad_token_id)
        M = B * S
        n = len(self.layers)
        stats = torch.empty(n, 2, M, 2, device=ids.device, dtype=torch.float32)   # (x rows, a rows) per layer
        x = ops.embed_ln(ids, self.word, self.pos, self.typ, self.emb_g, self.emb_b, eps).reshape(M, D)
        xg = xb = None             # x is raw (pre-LN2 of the previous layer) iff xg is not None
        h = None
        for i, L in enumerate(self.layers):
            st_x, st_a = stats[i, 0], stats[i, 1]
            d = Wd[i]
            if xg is None:
                ctx = ops.qkv_attention(x, d["wq"], d["bq"], B, S, H, lens=lens)
            else:
                ctx = ops.qkv_attention(x, d["wq"], None, B, S, H, lens=lens, lna=(d["csq"], d["bfq"], eps),
                                        stats_out=st_x)
            if i == n - 1 and self.cls_only_last_layer:
                xc = x.view(B, S, D)[:, 0, :]
                hc = xc if xg is None else ops.layer_norm(xc, xg, xb, eps)
                a = ops.linear(ctx.view(B, S, D)[:, 0, :], L["w_o"], L["b_o"], residual=hc)
                h1 = ops.layer_norm(a, L["ln1_g"], L["ln1_b"], eps)
                inter = ops.linear(h1, L["w_i"], L["b_i"], act="gelu")
                o = ops.linear(inter, L["w_out"], L["b_out"], residual=h1)
                h = ops.layer_norm(o, L["ln2_g"], L["ln2_b"], eps)
                break
            if xg is None:
                a = ops.linear(ctx, L["w_o"], L["b_o"], residual=x)
            else:
                a = ops.linear_ln(ctx, L["w_o"], L["b_o"], residual=x, lnr=(st_x, xg, xb, D, eps))
            inter = ops.linear_ln(a, d["w_i"], act="gelu", lna=(None, d["cs_i"], d["b_i"], D, eps), out_stats=st_a)
            o = ops.linear_ln(inter, L["w_out"], L["b_out"], residual=a, lnr=(st_a, L["ln1_g"], L["ln1_b"], D, eps))
            x, xg, xb = o, L["ln2_g"], L["ln2_b"]
        if h is None:
            h = ops.layer_norm(x, xg, xb, eps) if xg is not None else x
            h = h.view(B, S, D)[:, 0, :]
        pooled = ops.linear(h, self.w_pool, self.b_pool, act="tanh")
        return ops.linear(pooled, self.w_cls, self.b_cls, out_dtype=torch.float32)

    def _forward_hip_pstats(self, ids: torch.Tensor) -> torch.Tensor:
        """Four kernels per layer, no LayerNorm kernel and no statistics work in
        any main loop (gemm_core.h EPI_STG): the o-projection and FFN-down write
        per-N-tile partial (sum, sum of squares) of their raw (pre-LayerNorm)
        rows from the row-major phase of their staged epilogues; FFN-up and the
        next layer's fused QKV+attention consume those raw rows with the
        LayerNorm folded into their weights and correct in their epilogues
        (rstd (x W'^T - mean colsum) + b'); the residual adds normalise their
        operand on load.  Layer 0 reads embed_ln's normalised rows directly."""
        c = self.cfg
        B, S = ids.shape
        D, H, eps = c.hidden, c.heads, c.eps
        Wd = self._deferred_weights()
        kid = (ids.contiguous(), c.pad_token_id) if ids.dtype == torch.int32 else None
        lens = None if kid is not None else ops.seq_lens(ids, c.pad_token_id)
        M = B * S
        n = len(self.layers)
        x = ops.embed_ln(ids, self.word, self.pos, self.typ, self.emb_g, self.emb_b, eps).reshape(M, D)
        xst = xg = xb = None       # x is raw (pre-LN2 of the previous layer) iff xst is not None
        h = None
        for i, L in enumerate(self.layers):
            d = Wd[i]
            if xst is None:
                ctx = ops.qkv_attention(x, d["wq"], d["bq"], B, S, H, lens=lens, key_ids=kid)
            else:
                ctx = ops.qkv_attention(x, d["wq"], None, B, S, H, lens=lens, key_ids=kid,
                                        lna=(d["csq"], d["bfq"], eps), a_stats=xst)
            if i == n - 1 and self.cls_only_last_layer:
                xc = x.view(B, S, D)[:, 0, :]
                hc = xc if xst is None else ops.layer_norm(xc, xg, xb, eps)
                a = ops.linear(ctx.view(B, S, D)[:, 0, :], L["w_o"], L["b_o"], residual=hc)
                h1 = ops.layer_norm(a, L["ln1_g"], L["ln1_b"], eps)
                inter = ops.linear(h1, L["w_i"], L["b_i"], act="gelu")
                o = ops.linear(inter, L["w_out"], L["b_out"], residual=h1)
                h = ops.layer_norm(o, L["ln2_g"], L["ln2_b"], eps)
                break
            lnr = None if xst is None else (xst, xg, xb, D, eps)
            a, ast = ops.linear_ln_staged(ctx, L["w_o"], L["b_o"], residual=x, lnr=lnr, pstats=True)
            inter = ops.linear_ln_staged(a, d["w_i"], act="gelu", lna=(ast, d["cs_i"], d["b_i"], D, eps))
            # its partials feed the next layer's fused QKV+attention (at most 8 per row)
            o, ost = ops.linear_ln_staged(inter, L["w_out"], L["b_out"], residual=a,
                                          lnr=(ast, L["ln1_g"], L["ln1_b"], D, eps), pstats=True, max_parts=8)
            x, xst, xg, xb = o, ost, L["ln2_g"], L["ln2_b"]
        if h is None:
            h = ops.layer_norm(x, xg, xb, eps) if xst is not None else x
            h = h.view(B, S, D)[:, 0, :]
        pooled = ops.linear(h, self.w_pool, self.b_pool, act="tanh")
        return ops.linear(pooled, self.w_cls, self.b_cls, out_dtype=torch.float32)

    def _forward_hip_folded(self, ids: torch.Tensor) -> torch.Tensor:
        """Post-LN BERT with every in-stack LayerNorm deferred into the GEMMs
        (ops.linear_ln): o-proj / FFN-down accumulate row statistics of what they
        store, FFN-up / next QKV consume the raw rows with gamma folded into their
        weights, and the residual adds normalise their operand on load."""
        c = self.cfg
        B, S = ids.shape
        D, H, eps = c.hidden, c.heads, c.eps
        Fw = self._folded_weights()
        lens = ops.seq_lens(ids, c.pad_token_id)
        M = B * S
        n = len(self.layers)
        stats = torch.empty(n, 2, M, 2, device=ids.device, dtype=torch.float32)   # zeroed by embed_ln
        x = ops.embed_ln(ids, self.word, self.pos, self.typ, self.emb_g, self.emb_b, eps, zero_stats=stats)
        xs = xg = xb = None        # x is raw (pre-LN2 of the previous layer) iff xs is not None
        h = None
        for i, L in enumerate(self.layers):
            if xs is None:
                qkv = ops.linear(x, L["w_qkv"], L["b_qkv"])
            else:
                qkv = ops.linear_ln(x, Fw[i]["w_qkv"], lna=(xs, Fw[i]["cs_qkv"], Fw[i]["b_qkv"], D, eps))
            ctx = ops.attention(qkv, B, S, H, H, D // H, lens=lens)
            if i == n - 1 and self.cls_only_last_layer:
                # CLS rows only (see _forward_hip): materialise their normalised
                # residual and finish on the plain kernels (B rows)
                xc = x.view(B, S, D)[:, 0, :]
                hc = xc if xs is None else ops.layer_norm(xc, xg, xb, eps)
                a = ops.linear(ctx.view(B, S, D)[:, 0, :], L["w_o"], L["b_o"], residual=hc)
                h1 = ops.layer_norm(a, L["ln1_g"], L["ln1_b"], eps)
                inter = ops.linear(h1, L["w_i"], L["b_i"], act="gelu")
                o = ops.linear(inter, L["w_out"], L["b_out"], residual=h1)
                h = ops.layer_norm(o, L["ln2_g"], L["ln2_b"], eps)
                break
            s_a, s_o = stats[i, 0], stats[i, 1]
            a = ops.linear_ln(ctx, L["w_o"], L["b_o"], residual=x,
                              lnr=None if xs is None else (xs, xg, xb, D, eps), out_stats=s_a)
            inter = ops.linear_ln(a, Fw[i]["w_i"], act="gelu", lna=(s_a, Fw[i]["cs_i"], Fw[i]["b_i"], D, eps))
            o = ops.linear_ln(inter, L["w_out"], L["b_out"], residual=a, lnr=(s_a, L["ln1_g"], L["ln1_b"], D, eps),
                              out_stats=s_o)
            x, xs, xg, xb = o, s_o, L["ln2_g"], L["ln2_b"]
        if h is None:
            h = ops.layer_norm(x, xg, xb, eps) if xs is not None else x
            h = h.view(B, S, D)[:, 0, :]
        pooled = ops.linear(h, self.w_pool, self.b_pool, act="tanh")
        return ops.linear(pooled, self.w_cls, self.b_cls, out_dtype=torch.float32)

    def _forward_torch(self, ids: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        B, S = ids.shape
        D, H = c.hidden, c.heads
        Dh = D // H
        idl = ids.long()
        mask = (idl != c.pad_token_id)
        x = self.word[idl] + self.pos[:S][None] + self.typ[0][None, None]
        h = F.layer_norm(x, (D,), self.emb_g, self.emb_b, c.eps)
        attn_mask = mask[:, None, None, :]
        for L in self.layers:
            qkv = F.linear(h, L["w_qkv"], L["b_qkv"])
            q, k, v = qkv.split(D, dim=-1)
            q = q.view(B, S, H, Dh).transpose(1, 2)
            k = k.view(B, S, H, Dh).transpose(1, 2)
            v = v.view(B, S, H, Dh).transpose(1, 2)
            ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask)
            ctx = ctx.transpose(1, 2).reshape(B, S, D)
            h1 = F.layer_norm(F.linear(ctx, L["w_o"], L["b_o"]) + h, (D,), L["ln1_g"], L["ln1_b"], c.eps)
            inter = F.gelu(F.linear(h1, L["w_i"], L["b_i"]))
            h = F.layer_norm(F.linear(inter, L["w_out"], L["b_out"]) + h1, (D,), L["ln2_g"], L["ln2_b"], c.eps)
        pooled = torch.tanh(F.linear(h[:, 0], self.w_pool, self.b_pool))
        return F.linear(pooled, self.w_cls, self.b_cls).float()

    def example_input(self, batch: int, seed: int = 0, device=None) -> torch.Tensor:
        g = torch.Generator(device="cpu").manual_seed(seed)
        ids = torch.randint(1, self.cfg.vocab_size, (batch, self.cfg.seq_len), generator=g, dtype=torch.int32)
        ids[:, 0] = 101  # [CLS]
        return ids.to(device or self.device)
