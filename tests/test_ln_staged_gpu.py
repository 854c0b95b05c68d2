"""LayerNorm folded into the GEMMs around it, on the STAGED epilogue with
per-N-tile partial statistics (gemm_core.h EPI_STG; ops.linear_ln_staged,
qkv_attention(a_stats=...), BertForSequenceClassification._forward_hip_pstats):
every mode and every tile the staged modes run, against fp32 references that
apply the LayerNorm explicitly, at M = 32, 4096 and 4097 (a ragged last tile).

Reference behaviour: the post-LN BertLayer (LayerNorm(x + sublayer(x))) of the
served models (SURVEY §2.7 BERT row)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from ray_dynamic_batching_amd import ops

    return ops


@pytest.fixture(autouse=True)
def _experimental_build():
    # the staged-LN modes are in the opt-in RDB_EXPERIMENTAL_KERNELS build (ops/csrc/common.h)
    if not _ops().experimental_kernels_built():
        pytest.skip("opt-in RDB_EXPERIMENTAL_KERNELS build not loaded")


def _ln(x, g, b, eps):
    xf = x.float()
    mu = xf.mean(-1, keepdim=True)
    var = xf.var(-1, unbiased=False, keepdim=True)
    return (xf - mu) * torch.rsqrt(var + eps) * g.float() + b.float()


def _close(a, b, rtol, atol):
    a, b = a.float(), b.float()
    err = ((a - b).abs() - atol - rtol * b.abs()).max().item()
    assert err <= 0, f"max excess error {err} (max abs diff {(a - b).abs().max().item()})"


def _data(M, N, K, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)

    def r(*shape, s=1.0, mean=0.0):
        return (torch.randn(*shape, generator=g) * s + mean).to("cuda", torch.bfloat16)

    return dict(x=r(M, K, mean=0.3), w=r(N, K, s=0.03), b=r(N, s=0.1), res=r(M, N, s=2.0, mean=-0.5),
                g=(1 + 0.1 * torch.randn(N, generator=g)).to("cuda", torch.bfloat16), be=r(N, s=0.1))


@pytest.mark.parametrize("M", [32, 4096, 4097])
def test_linear_ln_staged_modes_every_tile(M):
    ops = _ops()
    N, K, eps = 768, 768, 1e-12
    d = _data(M, N, K, seed=M)
    for cfg in ops.STG_TILE_CFGS:
        # producer: y = x W^T + b + R, partial row statistics of the stored y
        y, st = ops.linear_ln_staged(d["x"], d["w"], d["b"], residual=d["res"], pstats=True, tile_cfg=cfg)
        ref = d["x"].float() @ d["w"].float().t() + d["b"].float() + d["res"].float()
        _close(y, ref, 2e-2, 2e-2)
        P = st.shape[1]
        assert P == -(-N // ops._ops().gemm_tile_bn(ops._ops().gemm_stg_cfg(cfg)))
        yf = y.float()
        _close(st.sum(1)[:, 0], yf.sum(1), 1e-3, 1e-2)
        _close(st.sum(1)[:, 1], (yf * yf).sum(1), 1e-3, 1e-1)
        # LNR + stats: y2 = x W^T + b + LN(y) (normalised on load)
        y2, st2 = ops.linear_ln_staged(d["x"], d["w"], d["b"], residual=y, lnr=(st, d["g"], d["be"], N, eps),
                                       pstats=True, tile_cfg=cfg)
        ref2 = d["x"].float() @ d["w"].float().t() + d["b"].float() + _ln(y, d["g"], d["be"], eps)
        _close(y2, ref2, 2e-2, 3e-2)
        _close(st2.sum(1)[:, 0], y2.float().sum(1), 1e-3, 1e-2)
        # LNR without stats out
        y3 = ops.linear_ln_staged(d["x"], d["w"], d["b"], residual=y, lnr=(st, d["g"], d["be"], N, eps), tile_cfg=cfg)
        _close(y3, ref2, 2e-2, 3e-2)
        # LNA: gelu(LN(y) W^T + b) on the raw y, the LayerNorm folded into the weight
        wf, cs, bf = ops.fold_ln_weights(d["w"], d["b"], d["g"], d["be"])
        z = ops.linear_ln_staged(y, wf, act="gelu", lna=(st, cs, bf, N, eps), tile_cfg=cfg)
        refz = torch.nn.functional.gelu(_ln(y, d["g"], d["be"], eps) @ d["w"].float().t() + d["b"].float())
        _close(z, refz, 3e-2, 3e-2)


def test_qkv_attention_with_partial_statistics():
    """The fused QKV+attention on raw rows whose LayerNorm is folded into its
    weight, statistics given as a producer's partials (no in-loop statistics)."""
    ops = _ops()
    B, S, H, D, eps = 8, 128, 12, 768, 1e-12
    d = _data(B * S, D, D, seed=5)
    x, st = ops.linear_ln_staged(d["x"], d["w"], d["b"], residual=d["res"], pstats=True, max_parts=8)
    assert st.shape[1] <= 8
    g = torch.Generator(device="cpu").manual_seed(9)
    wq = (torch.randn(3 * D, D, generator=g) * 0.03).to("cuda", torch.bfloat16)
    bq = (torch.randn(3 * D, generator=g) * 0.1).to("cuda", torch.bfloat16)
    w2, cs, bf = ops.fold_ln_weights(wq, bq, d["g"], d["be"])
    wp, bfp = ops.pack_qkv_heads(w2, bf, H)
    ctx = ops.qkv_attention(x, wp, None, B, S, H, lna=(ops.pack_qkv_vec(cs, H), bfp, eps), a_stats=st)
    hn = _ln(x, d["g"], d["be"], eps).to(torch.bfloat16)
    ref = ops.qkv_attention_ref(hn, wq, bq, B, S, H)
    _close(ctx, ref, 3e-2, 3e-2)


@pytest.mark.parametrize("B,S", [(1, 128), (32, 128), (241, 17)])
def test_bert_pstats_forward_matches_fp32_anchor(B, S):
    """Whole BERT forward without any in-stack LayerNorm kernel against the fp32
    PyTorch path of the same weights (M = B*S = 128, 4096, 4097)."""
    from ray_dynamic_batching_amd.models.bert import BertConfig, BertForSequenceClassification
    from ray_dynamic_batching_amd.models.reference import eager_reference, fp32_reference, parity_bound, rel_err

    m = BertForSequenceClassification(BertConfig(layers=4, seq_len=S), device="cuda", backend="hip", seed=1)
    m.ln_pstats = True
    ids = m.example_input(B, seed=2)
    ids[-1, S // 2:] = 0                      # a padded sequence
    out = m(ids)
    ref = fp32_reference(m)(ids)
    bound = parity_bound(rel_err(eager_reference(m)(ids), ref))
    err = rel_err(out, ref)
    assert err <= bound, (err, bound)
    m.ln_pstats = False
    assert rel_err(m(ids), out) <= 2 * bound
