"""Numerics of every HIP kernel against a plain-PyTorch fp32 reference (GPU)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from ray_dynamic_batching_amd import ops

    return ops


def _close(a, b, atol, rtol):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} / {a.numel()} elements out of tolerance; max err {err.max().item():.4g}"


def _need_experimental(ops):
    """Kernels that lost their A/Bs live in the opt-in RDB_EXPERIMENTAL_KERNELS
    build (ops/csrc/common.h); the default library's entry points throw."""
    if not ops.experimental_kernels_built():
        pytest.skip("opt-in RDB_EXPERIMENTAL_KERNELS build not loaded")


@pytest.mark.parametrize("M,N,K", [(4096, 768, 768), (4096, 2304, 768), (512, 3072, 768), (256, 768, 3072),
                                   (128, 768, 768), (7, 1000, 2048), (33, 40, 72), (1, 2, 768)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_linear_plain(M, N, K, dtype):
    ops = _ops()
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=dtype)
    w = torch.randn(N, K, device="cuda", dtype=dtype) * (K ** -0.5)
    y = ops.linear(x, w)
    _close(y, ops.linear_ref(x, w), 2e-2, 2e-2)


@pytest.mark.parametrize("cfg", list(range(30)))
def test_linear_tile_configs_asymmetric(cfg):
    """A = I with an asymmetric W catches a transposed C-write (guide §3)."""
    ops = _ops()
    M = K = 384
    N = 320
    x = torch.eye(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.arange(N * K, device="cuda").reshape(N, K) % 97).to(torch.bfloat16)
    y = ops.linear(x, w, tile_cfg=cfg)
    _close(y, w.t().contiguous(), 0, 0)


@pytest.mark.parametrize("act", ["gelu", "relu", "tanh", "silu", "gelu_tanh"])
def test_linear_epilogues(act):
    ops = _ops()
    torch.manual_seed(1)
    x = torch.randn(512, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(1024, 768, device="cuda", dtype=torch.bfloat16) * 0.03
    b = torch.randn(1024, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16)
    _close(ops.linear(x, w, b, act=act), ops.linear_ref(x, w, b, act=act), 3e-2, 2e-2)
    _close(ops.linear(x, w, b, residual=r), ops.linear_ref(x, w, b, residual=r), 3e-2, 2e-2)


def test_linear_swiglu_and_f32_out():
    ops = _ops()
    torch.manual_seed(2)
    x = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(1024, 512, device="cuda", dtype=torch.bfloat16) * 0.05
    _close(ops.linear(x, w, act="swiglu"), ops.linear_ref(x, w, act="swiglu"), 3e-2, 3e-2)
    y = ops.linear(x, w, out_dtype=torch.float32)
    assert y.dtype == torch.float32
    _close(y, ops.linear_ref(x, w, out_dtype=torch.float32), 1e-2, 1e-2)


def test_linear_strided_rows():
    """Pooler path: CLS rows of [B, S, D] as a row-strided view."""
    ops = _ops()
    h = torch.randn(8, 128, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(768, 768, device="cuda", dtype=torch.bfloat16) * 0.03
    cls = h[:, 0, :]
    _close(ops.linear(cls, w, act="tanh"), ops.linear_ref(cls.contiguous(), w, act="tanh"), 2e-2, 2e-2)


@pytest.mark.parametrize("D", [768, 1024, 4096, 320])
def test_norms(D):
    ops = _ops()
    torch.manual_seed(3)
    x = torch.randn(300, D, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(300, D, device="cuda", dtype=torch.bfloat16)
    g = torch.rand(D, device="cuda", dtype=torch.bfloat16) + 0.5
    b = torch.randn(D, device="cuda", dtype=torch.bfloat16)
    _close(ops.layer_norm(x, g, b), ops.layer_norm_ref(x, g, b), 3e-2, 2e-2)
    ro = torch.empty_like(x)
    _close(ops.layer_norm(x, g, b, residual=r, residual_out=ro), ops.layer_norm_ref(x, g, b, residual=r), 3e-2, 2e-2)
    _close(ro, x.float() + r.float(), 2e-2, 1e-2)
    _close(ops.rms_norm(x, g, 1e-5), ops.rms_norm_ref(x, g, 1e-5), 3e-2, 2e-2)


def test_embed_ln():
    ops = _ops()
    torch.manual_seed(4)
    V, D, S = 30522, 768, 128
    word = torch.randn(V, D, device="cuda", dtype=torch.bfloat16)
    pos = torch.randn(512, D, device="cuda", dtype=torch.bfloat16)
    typ = torch.randn(2, D, device="cuda", dtype=torch.bfloat16)
    g = torch.rand(D, device="cuda", dtype=torch.bfloat16) + 0.5
    b = torch.randn(D, device="cuda", dtype=torch.bfloat16)
    ids = torch.randint(0, V, (4, S), device="cuda", dtype=torch.int32)
    _close(ops.embed_ln(ids, word, pos, typ, g, b), ops.embed_ln_ref(ids, word, pos, typ, g, b), 3e-2, 2e-2)
    # token types, an odd token count (partial last block), both kernel forms: the 16-B
    # half-wave one (aligned tables) and the 8-B one (a table 8-B but not 16-B aligned)
    ids = torch.randint(0, V, (3, 37), device="cuda", dtype=torch.int32)
    types = torch.randint(0, 2, (3, 37), device="cuda", dtype=torch.int32)
    ref = ops.embed_ln_ref(ids, word, pos, typ, g, b, types=types)
    _close(ops.embed_ln(ids, word, pos, typ, g, b, types=types), ref, 3e-2, 2e-2)
    pos8 = torch.empty(512 * D + 4, device="cuda", dtype=torch.bfloat16)[4:].view(512, D)
    pos8.copy_(pos)
    assert pos8.data_ptr() % 16 == 8
    _close(ops.embed_ln(ids, word, pos8, typ, g, b, types=types), ref, 3e-2, 2e-2)


@pytest.mark.parametrize("B,S,H,Hkv,D,causal,use_lens", [
    (4, 128, 12, 12, 64, False, False),
    (3, 128, 12, 12, 64, False, True),
    (2, 100, 4, 4, 64, False, True),
    (2, 256, 8, 2, 128, True, False),
    (1, 200, 4, 1, 128, True, False),
    (2, 300, 4, 4, 64, False, True),
])
def test_attention(B, S, H, Hkv, D, causal, use_lens):
    ops = _ops()
    torch.manual_seed(5)
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    lens = None
    if use_lens:
        lens = torch.randint(1, S + 1, (B,), device="cuda", dtype=torch.int32)
        lens[0] = S
    y = ops.attention(qkv, B, S, H, Hkv, D, lens=lens, causal=causal)
    ref = ops.attention_ref(qkv, B, S, H, Hkv, D, lens=lens, causal=causal)
    _close(y, ref, 2e-2, 2e-2)


def test_attention_spike_rescale():
    """Force the online-softmax rescale branch: a key block late in the sequence
    dominates one query (guide rule 26)."""
    ops = _ops()
    B, S, H, D = 1, 384, 2, 64
    qkv = torch.randn(B * S, 3 * H * D, device="cuda", dtype=torch.bfloat16) * 0.1
    qkv[5, 0:D] = 3.0            # query 5, head 0
    qkv[300, H * D:H * D + D] = 3.0  # key 300 (third key block), head 0
    _close(ops.attention(qkv, B, S, H, H, D), ops.attention_ref(qkv, B, S, H, H, D), 2e-2, 2e-2)


@pytest.mark.parametrize("B,S,H,K", [(4, 128, 12, 768), (5, 128, 2, 256), (3, 100, 4, 256), (2, 64, 2, 136),
                                     (1, 1, 1, 64)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_qkv_attention(B, S, H, K, cfg, dtype):
    """Fused projection + attention (qkv_attention.hip) == GEMM -> attention in fp32,
    with padding lengths, every block-shape config, S < 128 (the 128-row tile
    reaches into the next sequence / past the last row) and K not a multiple of 64."""
    ops = _ops()
    torch.manual_seed(11)
    x = torch.randn(B * S, K, device="cuda", dtype=dtype)
    w = torch.randn(3 * H * 64, K, device="cuda", dtype=dtype) * (K ** -0.5)
    b = torch.randn(3 * H * 64, device="cuda", dtype=dtype) * 0.1
    lens = torch.randint(1, S + 1, (B,), device="cuda", dtype=torch.int32)
    lens[0] = S
    wp, bp = ops.pack_qkv_heads(w, b, H)
    for ln in (None, lens):
        y = ops.qkv_attention(x, wp, bp, B, S, H, lens=ln, cfg=cfg)
        ref = ops.qkv_attention_ref(x, w, b, B, S, H, lens=ln)
        _close(y, ref, 2e-2, 2e-2)
    # key lengths counted in-kernel from right-padded token ids (pad id 7): same result, bit for bit
    ids = torch.randint(8, 1000, (B, S), device="cuda", dtype=torch.int32)
    for i in range(B):
        ids[i, int(lens[i]):] = 7
    y_ids = ops.qkv_attention(x, wp, bp, B, S, H, cfg=cfg, key_ids=(ids, 7))
    assert torch.equal(ops.seq_lens(ids, 7), lens.clamp(min=1))
    assert torch.equal(y_ids, ops.qkv_attention(x, wp, bp, B, S, H, lens=lens, cfg=cfg))


def test_qkv_attention_matches_two_kernel_path():
    """The fused kernel against OUR unfused kernels (ops.linear -> ops.attention)
    at the BERT-base shape, row-strided input included."""
    ops = _ops()
    torch.manual_seed(12)
    B, S, H, D = 8, 128, 12, 768
    big = torch.randn(B * S, D + 64, device="cuda", dtype=torch.bfloat16)
    x = big[:, :D]                                      # row stride D + 64
    w = torch.randn(3 * D, D, device="cuda", dtype=torch.bfloat16) * 0.03
    b = torch.randn(3 * D, device="cuda", dtype=torch.bfloat16) * 0.1
    wp, bp = ops.pack_qkv_heads(w, b, H)
    y = ops.qkv_attention(x, wp, bp, B, S, H)
    two = ops.attention(ops.linear(x, w, b), B, S, H, H, 64)
    _close(y, two, 2e-2, 2e-2)


@pytest.mark.parametrize("C,k", [(1000, 5), (999, 5), (10, 1), (257, 16), (4096, 3), (1000, 1)])
def test_softmax_topk(C, k):
    """wave-per-row kernel (float4 lanes when C % 4 == 0, element loads otherwise)
    against the fp32 reference, including the tie rule (lowest index first)."""
    ops = _ops()
    torch.manual_seed(6)
    x = torch.randn(37, C, device="cuda")
    p, i = ops.softmax_topk(x, k)
    pr, ir = ops.softmax_topk_ref(x, k)
    assert torch.equal(i, ir)
    _close(p, pr, 1e-5, 1e-4)
    packed = ops.softmax_topk_packed(x, k)          # the serving row [k probs | k ids as f32]
    assert packed.shape == (37, 2 * k)
    assert torch.equal(packed[:, :k], p) and torch.equal(packed[:, k:], i.float())
    # ties: small integers, many equal maxima -> lowest column wins, like torch.topk on sorted ties
    xt = torch.randint(0, 3, (8, C), device="cuda").float()
    pt, it = ops.softmax_topk(xt, k)
    mx = xt.max(dim=1, keepdim=True).values
    first = torch.stack([torch.nonzero(xt[r] == mx[r]).flatten()[0] for r in range(8)])
    assert torch.equal(it[:, 0].long(), first)


def test_rope():
    ops = _ops()
    torch.manual_seed(7)
    B, S, H, Hkv, D = 2, 64, 8, 2, 128
    cos, sin = ops.rope_tables(4096, D, device="cuda")
    qkv = torch.randn(B * S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    ref = ops.rope_ref(qkv, cos, sin, B, S, H, Hkv, D)
    ops.rope_(qkv, cos, sin, B, S, H, Hkv, D)
    _close(qkv, ref, 2e-2, 2e-2)


@pytest.mark.parametrize("N,H,C,K,R,stride,pad", [
    (2, 56, 64, 64, 3, 1, 1), (2, 56, 64, 256, 1, 1, 0), (2, 56, 256, 128, 1, 2, 0),
    (1, 224, 8, 64, 7, 2, 3), (3, 14, 256, 256, 3, 2, 1), (2, 7, 512, 2048, 1, 1, 0)])
def test_conv2d(N, H, C, K, R, stride, pad):
    ops = _ops()
    torch.manual_seed(8)
    x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
    w = torch.randn(K, R, R, C, device="cuda", dtype=torch.float16) * (R * R * C) ** -0.5
    b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
    y = ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu")
    _close(y, ops.conv2d_nhwc_ref(x, w, b, stride=stride, pad=pad, act="relu"), 2e-2, 2e-2)
    r = torch.randn_like(y)
    y2 = ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", residual=r)
    _close(y2, ops.conv2d_nhwc_ref(x, w, b, stride=stride, pad=pad, act="relu", residual=r), 2e-2, 2e-2)


@pytest.mark.parametrize("N,H,C,K,R,stride,pad", [
    (32, 7, 512, 512, 3, 1, 1), (32, 14, 256, 256, 3, 1, 1), (4, 14, 1024, 256, 1, 1, 0),
    (2, 28, 128, 128, 3, 2, 1), (3, 7, 2048, 512, 1, 1, 0)])
def test_conv2d_splitk(N, H, C, K, R, stride, pad):
    """Split-K convolutions (tile | splits << 8; last-arriver hand-off) on one
    shared workspace, back to back: every result matches the fp32 reference and
    the workspace's tile counters are zero again afterwards."""
    ops = _ops()
    torch.manual_seed(11)
    x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
    w = torch.randn(K, R, R, C, device="cuda", dtype=torch.float16) * (R * R * C) ** -0.5
    b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
    ref = ops.conv2d_nhwc_ref(x, w, b, stride=stride, pad=pad, act="relu")
    r = torch.randn_like(ref)
    ref_r = ops.conv2d_nhwc_ref(x, w, b, stride=stride, pad=pad, act="relu", residual=r)
    ws = ops.splitk_workspace("cuda")
    nk = -(-(R * R * C) // 64)
    for cfg in (0, 3, 9, 12):
        for sp in (2, 3, 8):
            if -(-nk // -(-nk // sp)) < 2:
                continue
            c = cfg | (sp << 8)
            _close(ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", tile_cfg=c, workspace=ws), ref, 2e-2, 2e-2)
            _close(ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", residual=r, tile_cfg=c, workspace=ws),
                   ref_r, 2e-2, 2e-2)
    # DEEP tiles (one block per CU, up to 8 LDS stages), alone and split
    for c in (0 | ops.DEEP, 1 | ops.DEEP, 10 | ops.DEEP, 3 | (2 << 8) | ops.DEEP, 0 | (3 << 8) | ops.DEEP):
        if (c >> 8) & 15 and -(-nk // -(-nk // ((c >> 8) & 15))) < 2:
            continue
        _close(ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", residual=r, tile_cfg=c, workspace=ws),
               ref_r, 2e-2, 2e-2)
    # without a workspace: a private one
    _close(ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", tile_cfg=0 | (2 << 8)), ref, 2e-2, 2e-2)
    torch.cuda.synchronize()
    assert int(ws[:ops.SPLITK_HEADER].view(torch.int32).abs().sum()) == 0
    if R == 1 and stride == 1:
        for c in (0, 10, 19, 23):
            _close(ops.conv2d_nhwc(x, w, b, act="relu", residual=r, tile_cfg=ops.CONV_LINEAR | c), ref_r, 2e-2, 2e-2)


@pytest.mark.parametrize("N,H,C,K,R,stride,pad", [
    (2, 56, 64, 64, 3, 1, 1), (32, 7, 512, 512, 3, 1, 1), (4, 28, 128, 128, 3, 2, 1), (3, 14, 256, 256, 3, 2, 1),
    (2, 56, 256, 128, 1, 2, 0), (2, 15, 96, 40, 3, 1, 1)])
def test_conv2d_pingpong(N, H, C, K, R, stride, pad):
    """The 8-wave ping-pong kernel with the im2col operand (CONV_PP | v [| splits
    << 8]): every tile whose BK divides C, with and without residual, unsplit and
    split-K on one shared workspace (counters back to zero), ragged M / N edges."""
    ops = _ops()
    torch.manual_seed(13 + H)
    x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
    w = torch.randn(K, R, R, C, device="cuda", dtype=torch.float16) * (R * R * C) ** -0.5
    b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
    ref = ops.conv2d_nhwc_ref(x, w, b, stride=stride, pad=pad, act="relu")
    r = torch.randn_like(ref)
    ref_r = ops.conv2d_nhwc_ref(x, w, b, stride=stride, pad=pad, act="relu", residual=r)
    ws = ops.splitk_workspace("cuda")
    ran = 0
    for v in range(len(ops._CONV_PP_BM)):
        if C % ops._CONV_PP_BK[v]:
            continue
        nk = R * R * C // ops._CONV_PP_BK[v]
        for sp in (0, 2, 5):
            if sp and -(-nk // -(-nk // sp)) < 2:
                continue
            c = ops.CONV_PP | v | (sp << 8)
            _close(ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", tile_cfg=c, workspace=ws), ref, 2e-2, 2e-2)
            _close(ops.conv2d_nhwc(x, w, b, stride=stride, pad=pad, act="relu", residual=r, tile_cfg=c, workspace=ws),
                   ref_r, 2e-2, 2e-2)
            ran += 1
    assert ran >= 2
    torch.cuda.synchronize()
    assert int(ws[:ops.SPLITK_HEADER].view(torch.int32).abs().sum()) == 0


@pytest.mark.parametrize("N,H,C,K", [
    (2, 56, 64, 64), (3, 28, 128, 128), (3, 14, 256, 256), (5, 7, 512, 512), (3, 14, 128, 72), (2, 12, 64, 200),
    (32, 56, 64, 64), (32, 28, 128, 128), (32, 14, 256, 256), (32, 7, 512, 512)])
def test_conv2d_halo(N, H, C, K):
    """The halo-tile 3x3 kernel (CONV_HALO | v): every tile whose rows fit the
    image, against the fp32 reference with and without a residual; odd image
    counts (a tile of G images past the batch end), ragged output channels."""
    ops = _ops()
    torch.manual_seed(17 + H + K)
    x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
    w = torch.randn(K, 3, 3, C, device="cuda", dtype=torch.float16) * (9 * C) ** -0.5
    b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
    ref = ops.conv2d_nhwc_ref(x, w, b, pad=1, act="relu")
    r = torch.randn_like(ref)
    ref_r = ops.conv2d_nhwc_ref(x, w, b, pad=1, act="relu", residual=r)
    cands = ops.conv_halo_candidates(N, H, H, C, K, 3, 3, 1, 1, H, H, True)
    assert cands
    ws = ops.splitk_workspace("cuda")
    for c in cands:
        _close(ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=c), ref, 2e-2, 2e-2)
        if ops.splits_of(c) > 1:       # split-K on a shared workspace: the tile counters end at zero
            _close(ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=c, workspace=ws), ref, 2e-2, 2e-2)
            _close(ops.conv2d_nhwc(x, w, b, pad=1, act="relu", residual=r, tile_cfg=c, workspace=ws), ref_r, 2e-2, 2e-2)
            torch.cuda.synchronize()
            assert int(ws[:ops.SPLITK_HEADER].view(torch.int32).abs().sum()) == 0
            continue
        if (c & 255) in ops._CONV_HALO_RW:       # resident-weight tiles: no residual epilogue
            with pytest.raises(Exception):
                ops.conv2d_nhwc(x, w, b, pad=1, act="relu", residual=r, tile_cfg=c)
            continue
        _close(ops.conv2d_nhwc(x, w, b, pad=1, act="relu", residual=r, tile_cfg=c), ref_r, 2e-2, 2e-2)
    with pytest.raises(Exception):       # pad 0 is not a halo shape
        ops.conv2d_nhwc(x, w, b, stride=1, pad=0, tile_cfg=ops.CONV_HALO | 0)


@pytest.mark.parametrize("N,H,C,K", [(2, 56, 128, 128), (3, 28, 256, 256), (5, 14, 512, 512), (32, 56, 128, 128),
                                     (32, 14, 512, 512), (2, 15, 64, 72)])
def test_conv2d_halo_stride2(N, H, C, K):
    """The halo tiles at stride 2 (pad 1): patch rows 2p + r, columns 2q + s; the last
    row block of an image may be partial (odd sizes); split-K candidates on a shared
    workspace leave its counters at zero."""
    ops = _ops()
    torch.manual_seed(23 + H + K)
    x = torch.randn(N, H, H, C, device="cuda", dtype=torch.float16)
    w = torch.randn(K, 3, 3, C, device="cuda", dtype=torch.float16) * (9 * C) ** -0.5
    b = torch.randn(K, device="cuda", dtype=torch.float16) * 0.1
    ref = ops.conv2d_nhwc_ref(x, w, b, stride=2, pad=1, act="relu")
    r = torch.randn_like(ref)
    ref_r = ops.conv2d_nhwc_ref(x, w, b, stride=2, pad=1, act="relu", residual=r)
    P = (H - 1) // 2 + 1
    cands = ops.conv_halo_candidates(N, H, H, C, K, 3, 3, 2, 1, P, P, True)
    assert cands and all((c & 255) not in ops._CONV_HALO_RW for c in cands)
    ws = ops.splitk_workspace("cuda")
    for c in cands:
        _close(ops.conv2d_nhwc(x, w, b, stride=2, pad=1, act="relu", tile_cfg=c, workspace=ws), ref, 2e-2, 2e-2)
        _close(ops.conv2d_nhwc(x, w, b, stride=2, pad=1, act="relu", residual=r, tile_cfg=c, workspace=ws), ref_r,
               2e-2, 2e-2)
    torch.cuda.synchronize()
    assert int(ws[:ops.SPLITK_HEADER].view(torch.int32).abs().sum()) == 0


def test_conv2d_pingpong_splitk_graph_replay():
    """A split-K ping-pong conv chain captured in a graph (per-forward workspace,
    as ResNet50._logits_hip), replayed with new inputs."""
    ops = _ops()
    torch.manual_seed(14)
    x = torch.randn(32, 14, 14, 256, device="cuda", dtype=torch.float16)
    w = torch.randn(256, 3, 3, 256, device="cuda", dtype=torch.float16) * (9 * 256) ** -0.5
    b = torch.randn(256, device="cuda", dtype=torch.float16) * 0.1

    def fwd():
        ws = ops.splitk_workspace("cuda")
        h = ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=ops.CONV_PP | 0 | (4 << 8), workspace=ws)
        return ops.conv2d_nhwc(h, w, b, pad=1, act="relu", tile_cfg=ops.CONV_PP | 2 | (6 << 8), workspace=ws)

    def ref():
        h = ops.conv2d_nhwc_ref(x, w, b, pad=1, act="relu")
        return ops.conv2d_nhwc_ref(h, w, b, pad=1, act="relu")

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fwd()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            y = fwd()
    torch.cuda.synchronize()
    for _ in range(2):
        x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        _close(y, ref(), 3e-2, 3e-2)


@pytest.mark.parametrize("M,N,K", [(4096, 768, 768), (512, 768, 3072), (1000, 520, 1160)])
def test_linear_deep_tiles(M, N, K):
    """The DEEP 4-wave tiles (kStages up to 8, one block per CU; K tails and
    ragged M / N edges included) against the fp32 reference."""
    ops = _ops()
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    ref = torch.nn.functional.gelu(x.float() @ w.float().t() + b.float())
    ref_r = x.float() @ w.float().t() + b.float() + r.float()
    for c in (0, 1, 2, 3, 9, 10, 6, 7):
        _close(ops.linear(x, w, b, act="gelu", tile_cfg=c | ops.DEEP), ref, 2e-2, 2e-2)
        _close(ops.linear(x, w, b, residual=r, tile_cfg=c | ops.DEEP), ref_r, 2e-2, 2e-2)


@pytest.mark.parametrize("M,N,K", [(128, 4096, 14336), (256, 1000, 2056), (300, 768, 3072)])
def test_linear_splitk(M, N, K):
    """Split-K on the dense GEMM (tile | splits << 8): with a caller workspace,
    with a private one, and captured in a graph (the private workspace lives in
    the graph's pool) -- against the fp32 reference, ragged M / N / K tails."""
    ops = _ops()
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    ref = x.float() @ w.float().t() + b.float() + r.float()
    ref_g = torch.nn.functional.gelu(x.float() @ w.float().t() + b.float())
    ws = ops.splitk_workspace("cuda")
    for c in (0, 1, 3, 9, 12, 19, 21):       # 19 / 21: the ping-pong tiles' split-K instantiations
        for sp in (2, 4, 8):
            cfg = c | (sp << 8)
            _close(ops.linear(x, w, b, residual=r, tile_cfg=cfg, workspace=ws), ref, 2e-2, 2e-2)
            _close(ops.linear(x, w, b, act="gelu", tile_cfg=cfg), ref_g, 2e-2, 2e-2)
    torch.cuda.synchronize()
    assert int(ws[:ops.SPLITK_HEADER].view(torch.int32).abs().sum()) == 0
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.linear(x, w, b, residual=r, tile_cfg=0 | (4 << 8))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            y = ops.linear(x, w, b, residual=r, tile_cfg=0 | (4 << 8))
    torch.cuda.synchronize()
    for _ in range(2):
        x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        _close(y, x.float() @ w.float().t() + b.float() + r.float(), 2e-2, 2e-2)


def test_linear_splitk_capture_workspace():
    """``capture_splitk_workspace``: every split-K launch of a capture (no caller
    workspace) uses the installed workspace -- no memset node per launch, the
    engine's per-compute-stream workspace -- chained outputs are right on every
    replay and the counters are back to zero; outside the block the private
    per-launch behaviour is unchanged."""
    ops = _ops()
    torch.manual_seed(5)
    M, N, K = 512, 768, 3072
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    ws_ = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5 for _ in range(3)]
    w2 = torch.randn(K, N, device="cuda", dtype=torch.bfloat16) * N ** -0.5
    cws = ops.splitk_workspace("cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side), ops.capture_splitk_workspace(cws):
            assert ops._private_splitk_ws(x.device, 1 << 20) is cws
            ys = []
            h = x
            for w in ws_:
                y = ops.linear(h, w, tile_cfg=19 | (2 << 8))           # split-K, no caller workspace
                ys.append(y)
                h = ops.linear(y, w2, tile_cfg=19 | (2 << 8))          # back to K wide, split-K again
        assert getattr(ops._cap_ws_local, "ws", None) is None
    torch.cuda.synchronize()
    for _ in range(3):
        x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        h = x.float()
        for w, y in zip(ws_, ys):
            _close(y, h @ w.float().t(), 3e-2, 3e-2)
            h = y.float() @ w2.float().t()
        assert int(cws[:ops.SPLITK_HEADER].view(torch.int32).abs().sum()) == 0


def test_linear_splitk_private_workspace_per_graph():
    """Split-K without a caller workspace inside graph capture: each graph gets
    its own (graph-pool) workspace, so two graphs captured on ONE stream and
    replayed concurrently on two streams do not share counters / partials, and
    capturing again after the graphs are gone works (no cached pool tensor)."""
    ops = _ops()
    torch.manual_seed(21)
    M, N, K = 1024, 4096, 4096
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
    xs = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
    for rnd in range(2):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        gs, ys = [], []
        with torch.cuda.stream(side):
            for i in range(2):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=torch.cuda.graph_pool_handle(), stream=side):
                    ys.append(ops.linear(xs[i], w, b, tile_cfg=19 | (2 << 8)))
                gs.append(g)
        torch.cuda.synchronize()
        sts = [torch.cuda.Stream() for _ in range(2)]
        for _ in range(3):
            for g, st in zip(gs, sts):
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    g.replay()
            torch.cuda.synchronize()
            for i in range(2):
                _close(ys[i], xs[i].float() @ w.float().t() + b.float(), 2e-2, 2e-2)
        del gs, ys


def test_conv2d_splitk_graph_replay():
    """Split-K inside a captured graph with the per-forward workspace idiom of
    ResNet50._logits_hip, replayed with new inputs."""
    ops = _ops()
    torch.manual_seed(12)
    x = torch.randn(32, 7, 7, 512, device="cuda", dtype=torch.float16)
    w = torch.randn(512, 3, 3, 512, device="cuda", dtype=torch.float16) * (9 * 512) ** -0.5
    b = torch.randn(512, device="cuda", dtype=torch.float16) * 0.1

    def fwd():
        ws = ops.splitk_workspace("cuda")
        h = ops.conv2d_nhwc(x, w, b, pad=1, act="relu", tile_cfg=0 | (4 << 8), workspace=ws)
        return ops.conv2d_nhwc(h, w, b, pad=1, act="relu", tile_cfg=9 | (3 << 8), workspace=ws)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fwd()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            y = fwd()
    torch.cuda.synchronize()
    for it in range(3):
        x.copy_(torch.randn_like(x))
        g.replay()
        torch.cuda.synchronize()
        h = ops.conv2d_nhwc_ref(x, w, b, pad=1, act="relu")
        _close(y, ops.conv2d_nhwc_ref(h, w, b, pad=1, act="relu"), 3e-2, 3e-2)


def test_pools_and_dwconv():
    ops = _ops()
    torch.manual_seed(9)
    x = torch.randn(2, 112, 112, 64, device="cuda", dtype=torch.float16)
    _close(ops.maxpool_nhwc(x), ops.maxpool_nhwc_ref(x), 0, 0)
    _close(ops.avgpool_nhwc(x), ops.avgpool_nhwc_ref(x), 1e-3, 1e-2)
    w = torch.randn(3, 3, 64, device="cuda", dtype=torch.float16) * 0.3
    b = torch.randn(64, device="cuda", dtype=torch.float16) * 0.1
    for stride in (1, 2):
        _close(ops.dwconv_nhwc(x, w, b, stride=stride, pad=1, act="silu"),
               ops.dwconv_nhwc_ref(x, w, b, stride=stride, pad=1, act="silu"), 2e-2, 2e-2)


@pytest.mark.parametrize("N,HW,C", [(32, 49, 2048), (3, 1, 8), (2, 17, 264), (1, 196, 1024)])
def test_avgpool_shapes(N, HW, C):
    ops = _ops()
    torch.manual_seed(N + HW)
    x = torch.randn(N, HW, 1, C, device="cuda", dtype=torch.float16)
    _close(ops.avgpool_nhwc(x), ops.avgpool_nhwc_ref(x), 1e-3, 1e-2)


def test_image_to_s2d_and_space_to_depth_stem():
    """u8 image -> space-to-depth f16, and the 4x4 stride-1 stem conv on it (out
    cut to 112 x 112) against the 7x7 stride-2 conv of the channel-padded image."""
    ops = _ops()
    img = torch.randint(0, 256, (3, 224, 224, 3), device="cuda", dtype=torch.uint8)
    ws = ops.splitk_workspace("cuda", zeroed=False)
    ws[:ops.SPLITK_HEADER].fill_(0xFF)
    xs = ops.image_to_s2d(img, zero=ws)             # the side job zeroes the split-K counters
    _close(xs, ops.image_to_s2d_ref(img), 1e-2, 1e-2)
    assert int(ws[:ops.SPLITK_HEADER].sum()) == 0
    img2 = torch.randint(0, 256, (2, 36, 20, 3), device="cuda", dtype=torch.uint8)   # a small odd-shaped batch
    _close(ops.image_to_s2d(img2), ops.image_to_s2d_ref(img2), 1e-2, 1e-2)
    g = torch.Generator().manual_seed(3)
    w = torch.zeros(64, 7, 7, 8, dtype=torch.float16)
    w[..., :3] = (torch.randn(64, 7, 7, 3, generator=g) * (147 ** -0.5)).half()
    w = w.cuda()
    b = (torch.randn(64, generator=g) * 0.1).half().cuda()
    ref = ops.conv2d_nhwc_ref(ops.image_to_nhwc(img, 8), w, b, stride=2, pad=3, act="relu")
    y = ops.conv2d_nhwc(xs, ops.stem_weight_s2d(w), b, stride=1, pad=2, act="relu", out_hw=(112, 112))
    assert y.shape == (3, 112, 112, 64)
    _close(y, ref, 2e-2, 2e-2)


@pytest.mark.parametrize("N,H,W", [(3, 224, 224), (2, 64, 96), (1, 32, 32)])
def test_stem_s2d_pool_fused(N, H, W):
    """Image -> space-to-depth -> 4x4 stem conv -> ReLU -> 3x3/2 max-pool in one
    kernel, against the three-kernel path and the fp32 7x7 / stride-2 reference;
    the side job zeroes a split-K counter header."""
    ops = _ops()
    torch.manual_seed(H + W)
    img = torch.randint(0, 256, (N, H, W, 3), device="cuda", dtype=torch.uint8)
    g = torch.Generator().manual_seed(4)
    w7 = torch.zeros(64, 7, 7, 8, dtype=torch.float16)
    w7[..., :3] = (torch.randn(64, 7, 7, 3, generator=g) * (147 ** -0.5)).half()
    w7 = w7.cuda()
    b = (torch.randn(64, generator=g) * 0.1).half().cuda()
    ws4 = ops.stem_weight_s2d(w7)
    ws = ops.splitk_workspace("cuda", zeroed=False)
    ws[:ops.SPLITK_HEADER].fill_(0x5A)
    y = ops.stem_s2d_pool(img, ws4, b, zero=ws)
    torch.cuda.synchronize()
    assert y.shape == (N, H // 4, W // 4, 64)
    assert int(ws[:ops.SPLITK_HEADER].sum()) == 0
    three = ops.maxpool_nhwc(ops.conv2d_nhwc(ops.image_to_s2d(img), ws4, b, stride=1, pad=2, act="relu",
                                             out_hw=(H // 2, W // 2)), 3, 2, 1)
    _close(y, three, 1e-2, 1e-2)
    ref = ops.maxpool_nhwc_ref(ops.conv2d_nhwc_ref(ops.image_to_nhwc(img, 8), w7, b, stride=2, pad=3, act="relu"))
    _close(y, ref, 2e-2, 2e-2)


def test_image_to_nhwc_and_gather():
    ops = _ops()
    img = torch.randint(0, 256, (3, 32, 32, 3), device="cuda", dtype=torch.uint8)
    _close(ops.image_to_nhwc(img), ops.image_to_nhwc_ref(img), 1e-2, 1e-2)
    # gather from pinned host rows
    rows = torch.arange(4 * 64, dtype=torch.int32).reshape(4, 64).pin_memory()
    ptrs = torch.tensor([rows[i].data_ptr() for i in (2, 0, 3)], dtype=torch.int64).pin_memory()
    dst = torch.full((5, 64), -1, device="cuda", dtype=torch.int32)
    ops.gather_rows(ptrs, 3, 5, 256, dst)
    torch.cuda.synchronize()
    exp = torch.zeros(5, 64, dtype=torch.int32)
    exp[0], exp[1], exp[2] = rows[2], rows[0], rows[3]
    assert torch.equal(dst.cpu(), exp)


@pytest.mark.parametrize("N", [392, 388])   # 388 % 8 != 0: the direct (unstaged) epilogue
@pytest.mark.parametrize("cfg", list(range(30)))
def test_linear_all_tiles_random(cfg, N):
    ops = _ops()
    torch.manual_seed(11)
    x = torch.randn(300, 520, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, 520, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(300, N, device="cuda", dtype=torch.bfloat16)
    _close(ops.linear(x, w, b, act="gelu", residual=r, tile_cfg=cfg),
           ops.linear_ref(x, w, b, act="gelu", residual=r), 3e-2, 2e-2)


@pytest.mark.parametrize("cfg", [26, 27, 28])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_linear_v4_tiles(cfg, dtype):
    """The 4-wave VGPR-staged tiles (gemm_v4.h, K % 64 == 0): ragged M / N edges,
    every epilogue combination, both 16-bit dtypes, against the fp32 reference;
    K % 64 != 0 falls back to an 8-wave tile (still correct).  Experimental build
    only: no shipped table uses them (the default build falls back to tile 15)."""
    ops = _ops()
    if not ops.experimental_kernels_built():
        pytest.skip("tiles 26..28: opt-in RDB_EXPERIMENTAL_KERNELS build not loaded")
    torch.manual_seed(cfg)
    for M, N, K in ((300, 392, 512), (4096, 768, 768), (129, 200, 3072), (256, 96, 128)):
        x = torch.randn(M, K, device="cuda", dtype=dtype)
        w = torch.randn(N, K, device="cuda", dtype=dtype) * K ** -0.5
        b = torch.randn(N, device="cuda", dtype=dtype) * 0.1
        r = torch.randn(M, N, device="cuda", dtype=dtype)
        _close(ops.linear(x, w, tile_cfg=cfg), ops.linear_ref(x, w), 2e-2, 2e-2)
        _close(ops.linear(x, w, b, act="gelu", tile_cfg=cfg), ops.linear_ref(x, w, b, act="gelu"), 2e-2, 2e-2)
        _close(ops.linear(x, w, b, residual=r, tile_cfg=cfg), ops.linear_ref(x, w, b, residual=r), 2e-2, 2e-2)
        _close(ops.linear(x, w, residual=r, act="relu", tile_cfg=cfg), ops.linear_ref(x, w, residual=r, act="relu"),
               2e-2, 2e-2)
    x = torch.randn(200, 520, device="cuda", dtype=dtype)
    w = torch.randn(264, 520, device="cuda", dtype=dtype) * 0.05
    _close(ops.linear(x, w, tile_cfg=cfg), ops.linear_ref(x, w), 2e-2, 2e-2)


@pytest.mark.parametrize("cfg", [0, 8, 15, 19, 20, 21, 22, 24, 29])
def test_linear_swiglu_and_f16_tiles(cfg):
    """SwiGLU pairing epilogue and f16 on the 8-wave and ping-pong tiles."""
    ops = _ops()
    torch.manual_seed(12)
    x = torch.randn(272, 256, device="cuda", dtype=torch.float16)
    w = torch.randn(512, 256, device="cuda", dtype=torch.float16) * 0.05
    _close(ops.linear(x, w, act="swiglu", tile_cfg=cfg), ops.linear_ref(x, w, act="swiglu"), 3e-2, 2e-2)
    _close(ops.linear(x, w, tile_cfg=cfg), ops.linear_ref(x, w), 3e-2, 2e-2)
    # staged SwiGLU epilogue with bias (N % 16 == 0), and the direct one (N % 16 == 8)
    for n in (1040, 520):
        w2 = torch.randn(n, 256, device="cuda", dtype=torch.float16) * 0.05
        b2 = torch.randn(n, device="cuda", dtype=torch.float16) * 0.1
        _close(ops.linear(x, w2, b2, act="swiglu", tile_cfg=cfg), ops.linear_ref(x, w2, b2, act="swiglu"), 3e-2, 2e-2)


@pytest.mark.parametrize("cfg", list(range(13)))
def test_conv_all_tiles(cfg):
    ops = _ops()
    torch.manual_seed(12)
    x = torch.randn(2, 20, 20, 48, device="cuda", dtype=torch.float16)
    w = torch.randn(200, 3, 3, 48, device="cuda", dtype=torch.float16) * 0.07
    b = torch.randn(200, device="cuda", dtype=torch.float16) * 0.1
    _close(ops.conv2d_nhwc(x, w, b, stride=1, pad=1, act="relu", tile_cfg=cfg),
           ops.conv2d_nhwc_ref(x, w, b, stride=1, pad=1, act="relu"), 2e-2, 2e-2)


def test_shuffle_remap_split_and_full():
    from ray_dynamic_batching_amd import ops

    torch.manual_seed(0)
    base_a = torch.randn(2, 7, 5, 64, device="cuda", dtype=torch.float16)
    b = torch.randn(2, 7, 5, 64, device="cuda", dtype=torch.float16)
    a = base_a[..., :64]
    for ch in (58, 64):
        o1, o2 = ops.shuffle_remap(a, b, ch, True, 64, 64)
        r1, r2 = ops.shuffle_remap_ref(a, b, ch, True, 64, 64)
        assert torch.equal(o1, r1) and torch.equal(o2, r2)
        full = ops.shuffle_remap(a, b, ch, False, 128)
        assert torch.equal(full, ops.shuffle_remap_ref(a, b, ch, False, 128))
    # channel-slice view inputs (x1 = first half of a padded tensor)
    x = torch.randn(3, 4, 4, 128, device="cuda", dtype=torch.float16)
    o = ops.shuffle_remap(x[..., :64], x[..., 64:], 58, False, 120)
    assert torch.equal(o, ops.shuffle_remap_ref(x[..., :64], x[..., 64:], 58, False, 120))


def test_se_scale_and_sigmoid_gemm():
    from ray_dynamic_batching_amd import ops

    torch.manual_seed(1)
    x = torch.randn(4, 9, 9, 96, device="cuda", dtype=torch.float16)
    s = torch.rand(4, 96, device="cuda", dtype=torch.float16)
    assert torch.allclose(ops.se_scale(x, s).float(), ops.se_scale_ref(x, s).float(), atol=1e-2)
    a = torch.randn(8, 64, device="cuda", dtype=torch.float16)
    w = torch.randn(96, 64, device="cuda", dtype=torch.float16) * 0.1
    bias = torch.randn(96, device="cuda", dtype=torch.float16) * 0.1
    y = ops.linear(a, w, bias, act="sigmoid")
    r = ops.linear_ref(a, w, bias, act="sigmoid")
    assert torch.allclose(y.float(), r.float(), atol=5e-3)


@pytest.mark.parametrize("D", [100, 1664, 4100])
def test_norms_non_multiple_of_256(D):
    from ray_dynamic_batching_amd import ops

    torch.manual_seed(D)
    x = torch.randn(37, D, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(37, D, device="cuda", dtype=torch.bfloat16)
    g = torch.rand(D, device="cuda", dtype=torch.bfloat16) + 0.5
    b = torch.randn(D, device="cuda", dtype=torch.bfloat16)
    y = ops.layer_norm(x, g, b, 1e-5, residual=r)
    ref = ops.layer_norm_ref(x, g, b, 1e-5, residual=r)
    assert torch.allclose(y.float(), ref.float(), atol=3e-2, rtol=3e-2)
    y2 = ops.rms_norm(x, g, 1e-5)
    assert torch.allclose(y2.float(), ops.rms_norm_ref(x, g, 1e-5).float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M,N,K", [(1, 1000, 2048), (8, 2304, 768), (32, 768, 3072), (32, 2, 768),
                                   (33, 3072, 768), (64, 130, 96), (17, 4008, 4096)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_skinny_gemm_matches_fp32(M, N, K, dtype):
    """M <= 64 runs the weight-streaming skinny kernel (gemm_skinny.hip)."""
    ops = _ops()
    torch.manual_seed(M * 7 + N)
    x = torch.randn(M, K, device="cuda", dtype=dtype)
    w = torch.randn(N, K, device="cuda", dtype=dtype) * (K ** -0.5)
    b = torch.randn(N, device="cuda", dtype=dtype)
    r = torch.randn(M, N, device="cuda", dtype=dtype)
    _close(ops.linear(x, w), ops.linear_ref(x, w), 2e-2, 2e-2)
    _close(ops.linear(x, w, b, act="gelu", residual=r), ops.linear_ref(x, w, b, act="gelu", residual=r), 3e-2, 2e-2)
    y = ops.linear(x, w, b, act="tanh", out_dtype=torch.float32)
    _close(y, ops.linear_ref(x, w, b, act="tanh", out_dtype=torch.float32), 1e-2, 1e-2)
    # identical to the tiled kernel up to accumulation order
    _close(ops.linear(x, w, b), ops.linear(x, w, b, tile_cfg=ops.FORCE_TILED), 2e-2, 2e-2)


def test_skinny_gemm_strided_rows_and_residual():
    """BERT's CLS-only last layer: A and the residual are row-strided views."""
    ops = _ops()
    h = torch.randn(8, 128, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(768, 768, device="cuda", dtype=torch.bfloat16) * 0.03
    cls = h[:, 0, :]
    y = ops.linear(cls, w, residual=cls)
    _close(y, ops.linear_ref(cls.contiguous(), w, residual=cls.contiguous()), 2e-2, 2e-2)


def test_seq_lens():
    ops = _ops()
    ids = torch.randint(1, 100, (37, 128), device="cuda", dtype=torch.int32)
    ids[3, 50:] = 0
    ids[5, :] = 0
    ids[7, 1:] = 0
    assert torch.equal(ops.seq_lens(ids), ops.seq_lens_ref(ids))


def _ln_stats(x):
    xf = x.float()
    return torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).contiguous()


@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (4096, 2304, 768), (300, 768, 768)])
@pytest.mark.parametrize("act", ["none", "gelu"])
def test_linear_ln_lna_matches_layernorm_then_gemm(M, N, K, act):
    """LNA: raw rows + folded gamma/beta == LayerNorm(x) @ W.T + b (fp32 reference)."""
    ops = _ops()
    torch.manual_seed(0)
    x = (torch.randn(M, K, device="cuda") * 1.5 + 0.3).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    g = (1 + 0.2 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    be = (0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    w2, cs, b2 = ops.fold_ln_weights(w, b, g, be)
    y = ops.linear_ln(x, w2, act=act, lna=(_ln_stats(x), cs, b2, K, 1e-12))
    _close(y, ops.linear_ln_ref(x, w, b, act=act, ln_x=(g, be)), 3e-2, 3e-2)


@pytest.mark.parametrize("cfg", list(range(19)))
def test_linear_ln_stats_and_lnr_all_tiles(cfg):
    """LNR|STATS on every tile: the residual is normalised on load and the row
    statistics of the stored output match a torch reduction of it."""
    ops = _ops()
    torch.manual_seed(cfg)
    M, N, K = 520, 768, 384
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    r = (torch.randn(M, N, device="cuda") * 2 - 0.5).to(torch.bfloat16)
    g = (1 + 0.2 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    be = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    st = torch.zeros(M, 2, device="cuda")
    y = ops.linear_ln(x, w, b, residual=r, lnr=(_ln_stats(r), g, be, N, 1e-12), out_stats=st, tile_cfg=cfg)
    _close(y, ops.linear_ln_ref(x, w, b, residual=r, ln_res=(g, be)), 3e-2, 3e-2)
    ref = _ln_stats(y)
    assert torch.allclose(st, ref, rtol=1e-4, atol=1e-2), (st - ref).abs().max()
    # plain-residual STATS mode (first layer of the stack)
    st2 = torch.zeros(M, 2, device="cuda")
    y2 = ops.linear_ln(x, w, b, residual=r, out_stats=st2, tile_cfg=cfg)
    _close(y2, ops.linear_ref(x, w, b, residual=r), 3e-2, 3e-2)
    assert torch.allclose(st2, _ln_stats(y2), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("offset", [0.0, 8.0, 32.0])
def test_deferred_ln_large_row_mean(offset):
    """Deferred LayerNorm with rows far from zero mean: the variance
    comes from E[y^2] - mean^2 of f32 atomic sums, which cancels as |mean|/std
    grows.  Up to |mean| = 32 std -- beyond which bf16 activations cannot hold a
    unit-variance row anyway (their ulp at 32 is 0.25) -- the folded GEMM must
    still match LayerNorm-then-GEMM."""
    ops = _ops()
    torch.manual_seed(5)
    M, N, K = 512, 768, 768
    x = (torch.randn(M, K, device="cuda") + offset).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    g = (1 + 0.2 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    be = (0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    # the statistics as the producing GEMM's STATS epilogue accumulates them (f32 atomics)
    st = torch.zeros(M, 2, device="cuda")
    eye = torch.eye(K, device="cuda", dtype=torch.bfloat16)
    zb = torch.zeros(K, device="cuda", dtype=torch.bfloat16)
    zr = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    xr = ops.linear_ln(x, eye, zb, residual=zr, out_stats=st)   # y = x, stats of y accumulated in the epilogue
    assert torch.equal(xr, x)
    w2, cs, b2 = ops.fold_ln_weights(w, b, g, be)
    y = ops.linear_ln(x, w2, lna=(st, cs, b2, K, 1e-12))
    _close(y, ops.linear_ln_ref(x, w, b, ln_x=(g, be)), 3e-2, 3e-2)


@pytest.mark.parametrize("cfg", list(range(19)))
def test_linear_ln_self_stats_and_lnr_only_all_tiles(cfg):
    """LNA with in-kernel row statistics (no producer pass) on every tile: the
    output == LayerNorm-then-GEMM, the published (sum, sumsq) == a torch
    reduction of A; then LNR alone consumes them as the residual's LayerNorm.
    K = 776 leaves a partial last K tile (zero-filled, must not bias the sums)."""
    ops = _ops()
    torch.manual_seed(40 + cfg)
    M, N, K = 520, 768, 776
    x = (torch.randn(M, K, device="cuda") * 1.5 + 0.4).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    g = (1 + 0.2 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    be = (0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    w2, cs, b2 = ops.fold_ln_weights(w, b, g, be)
    st = torch.full((M, 2), float("nan"), device="cuda")
    y = ops.linear_ln(x, w2, act="gelu", lna=(None, cs, b2, K, 1e-12), out_stats=st, tile_cfg=cfg)
    _close(y, ops.linear_ln_ref(x, w, b, act="gelu", ln_x=(g, be)), 3e-2, 3e-2)
    ref = _ln_stats(x)
    assert torch.allclose(st, ref, rtol=1e-4, atol=1e-2), (st - ref).abs().max()
    # LNR only: y2 = h @ w3.T + b3 + LN(x)
    h = torch.randn(M, 384, device="cuda").to(torch.bfloat16)
    w3 = (torch.randn(K, 384, device="cuda") * 384 ** -0.5).to(torch.bfloat16)
    b3 = (torch.randn(K, device="cuda") * 0.1).to(torch.bfloat16)
    y2 = ops.linear_ln(h, w3, b3, residual=x, lnr=(st, g, be, K, 1e-12), tile_cfg=cfg)
    _close(y2, ops.linear_ln_ref(h, w3, b3, residual=x, ln_res=(g, be)), 3e-2, 3e-2)


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
def test_qkv_attention_folded_layernorm(cfg):
    """Fused projection+attention on RAW rows with the LayerNorm folded into the
    packed weight == LayerNorm -> unfused reference; the statistics it
    publishes (head 0) == a torch reduction; S < 128 so the 128-row tile
    reaches into the next sequence (whose rows it must not publish)."""
    ops = _ops()
    torch.manual_seed(50 + cfg)
    B, S, H, K = 5, 100, 4, 256
    x = (torch.randn(B * S, K, device="cuda") * 1.3 - 0.2).to(torch.bfloat16)
    w = (torch.randn(3 * H * 64, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(3 * H * 64, device="cuda") * 0.1).to(torch.bfloat16)
    g = (1 + 0.2 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    be = (0.1 * torch.randn(K, device="cuda")).to(torch.bfloat16)
    lens = torch.randint(1, S + 1, (B,), device="cuda", dtype=torch.int32)
    w2, cs, bf = ops.fold_ln_weights(w, b, g, be)
    wp, bfp = ops.pack_qkv_heads(w2, bf, H)
    csp = ops.pack_qkv_vec(cs, H)
    st = torch.full((B * S, 2), float("nan"), device="cuda")
    y = ops.qkv_attention(x, wp, None, B, S, H, lens=lens, cfg=cfg, lna=(csp, bfp, 1e-12), stats_out=st)
    xn = ops.layer_norm_ref(x, g, be, 1e-12)
    _close(y, ops.qkv_attention_ref(xn, w, b, B, S, H, lens=lens), 3e-2, 3e-2)
    ref = _ln_stats(x)
    assert torch.allclose(st, ref, rtol=1e-4, atol=1e-2), (st - ref).abs().max()


@pytest.mark.parametrize("cfg", list(range(19)))
@pytest.mark.parametrize("M", [4096, 520])
def test_linear_residual_ln_all_tiles(cfg, M):
    """GEMM + bias + residual + LayerNorm in one kernel (row-panel statistics):
    every tile (those that cannot hold the f32 tile are remapped on the host),
    M = 520 leaves a partial last row panel and makes panels straddle XCDs
    (xcd_remap: 9 tiles per XCD with 8 tiles per panel at 64x96).  Repeated
    launches on re-zeroed workspaces agree (up to the f32 atomic order)."""
    ops = _ops()
    _need_experimental(ops)
    torch.manual_seed(60 + cfg)
    N, K = 768, 768
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    r = (torch.randn(M, N, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    g = (1 + 0.2 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    be = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    ref = ops.linear_residual_ln_ref(x, w, b, r, g, be)
    outs = []
    for _ in range(2):
        st = torch.zeros(M, 2, device="cuda")
        pn = torch.zeros(M, device="cuda", dtype=torch.int32)
        outs.append(ops.linear_residual_ln(x, w, b, r, g, be, 1e-12, st, pn, tile_cfg=cfg))
    torch.cuda.synchronize()
    assert not ops.ln_out_error()
    _close(outs[0], ref, 3e-2, 3e-2)
    _close(outs[1], outs[0], 1e-2, 1e-2)


@pytest.mark.parametrize("M,K", [(32, 768), (4096, 768), (4097, 768), (4096, 3072), (200, 800), (64, 832)])
def test_linear_rowln_vs_fp32(M, K):
    """Full-row GEMM + bias + residual + LayerNorm (gemm_rowln.hip) against the
    fp32 reference: partial last block (M = 4097, 200), K steps not a multiple of
    the 3-step unroll (800 = 25 steps, 832 = 26), FFN-down's K = 3072.  Repeat
    launches are bit-identical (no atomics: the statistics are block-local)."""
    ops = _ops()
    _need_experimental(ops)
    torch.manual_seed(M + K)
    N = 768
    x = (torch.randn(M, K, device="cuda") * 1.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    r = (torch.randn(M, N, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    g = (1 + 0.2 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    be = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    ref = ops.linear_residual_ln_ref(x, w, b, r, g, be)
    wp = ops.pack_rowln_weight(w)
    y1 = ops.linear_rowln(x, wp, b, r, g, be, 1e-12)
    y2 = ops.linear_rowln(x, wp, b, r, g, be, 1e-12)
    torch.cuda.synchronize()
    _close(y1, ref, 3e-2, 3e-2)
    assert torch.equal(y1, y2)
    # row-strided operands (a CLS-style view of x, a wider output buffer)
    xs = torch.zeros(M, K + 64, device="cuda", dtype=torch.bfloat16)
    xs[:, :K] = x
    ob = torch.full((M, N + 32), float("nan"), device="cuda", dtype=torch.bfloat16)
    ops.linear_rowln(xs[:, :K], wp, b, r, g, be, 1e-12, out=ob[:, :N])
    torch.cuda.synchronize()
    assert torch.equal(ob[:, :N], y1) and torch.isnan(ob[:, N:].float()).all()


def test_layer_norm_row_strided_view_and_embed_zeroes_stats():
    ops = _ops()
    torch.manual_seed(1)
    B, S, D = 6, 16, 768
    h = torch.randn(B * S, D, device="cuda", dtype=torch.bfloat16)
    g = (1 + 0.1 * torch.randn(D, device="cuda")).to(torch.bfloat16)
    b = (0.1 * torch.randn(D, device="cuda")).to(torch.bfloat16)
    cls = h.view(B, S, D)[:, 0, :]
    _close(ops.layer_norm(cls, g, b), ops.layer_norm_ref(cls.contiguous(), g, b), 2e-2, 2e-2)
    ids = torch.randint(1, 1000, (B, S), device="cuda", dtype=torch.int32)
    word = torch.randn(1000, D, device="cuda", dtype=torch.bfloat16)
    pos = torch.randn(S, D, device="cuda", dtype=torch.bfloat16)
    typ = torch.randn(2, D, device="cuda", dtype=torch.bfloat16)
    st = torch.full((3, 2, B * S, 2), 7.0, device="cuda")
    y = ops.embed_ln(ids, word, pos, typ, g, b, zero_stats=st)
    _close(y, ops.embed_ln_ref(ids, word, pos, typ, g, b), 2e-2, 2e-2)
    assert st.abs().max().item() == 0.0


@pytest.mark.parametrize("readback", ["sdma", "blit"])
def test_graph_replayed_plain_store_kernel_visible_to_d2h(readback):
    """A graph-replayed kernel writing with plain (L2 write-back) stores -- a
    GEMM with the staged epilogue -- must be read back correctly by the
    device->host copy that follows, replay after replay with new inputs:
    the regression guard for the xGMI fused-norm readback finding
    (parallel/xgmi.py norm_store).  ``blit``: read through a device-side copy
    kernel first (what a copy engine that bypassed the L2 would not see)."""
    ops = _ops()
    torch.manual_seed(0)
    M, N, K = 4096, 768, 768
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * (K ** -0.5)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.linear(x, w, b)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            y = ops.linear(x, w, b, act="gelu")
    torch.cuda.synchronize()
    for it in range(5):
        x.copy_(torch.randn(M, K, device="cuda", dtype=torch.bfloat16))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        got = (y.clone() if readback == "blit" else y).cpu()
        ref = ops.linear_ref(x, w, b, act="gelu").cpu()
        _close(got, ref, 2e-2, 2e-2)


@pytest.mark.parametrize("M,N,K,tile,grid", [(4096, 768, 3072, 0, 192), (4096, 768, 768, 1, 192),
                                             (1000, 768, 3072, 0, 256), (37, 256, 512, 0, 64),
                                             (4096, 2304, 768, 1, 256)])
def test_linear_streamk(M, N, K, tile, grid):
    """stream-K GEMM (split tiles finished by the last-arriving segment) against
    the fp32 reference, over repeated launches on one workspace (the arrival
    counters must reset themselves) and on a ragged M."""
    ops = _ops()
    _need_experimental(ops)
    torch.manual_seed(11)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    ws = ops.streamk_workspace("cuda", grid, tile)
    ref = x.float() @ w.float().t() + b.float() + r.float()
    for _ in range(3):
        y = ops.linear_streamk(x, w, b, residual=r, workspace=ws, grid=grid, tile=tile)
        _close(y, ref, 2e-2, 2e-2)
    g = ops.linear_streamk(x, w, b, act="gelu", workspace=ws, grid=grid, tile=tile)
    _close(g, torch.nn.functional.gelu(x.float() @ w.float().t() + b.float()), 2e-2, 2e-2)
    assert int(ws[:65536].view(torch.int32).abs().sum()) == 0     # counters clean after every launch
