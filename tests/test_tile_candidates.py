"""Tile-choice encodings the conv / GEMM tuners rank (ops/__init__.py; decoded
by gemm_core.h launch_mfma_gemm / conv.hip): tile | splits << 8 | DEEP, and
CONV_LINEAR | cfg for 1x1 convolutions on the dense GEMM tiles.  CPU-only:
the candidate lists, not the kernels."""
from ray_dynamic_batching_amd import ops


def _decode(c):
    return c & 255, (c >> 8) & 15, bool(c & ops.DEEP), bool(c & ops.CONV_LINEAR)


def test_conv_candidates_encode_valid_choices():
    # ResNet-50 layer-3 3x3 conv at bs32 and a layer-1 1x1 conv
    for M, N, Kg, one in ((6272, 256, 2304, False), (100352, 256, 64, True), (1568, 512, 4608, False)):
        cands = ops._conv_candidates(M, N, Kg, one)
        assert len(cands) == len(set(cands))
        nk = -(-Kg // 64)
        for c in cands:
            tile, splits, deep, linear = _decode(c)
            if linear:
                assert one and (c - ops.CONV_LINEAR) & 0xFF < ops.NUM_TILE_CFGS
                continue
            assert 0 <= tile < ops.NUM_CONV_TILE_CFGS
            if deep:
                assert tile in ops._DEEP_TILES
            if splits:
                kper = -(-nk // splits)
                assert kper >= 4 and -(-nk // kper) >= 2          # every split non-empty, >= 4 K steps
                tiles = -(-M // ops._TILE_BM[tile]) * -(-N // ops._TILE_BN[tile])
                assert ops.SPLITK_HEADER + tiles * -(-nk // kper) * ops._TILE_BM[tile] * ops._TILE_BN[tile] * 4 \
                    <= ops.SPLITK_WS_BYTES
        if one:
            assert any(c & ops.CONV_LINEAR for c in cands)
        if M == 1568:
            assert any((c >> 8) & 15 for c in cands)                # the small-grid conv gets split-K choices


def test_gemm_candidates_deep_only_where_a_block_per_cu():
    cands = ops._gemm_candidates(4096, 768, 3072)
    # every tile, except the VGPR-staged 26..28 outside the experimental build
    want = {c for c in range(ops.NUM_TILE_CFGS) if not 26 <= c <= 28 or ops._v4_tiles_built()}
    assert want <= set(cands)
    assert ops._v4_tiles_built() or not {26, 27, 28} & set(cands)
    for c in cands:
        if c & ops.DEEP:
            t = c & 255
            assert t in ops._DEEP_TILES
            if t not in ops._DEEP_BIG:
                assert -(-4096 // ops._TILE_BM[t]) * -(-768 // ops._TILE_BN[t]) <= ops._DEEP_MAX_BLOCKS
    assert all(not (c & ops.DEEP) for c in ops._gemm_candidates(4096, 768, 128))   # short K: none


def test_tile_tables_match_the_tuned_directory():
    """Every shipped table entry decodes to a valid choice."""
    import glob
    import json
    import os

    d = os.path.join(os.path.dirname(ops.__file__), "tuned")
    for f in glob.glob(os.path.join(d, "*.json")):
        for key, c in json.load(open(f)):
            assert isinstance(c, int) and c >= -1, (f, key, c)
            if key[0] == "conv" and c >= 0 and c < ops.CONV_LINEAR:
                assert (c & 255) < ops.NUM_CONV_TILE_CFGS, (f, key, c)


def test_cu_share_of_tile_grids():
    """CU share the tuner multiplies a tile's time by to rank CU-time: BERT's
    o-projection (4096 x 768) holds half the CUs on 256 4-wave 128x96 blocks (two
    per CU) and 3/8 of them on 96 ping-pong 256x128 blocks; a full grid holds all."""
    assert ops._cu_share(10, 4096, 768) == 0.5
    assert ops._cu_share(19, 4096, 768) == 96 / 256
    assert ops._cu_share(3, 4096, 768) == 1.0
    assert ops._cu_share(0 | (2 << 8), 4096, 768) == 1.0 or ops._cu_share(0 | (2 << 8), 4096, 768) > ops._cu_share(0, 4096, 768)
    assert ops._cu_share(0 | ops.DEEP, 1024, 768) == min(1.0, 8 * 6 / 256)


def test_key_output_shape_for_cu_time():
    assert ops._key_mn(("gemm", "torch.bfloat16", 4096, 768, 3072, 3072, "none", True, True)) == (4096, 768)
    assert ops._key_mn(("conv", 32, 14, 14, 256, 256, 3, 3, 1, 1, "relu", True, False)) == (32 * 14 * 14, 256)
    assert ops._key_mn(("conv", 32, 112, 112, 16, 64, 4, 4, 1, 2, "relu", True, False, 112, 112)) == (32 * 112 * 112, 64)
    assert ops._key_mn(("qkv_attn", "torch.bfloat16", 32, 128, 12, 768, 768, False)) is None
    # a 1x1 conv on the dense ping-pong tile: its share follows the GEMM grid
    assert ops._cu_share(ops.CONV_LINEAR | 19, 1568, 2048) == ops._cu_share(19, 1568, 2048)


def test_conv_pp_candidates():
    """Ping-pong conv tiles (CONV_PP | v | splits << 8) for the im2col convs of
    ResNet-50 at bs32: only where BK divides C and a bias is fused, split-K only
    under ~one block per CU, every split non-empty, partials within the workspace."""
    assert ops.splits_of(ops.CONV_PP | 2 | (4 << 8)) == 4
    assert ops.splits_of(ops.CONV_PP | 3) == 0
    assert ops.splits_of(ops.CONV_LINEAR | 19) == 0
    for M, N, Kg, C in ((100352, 64, 576, 64), (25088, 128, 1152, 128), (6272, 256, 2304, 256), (1568, 512, 4608, 512)):
        cands = ops._conv_candidates(M, N, Kg, False, C, True)
        pp = [c for c in cands if c & ops.CONV_PP]
        assert pp and len(cands) == len(set(cands))
        assert not [c for c in ops._conv_candidates(M, N, Kg, False, C, False) if c & ops.CONV_PP]   # no bias: none
        for c in pp:
            v, sp = c & 255, ops.splits_of(c)
            assert not c & ops.CONV_LINEAR and not c & ops.DEEP
            bm, bn, bk = ops._CONV_PP_BM[v], ops._CONV_PP_BN[v], ops._CONV_PP_BK[v]
            assert C % bk == 0
            tiles = -(-M // bm) * -(-N // bn)
            if sp:
                assert tiles < 256
                nk = Kg // bk
                kper = -(-nk // sp)
                eff = -(-nk // kper)
                assert eff >= 2 and kper >= 3
                assert ops.SPLITK_HEADER + tiles * eff * bm * bn * 4 <= ops.SPLITK_WS_BYTES
            share = ops._cu_share(c, M, N)
            assert 0 < share <= 1.0
        if M == 1568:
            assert any(ops.splits_of(c) for c in pp)                   # stage 4: split-K choices
    # C = 96 (no BK divides it... 96 % 32 == 0): the BK 32 tiles only
    pp = [c for c in ops._conv_candidates(6272, 96, 864, False, 96, True) if c & ops.CONV_PP]
    assert pp and all(ops._CONV_PP_BK[c & 255] == 32 for c in pp)


def test_gemm_candidates_pingpong_splitk():
    """Llama-3-8B prefill down projection at 8 x 128 tokens (1024 x 4096 x 14336):
    128 ping-pong 256x128 tiles leave half the CUs idle, so tiles 19 / 21 get
    split-K choices (workspace-bounded); a full grid gets none."""
    cands = ops._gemm_candidates(1024, 4096, 14336, splitk=True)
    pp = [c for c in cands if (c & 255) in ops._PP_SPLITK_TILES and ops.splits_of(c) > 1]
    assert pp
    for c in pp:
        t, sp = c & 255, ops.splits_of(c)
        tiles = -(-1024 // ops._ALL_BM[t]) * -(-4096 // ops._ALL_BN[t])
        nk = 14336 // 64
        eff = -(-nk // -(-nk // sp))
        assert ops.SPLITK_HEADER + tiles * eff * ops._ALL_BM[t] * ops._ALL_BN[t] * 4 <= ops.SPLITK_WS_BYTES
    assert not [c for c in ops._gemm_candidates(4096, 3072, 768, splitk=True) if ops.splits_of(c) > 1 and (c & 255) >= 19]


def test_conv_halo_candidates():
    """Halo-tile 3x3 tiles (CONV_HALO | v): only for same-size 3x3 convs with a
    bias and C % 64 == 0; each candidate's rows fit the image (conv_halo_tiles
    > 0, the C++ geometry); never split."""
    import pytest

    try:
        tiles = ops._ops().conv_halo_tiles
    except Exception as e:   # extension not built in this checkout
        pytest.skip(f"ops extension unavailable: {e}")
    for N, H, C, K in ((32, 56, 64, 64), (32, 28, 128, 128), (32, 14, 256, 256), (32, 7, 512, 512)):
        cands = ops.conv_halo_candidates(N, H, H, C, K, 3, 3, 1, 1, H, H, True)
        assert cands and len(cands) == len(set(cands))
        for c in cands:
            v, sp = c & 255, ops.splits_of(c)
            assert c & ops.CONV_HALO and tiles(v, N, H, H, C, K) > 0
            if sp:      # split-K: a two-buffer streamed tile, an under-filled grid, every split non-empty
                assert v in ops._CONV_HALO_SK and tiles(v, N, H, H, C, K) < 256 and C // 64 >= 2
                need = ops._ops().conv_halo_ws_bytes(v, N, H, H, C, K, sp, 1)
                assert ops.SPLITK_HEADER < need <= ops.SPLITK_WS_BYTES
        assert not ops.conv_halo_candidates(N, H, H, C, K, 3, 3, 1, 1, H, H, False)      # no bias
        # stride 2 (pad 1): streamed tiles only, never the resident-weight ones
        s2 = ops.conv_halo_candidates(N, 2 * H, 2 * H, C, K, 3, 3, 2, 1, H, H, True)
        assert all((c & 255) not in ops._CONV_HALO_RW for c in s2)
        assert not ops.conv_halo_candidates(N, H, H, C, K, 3, 3, 2, 0, H // 2, H // 2, True)   # pad 0
    assert not ops.conv_halo_candidates(32, 56, 56, 96, 64, 3, 3, 1, 1, 56, 56, True)      # C % 64
    # stage 1 (56 wide): the 256-pixel tile takes 4 output rows; 64 px cannot hold one
    assert tiles(0, 32, 56, 56, 64, 64) == 32 * 14 and tiles(3, 32, 56, 56, 64, 64) == -1
    # one patch buffer: only a single 64-channel block
    assert tiles(0, 32, 28, 28, 128, 128) == -1 and tiles(2, 32, 28, 28, 128, 128) == 32 * 7 * 2
    # stage 4 (7 x 7): two images per 112-pixel tile
    assert tiles(2, 32, 7, 7, 512, 512) == 16 * 8
    # split-K offered for the small-image layers only (stage 1 has one channel block)
    assert any(ops.splits_of(c) for c in ops.conv_halo_candidates(32, 7, 7, 512, 512, 3, 3, 1, 1, 7, 7, True))
    assert not any(ops.splits_of(c) for c in ops.conv_halo_candidates(32, 56, 56, 64, 64, 3, 3, 1, 1, 56, 56, True))
    assert ops._cu_share(ops.CONV_HALO | 0, 100352, 64) == 1.0
