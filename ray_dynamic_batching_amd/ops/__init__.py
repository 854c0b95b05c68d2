"""Python wrappers of the gfx950 kernels, plus plain-PyTorch fp32 references.

Every wrapper validates shapes / dtypes / strides / alignment on the host
before launching (a mis-shaped launch on the GPU can take the whole node down),
allocates its output with the torch caching allocator and launches on
``torch.cuda.current_stream()`` -- so the calls are capturable into hipGraphs.

The ``*_ref`` functions are the numerics references used by the tests and the
eager baseline path of the models (``backend="torch"``).
"""
from __future__ import annotations

import contextlib
import math
import os
import threading
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from ..utils.native import require_gpu_ops

DTYPE_CODE = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2}
ACT_CODE = {"none": 0, "gelu": 1, "relu": 2, "tanh": 3, "silu": 4, "gelu_tanh": 5, "swiglu": 6, "sigmoid": 7}


def _ops():
    return require_gpu_ops()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def _aligned(t: torch.Tensor, n: int = 16) -> bool:
    return t.data_ptr() % n == 0


# ---------------------------------------------------------------------------
# Per-shape autotuning of the GEMM / conv tile configuration.  The kernels
# take a tile index (see gemm_core.h kTileBM/kTileBN); on the first eager call
# of a shape every candidate is timed and the fastest is cached.  Never runs
# while a hipGraph is being captured (those calls use the cached choice, or the
# on-device heuristic if the shape was never seen eagerly).
# ---------------------------------------------------------------------------
NUM_TILE_CFGS = 30   # gemm_core.h kTileBM/BN: 0..12 4-wave (GEMM and conv), 13..18 8-wave, 19..25 ping-pong,
                     # 26..28 4-wave VGPR-staged one-block-per-CU tiles (gemm_v4.h; GEMM only, K % 64 == 0),
                     # 29 ping-pong 256x224 (the Llama gate-up N = 28672 = 128 x 224)
NUM_LN_TILE_CFGS = 19  # the deferred-LayerNorm epilogues run on tiles 0..18
NUM_CONV_TILE_CFGS = 13
FORCE_TILED = 99      # tile_cfg value that bypasses the skinny-M GEMM (M <= 64)
SKINNY_MAX_M = 64
_TUNE: Dict[tuple, int] = {}


def autotune_enabled() -> bool:
    return os.environ.get("RDB_AUTOTUNE", "1") == "1"


def tuning_table() -> Dict[tuple, int]:
    return dict(_TUNE)


def _key_json(key: tuple) -> list:
    return [str(v) if isinstance(v, torch.dtype) else v for v in key]


def _key_from_json(key: list) -> tuple:
    return tuple(getattr(torch, v.split(".", 1)[1]) if isinstance(v, str) and v.startswith("torch.") else v
                 for v in key)


def save_tuning(path: str) -> None:
    """Write the per-shape tile table (JSON) so another process replays the same
    kernel choices (profiling passes, A/B runs) instead of re-tuning."""
    import json

    with open(path, "w") as f:
        json.dump([[_key_json(k), c] for k, c in _TUNE.items()], f)


def load_tuning(path: str) -> int:
    """Load a table written by save_tuning(); returns the number of entries."""
    import json

    with open(path) as f:
        rows = json.load(f)
    for k, c in rows:
        _TUNE[_key_from_json(k)] = int(c)
    return len(rows)


_TUNE_TOP: Dict[tuple, list] = {}


def tune_in_context(time_forward: Callable[[], float], keys: Optional[list] = None, min_gain: float = 0.01) -> dict:
    """Pick among each GEMM shape's near-tied tiles by timing the WHOLE forward.

    The per-shape tuner times a GEMM alone; inside a forward its inputs were just
    written by the previous kernel (dirty L2 lines, MALL residency) and its
    neighbours compete for the chip, and tiles within a few percent of each other
    alone can differ by 20 % there.  ``time_forward()`` must re-capture/replay the
    forward with the current ``_TUNE`` table and return its time; shapes are
    visited one at a time (coordinate descent), a change is kept only if it beats
    the current best by ``min_gain``.  Returns {key: (old, new)} for changed keys."""
    changed = {}
    best = time_forward()
    for key in list(keys if keys is not None else _TUNE_TOP):
        cands = _TUNE_TOP.get(key, [])
        if len(cands) < 2 or key not in _TUNE:
            continue
        start = cur = _TUNE[key]
        for c in cands:
            if c == cur:
                continue
            _TUNE[key] = c
            t = time_forward()
            if t < best * (1 - min_gain):
                best, cur = t, c
        _TUNE[key] = cur
        if cur != start:
            changed[key] = (start, cur)
    return changed


# gemm_core.h kTileBM / kTileBN / kTileNW and tile_blocks_per_cu (CU-time estimates of the tuner)
_ALL_BM = (128, 64, 128, 64, 128, 192, 256, 128, 128, 64, 128, 256, 128, 256, 128, 256, 256, 128, 256, 256, 256, 128,
           256, 256, 256, 256, 128, 128, 256, 256)
_ALL_BN = (128, 128, 64, 64, 192, 128, 128, 256, 144, 96, 96, 144, 48, 128, 256, 192, 144, 96, 96, 128, 144, 256, 256,
           128, 192, 192, 96, 128, 192, 224)
_ALL_NW = (4,) * 13 + (8,) * 13 + (4,) * 3 + (8,)


def _blocks_per_cu(t: int) -> int:
    if t == 23:
        return 2
    if t >= 19:                     # ping-pong and VGPR-staged tiles: one block per CU
        return 1
    q = 8 * _ALL_NW[t]
    bnp = -(-_ALL_BN[t] // q) * q
    return max(1, min(8 // _ALL_NW[t], 163840 // (2 * (_ALL_BM[t] + bnp) * 64 * 2)))


def _key_mn(key: tuple):
    """(M, N) of the output a tuning key's launches write: dense GEMM keys carry
    them, conv keys give N*P*Q output pixels x K channels; None otherwise."""
    if key[0] == "gemm":
        return key[2], key[3]
    if key[0] == "conv":
        N, H, W, C, K, R, S, stride, pad = key[1:10]
        P, Q = (key[13], key[14]) if len(key) >= 15 else ((H + 2 * pad - R) // stride + 1,
                                                           (W + 2 * pad - S) // stride + 1)
        return N * P * Q, K
    return None


def _cu_share(c: int, M: int, N: int, cus: int = 256) -> float:
    """Share of the GPU's CUs a GEMM launch with tile choice ``c`` holds (split-K
    multiplies the blocks, DEEP holds a whole CU per block)."""
    t = c & 255
    if c >= 0 and c & CONV_HALO:
        if not 0 <= t < len(_CONV_HALO_BM):
            return 1.0
        return min(1.0, -(-M // _CONV_HALO_BM[t]) * -(-N // _CONV_HALO_BN[t]) * max(1, (c >> 8) & 15) / cus)
    if c >= 0 and c & CONV_PP:
        if not 0 <= t < len(_CONV_PP_BM):
            return 1.0
        blocks = -(-M // _CONV_PP_BM[t]) * -(-N // _CONV_PP_BN[t]) * max(1, (c >> 8) & 15)
        return min(1.0, blocks / (cus * (2 if _CONV_PP_BK[t] == 32 else 1)))   # BK 32 tiles: 2 blocks / CU
    if not 0 <= t < len(_ALL_BM):
        return 1.0
    blocks = -(-M // _ALL_BM[t]) * -(-N // _ALL_BN[t]) * max(1, (c >> 8) & 15)
    per_cu = 1 if c & DEEP else _blocks_per_cu(t)
    return min(1.0, blocks / (cus * per_cu))


_KEY_LOG: Optional[list] = None


class record_tuning_keys:
    """``with record_tuning_keys() as keys: model(x)`` -> the tuned GEMM/conv keys that forward used."""

    def __enter__(self):
        global _KEY_LOG
        _KEY_LOG = []
        return _KEY_LOG

    def __exit__(self, *exc):
        global _KEY_LOG
        _KEY_LOG = None
        return False


# RDB_TUNE_GRAPH=1: time tuning candidates from a replayed hipGraph instead of eager launches.  Off by
# default: it ranks the kernels themselves without the Python launch path, but tables tuned that way
# served no better than eager-tuned ones (BERT 35.3k vs 35.0-35.8k, ResNet-50 41.1k vs 41.8-44.2k
# img/s, profiles/tuner_graph_timing_r6.json) -- the in-context pass decides among the top candidates
_TUNE_GRAPH = os.environ.get("RDB_TUNE_GRAPH", "0") == "1"
_tune_graph_broken = False
_TUNE_STREAMS: Dict[tuple, list] = {}


def _tune_streams(n: int) -> list:
    """The tuner's own streams on the current device (created once: per-stream
    split-K workspaces are cached by stream, so fresh streams per shape would
    each pin another workspace): [capture stream, side stream 1, ...]."""
    key = (torch.cuda.current_device(), n)
    st = _TUNE_STREAMS.get(key)
    if st is None:
        st = _TUNE_STREAMS[key] = [torch.cuda.Stream() for _ in range(n)]
    return st


def _time_tile_graph(launch: Callable[[int], None], c: int, cap, side: list, s, e, reps: int = 4) -> float:
    """Best-of-3 time of ``reps`` launches of tile ``c`` on the current stream
    (plus one per side stream each) replayed from a captured hipGraph.  Eager
    timing includes the Python launch path (~15 us per launch, as long as the
    faster BERT / ResNet kernels themselves at RDB_TUNE_STREAMS=3).  Every
    lazily allocated buffer (split-K workspaces) exists before the capture:
    the caller launched ``c`` eagerly on every stream first."""
    cur = torch.cuda.current_stream()
    cap.wait_stream(cur)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
        for _ in range(reps):
            launch(c)
            for sd in side:
                sd.wait_stream(cap)
                with torch.cuda.stream(sd):
                    launch(c)
        for sd in side:
            cap.wait_stream(sd)
    cur.wait_stream(cap)
    g.replay()                       # first replay: uploads the graph
    t = float("inf")
    for _trial in range(3):          # best of 3: clock / neighbour noise only ever adds time
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        t = min(t, s.elapsed_time(e))
    del g
    return t


def _tuned_cfg(key: tuple, launch: Callable[[int], None], candidates=range(NUM_TILE_CFGS)) -> int:
    global _tune_graph_broken
    if _KEY_LOG is not None and key not in _KEY_LOG:
        _KEY_LOG.append(key)
    cfg = _TUNE.get(key)
    if cfg is not None:
        return cfg
    if not autotune_enabled() or torch.cuda.is_current_stream_capturing():
        return -1
    best_t, best_c = float("inf"), -1
    times: Dict[int, float] = {}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # RDB_TUNE_STREAMS=n (n > 1): rank tiles by THROUGHPUT with n launches in
    # flight on n streams -- what a replica running n concurrent batches sees --
    # instead of the isolated latency, which favours small tiles that fill the
    # CUs alone but cost more LDS/VMEM traffic per FLOP when streams overlap.
    ns = max(1, int(os.environ.get("RDB_TUNE_STREAMS", "1")))
    streams = _tune_streams(ns)
    cap, side = streams[0], streams[1:]
    cur = torch.cuda.current_stream()
    for c in candidates:
        launch(c)
        for sd in streams:               # every stream's lazily allocated buffers, outside any capture
            sd.wait_stream(cur)
            with torch.cuda.stream(sd):
                launch(c)
            cur.wait_stream(sd)
        t = float("inf")
        if _TUNE_GRAPH and not _tune_graph_broken:
            try:
                t = _time_tile_graph(launch, c, cap, side, s, e)
            except Exception:            # a launch path that cannot be captured: eager timing from here on
                _tune_graph_broken = True
                torch.cuda.synchronize()
        if t == float("inf"):
            for _trial in range(3):          # best of 3: clock / neighbour noise only ever adds time
                s.record()
                for sd in side:
                    sd.wait_stream(cur)
                for _ in range(4):
                    launch(c)
                    for sd in side:
                        with torch.cuda.stream(sd):
                            launch(c)
                for sd in side:
                    cur.wait_stream(sd)
                e.record()
                e.synchronize()
                t = min(t, s.elapsed_time(e))
        times[c] = t
        if t < best_t:
            best_t, best_c = t, c
    # the runners-up within 15 %: candidates for in-context selection (tune_in_context) ...
    top = [c for c in sorted(times, key=times.get) if times[c] <= best_t * 1.15][:3]
    mn = _key_mn(key)
    if mn is not None:
        # ... plus the two with the least CU-TIME (time x share of the CUs the grid holds): beside
        # another stream's batch a slower tile on fewer blocks can win (profiles/ab_r4_tables_cu_time.json:
        # BERT's o-projection on 96 ping-pong blocks, +2.7..6.5 % over the fastest-alone 256-block tile)
        cu = {c: t * _cu_share(c, *mn) for c, t in times.items() if t < float("inf")}
        top += [c for c in sorted(cu, key=cu.get)[:2] if c not in top]
    _TUNE_TOP[key] = top
    _TUNE[key] = best_c
    return best_c


# ---------------------------------------------------------------------------
# GEMM (+ fused bias / activation / residual epilogue)
# ---------------------------------------------------------------------------
_SWIGLU_TILE_CFGS = tuple(range(26)) + (29,)   # the VGPR-staged tiles (26..28) have no SwiGLU epilogue


def _gemm_candidates(M: int, N: int, K: int, splitk: bool = False):
    """Dense GEMM tile choices: every tile cfg, plus the DEEP variants of the
    4-wave tiles whose grid is about one block per CU (``DEEP`` flag), plus
    (``splitk``) split-K variants of the 4-wave tiles and the BK-64 ping-pong
    tiles 19 / 21 where the tile grid leaves CUs idle and each split keeps >= 8 K
    steps (long-K GEMMs of small M: the Llama prefill's down projection at 128
    tokens is 128 blocks x 224 K steps; at 1024 tokens 128 ping-pong tiles)."""
    # VGPR-staged tiles 26..28: K % 64 == 0, and only in the experimental build (they tied
    # or lost every engine A/B, profiles/ab_r5_v4_bert.json)
    v4 = K % 64 == 0 and _v4_tiles_built()
    cands = [c for c in range(NUM_TILE_CFGS) if not 26 <= c <= 28 or v4]
    if _GEMM_DEEP and K >= 256:
        cands += [c | DEEP for c in _DEEP_TILES
                  if c in _DEEP_BIG or -(-M // _TILE_BM[c]) * -(-N // _TILE_BN[c]) <= _DEEP_MAX_BLOCKS]
    if splitk and _GEMM_SPLITK:
        nk = -(-K // 64)
        for c in list(range(NUM_CONV_TILE_CFGS)) + list(_PP_SPLITK_TILES):
            tiles = -(-M // _ALL_BM[c]) * -(-N // _ALL_BN[c])
            if tiles >= 256:
                continue
            for sp in _SPLITS:
                kper = -(-nk // sp)
                eff = -(-nk // kper)
                if eff < 2 or kper < 8 or tiles * eff > 1024:
                    continue
                if SPLITK_HEADER + tiles * eff * _ALL_BM[c] * _ALL_BN[c] * 4 > SPLITK_WS_BYTES:
                    continue
                cands.append(c | (sp << 8))
    return cands


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: str = "none",
           residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           out_dtype: Optional[torch.dtype] = None, alpha: float = 1.0, tile_cfg: int = -1,
           workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = act(alpha * x @ w.T + bias + residual).  x: [..., K] or a 2-D row-strided
    view; w: [N, K] contiguous.  act="swiglu" expects w rows interleaved (gate, up)
    and returns N/2 columns.  ``workspace`` (``splitk_workspace``): used when the
    chosen tile is split-K (else a private one is allocated)."""
    _check(x.is_cuda and w.is_cuda, "linear: tensors must be on the GPU")
    _check(x.dtype in (torch.bfloat16, torch.float16) and w.dtype == x.dtype, "linear: bf16/f16 inputs of equal dtype")
    _check(w.dim() == 2 and w.is_contiguous(), "linear: w must be a contiguous [N, K] matrix")
    N, K = w.shape
    _check(x.shape[-1] == K, f"linear: K mismatch {tuple(x.shape)} vs {tuple(w.shape)}")
    _check(K % 8 == 0, "linear: K must be a multiple of 8")
    if x.dim() == 2 and x.stride(1) == 1:
        x2, lead = x, (x.shape[0],)
    else:
        _check(x.is_contiguous(), "linear: x must be contiguous (or a 2-D row-strided view)")
        lead = tuple(x.shape[:-1])
        x2 = x.reshape(-1, K)
    M = x2.shape[0]
    lda = x2.stride(0)
    _check(lda % 8 == 0 and _aligned(x2) and _aligned(w), "linear: rows must be 16-byte aligned")
    n_out = N // 2 if act == "swiglu" else N
    od = out_dtype or x.dtype
    if out is None:
        out = torch.empty(*lead, n_out, device=x.device, dtype=od)
    _check(out.is_contiguous() and out.shape[-1] == n_out and out.numel() == M * n_out, "linear: bad out")
    if bias is not None:
        _check(bias.is_contiguous() and bias.numel() == N and bias.dtype == x.dtype, "linear: bad bias")
    ldr = 0
    if residual is not None:
        if residual.is_contiguous():
            _check(residual.numel() == M * n_out, "linear: bad residual")
            ldr = n_out
        else:
            _check(residual.dim() == 2 and residual.stride(1) == 1 and residual.shape[0] == M
                   and residual.stride(0) % 4 == 0 and _aligned(residual, 8), "linear: bad strided residual")
            ldr = residual.stride(0)          # 2-D row-strided view (e.g. the CLS rows)
        _check(residual.dtype == x.dtype and residual.shape[-1] == n_out, "linear: bad residual")
    args = (DTYPE_CODE[x.dtype], DTYPE_CODE[od], x2.data_ptr(), lda, w.data_ptr(), K, out.data_ptr(),
            n_out, _ptr(bias), _ptr(residual), ldr, M, N, K, float(alpha), ACT_CODE[act])
    fn = _ops().gemm_tn_sk
    skinny = M <= SKINNY_MAX_M and K % 32 == 0 and act != "swiglu"   # C++ routes these to the skinny-M kernel

    def launch(c: int, ws: Optional[torch.Tensor]) -> None:
        if c >= 0 and splits_of(c) > 1 and ws is None:
            # a split-K choice without a caller workspace: the cached one of this stream
            ws = _private_splitk_ws(x.device, int(_ops().conv_splitk_bytes(M, N, c & 255, splits_of(c))))
        fn(*args, _stream(), int(c), _ptr(ws), 0 if ws is None else ws.numel())

    if tile_cfg < 0 and od != torch.float32 and not skinny:
        key = ("gemm", x.dtype, M, N, K, lda, act, bias is not None, residual is not None)

        def tune_launch(c: int) -> None:
            ws = None
            if splits_of(c) > 1:
                sid = _stream()
                ws = _tune_ws.get(sid)
                if ws is None:
                    ws = _tune_ws[sid] = splitk_workspace(x.device)
            launch(c, ws)
        tile_cfg = _tuned_cfg(key, tune_launch,
                              _gemm_candidates(M, N, K, splitk=True) if act != "swiglu" else _SWIGLU_TILE_CFGS)
    launch(int(tile_cfg), workspace)
    return out


def streamk_workspace(device, grid: int = 192, tile: int = 0) -> torch.Tensor:
    """A zeroed workspace for ``linear_streamk`` (arrival counters + f32 partial
    tiles).  One per stream: two launches must never share one at the same time."""
    n = int(_ops().gemm_sk_workspace_size(int(tile), int(grid)))
    return torch.zeros(n, device=device, dtype=torch.uint8)


def linear_streamk(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: str = "none",
                   residual: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
                   grid: int = 192, tile: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``linear`` on the stream-K ping-pong GEMM (ops/csrc/gemm_sk.h): the
    (tile, K-step) space split evenly over ``grid`` workgroups, split tiles
    finished by their last-arriving segment.  bf16 only, contiguous operands,
    N % 8 == 0.  tile 0 = 256 x 128 (BK 64, 3 stages), 1 = 128 x 128 (BK 64, 4 stages)."""
    _check(x.is_cuda and w.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16,
           "linear_streamk: bf16 GPU tensors")
    _check(w.dim() == 2 and w.is_contiguous() and x.is_contiguous(), "linear_streamk: contiguous x, w")
    N, K = w.shape
    _check(x.shape[-1] == K and K % 8 == 0 and N % 8 == 0, "linear_streamk: shapes")
    _check(act != "swiglu", "linear_streamk: no SwiGLU")
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if out is None:
        out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=x.dtype)
    _check(out.is_contiguous() and out.numel() == M * N, "linear_streamk: bad out")
    if residual is not None:
        _check(residual.is_contiguous() and residual.numel() == M * N and residual.dtype == x.dtype,
               "linear_streamk: bad residual")
    if bias is not None:
        _check(bias.is_contiguous() and bias.numel() == N and bias.dtype == x.dtype, "linear_streamk: bad bias")
    need = int(_ops().gemm_sk_workspace_size(int(tile), int(grid)))
    _check(workspace is not None and workspace.is_cuda and workspace.numel() >= need,
           f"linear_streamk: needs a zeroed workspace of {need} bytes (ops.streamk_workspace)")
    _ops().gemm_sk_bf16(x2.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N, _ptr(bias), _ptr(residual), N, M, N,
                        K, 1.0, ACT_CODE[act], workspace.data_ptr(), int(grid), int(tile), _stream())
    return out


LN_LNA, LN_LNR, LN_STATS, LN_SELF = 1, 2, 4, 8
LN_STG = 32            # gemm_core.h EPI_STG: staged LayerNorm epilogues with per-N-tile partial statistics
STG_TILE_CFGS = (0, 9, 10, 12, 19, 21, 23, 24)   # gemm_core.h kStgTiles
_PSTATS_MAX = 16       # partials per row a producer may write (N / smallest staged BN, N = 768: 768 / 48)


def _pstats_layout(st: torch.Tensor, M: int, what: str):
    """(row stride in floats, partials per row) of a [M, P, 2] f32 partial-statistics view."""
    _check(st.dtype == torch.float32 and st.dim() == 3 and st.shape[0] == M and st.shape[2] == 2
           and st.stride(2) == 1 and st.stride(1) == 2 and st.stride(0) % 2 == 0 and _aligned(st, 8),
           f"{what}: partial statistics must be a [M, P, 2] f32 row-strided view")
    return st.stride(0), st.shape[1]


def _stats_ld(st: torch.Tensor, M: int, what: str) -> int:
    _check(st.dtype == torch.float32 and st.dim() == 2 and st.shape[0] == M and st.shape[1] >= 2
           and st.stride(1) == 1 and st.stride(0) % 2 == 0 and _aligned(st, 8), f"linear_ln: bad {what} stats")
    return st.stride(0)


def linear_ln_staged(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: str = "none",
                     residual: Optional[torch.Tensor] = None, lna: Optional[tuple] = None,
                     lnr: Optional[tuple] = None, pstats: bool = False, out: Optional[torch.Tensor] = None,
                     tile_cfg: int = -1, max_parts: int = _PSTATS_MAX):
    """The deferred-LayerNorm GEMM on the STAGED epilogue with partial statistics
    (gemm_core.h EPI_STG; ping-pong and 4-wave tiles):

    * ``lna=(stats, colsum, bias_f32, D, eps)``: x holds RAW rows whose LayerNorm
      is folded into w (``fold_ln_weights``); ``stats`` [M, P, 2] f32 = the
      producer's per-N-tile partial (sum, sum of squares) of every row.
      y = act(LN(x) @ W.T + b); no ``bias`` / ``residual``.
    * ``lnr=(stats, gamma, beta, D, eps)``: ``residual`` holds RAW rows (partials
      ``stats``), added as LayerNorm(residual).
    * ``pstats=True``: also returns this GEMM's output statistics as partials
      [M, P, 2] (P = N-tiles of the tile it ran): ``(out, stats)``.  No zeroing,
      no atomics: each N-tile writes its own partial.  ``max_parts``: only tiles
      with at most that many N-tiles (a consumer's limit, e.g. 8 for
      ``qkv_attention(a_stats=...)``).
    """
    _check(x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16, "linear_ln_staged: bf16 on the GPU")
    _check(w.dim() == 2 and w.is_contiguous(), "linear_ln_staged: w must be a contiguous [N, K] matrix")
    N, K = w.shape
    _check(x.dim() == 2 and x.stride(1) == 1 and x.shape[1] == K, "linear_ln_staged: x must be a 2-D [M, K] view")
    M, lda = x.shape[0], x.stride(0)
    _check(K % 8 == 0 and lda % 8 == 0 and N % 8 == 0 and _aligned(x) and _aligned(w), "linear_ln_staged: alignment")
    _check(act != "swiglu", "linear_ln_staged: no swiglu")
    mode = LN_STG | (LN_LNA if lna is not None else 0) | (LN_LNR if lnr is not None else 0) | \
        (LN_STATS if pstats else 0)
    _check(mode in (LN_STG | LN_LNA, LN_STG | LN_STATS, LN_STG | LN_LNR | LN_STATS, LN_STG | LN_LNR),
           "linear_ln_staged: modes are lna, pstats, lnr + pstats, lnr")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    _check(out.is_contiguous() and out.shape == (M, N) and _aligned(out), "linear_ln_staged: bad out")
    if bias is not None:
        _check(bias.is_contiguous() and bias.numel() == N and bias.dtype == x.dtype, "linear_ln_staged: bad bias")
    ldr = 0
    if residual is not None:
        _check(residual.dim() == 2 and residual.shape == (M, N) and residual.stride(1) == 1
               and residual.stride(0) % 8 == 0 and residual.dtype == x.dtype and _aligned(residual),
               "linear_ln_staged: bad residual")
        ldr = residual.stride(0)
    a_st = a_cs = a_b = r_st = r_g = r_b = None
    a_ld = r_ld = 0
    a_parts = r_parts = 1
    a_inv = r_inv = 0.0
    eps = 0.0
    if lna is not None:
        a_st, a_cs, a_b, d, eps = lna
        a_ld, a_parts = _pstats_layout(a_st, M, "lna")
        _check(a_cs.dtype == torch.float32 and a_cs.numel() == N and a_cs.is_contiguous()
               and a_b.dtype == torch.float32 and a_b.numel() == N and a_b.is_contiguous(),
               "linear_ln_staged: bad lna vectors")
        a_inv = 1.0 / d
    if lnr is not None:
        _check(residual is not None, "linear_ln_staged: lnr needs the residual")
        r_st, r_g, r_b, d, eps = lnr
        r_ld, r_parts = _pstats_layout(r_st, M, "lnr")
        _check(r_g.numel() == N and r_b.numel() == N and r_g.dtype == x.dtype and r_b.dtype == x.dtype
               and r_g.is_contiguous() and r_b.is_contiguous(), "linear_ln_staged: bad lnr gamma/beta")
        r_inv = 1.0 / d
    o_buf = None
    if pstats:
        o_buf = torch.empty(M, _PSTATS_MAX, 2, device=x.device, dtype=torch.float32)
    fn = _ops().gemm_tn_ln

    def launch(c):
        fn(x.data_ptr(), lda, w.data_ptr(), K, out.data_ptr(), N, _ptr(bias), _ptr(residual), ldr, M, N, K, 1.0,
           ACT_CODE[act], mode, _ptr(a_st), a_ld, _ptr(a_cs), _ptr(a_b), _ptr(r_st), r_ld, _ptr(r_g), _ptr(r_b),
           _ptr(o_buf), 2 * _PSTATS_MAX if pstats else 0, float(a_inv), float(r_inv), float(eps), _stream(), c,
           0, 0, a_parts, r_parts)

    def parts(c):
        return -(-N // int(_ops().gemm_tile_bn(int(_ops().gemm_stg_cfg(int(c))))))

    cands = [c for c in STG_TILE_CFGS if not pstats or parts(c) <= max_parts]
    _check(len(cands) > 0, f"linear_ln_staged: no tile writes <= {max_parts} partials for N = {N}")
    if tile_cfg < 0:
        key = ("gemm_stg", x.dtype, M, N, K, lda, act, mode, a_parts, r_parts) + \
            ((max_parts,) if pstats and max_parts < _PSTATS_MAX else ())
        tile_cfg = _tuned_cfg(key, launch, cands)
    tile_cfg = int(_ops().gemm_stg_cfg(int(tile_cfg)))
    if tile_cfg not in cands:
        tile_cfg = int(_ops().gemm_stg_cfg(int(cands[0])))
    launch(tile_cfg)
    if not pstats:
        return out
    bn = int(_ops().gemm_tile_bn(tile_cfg))
    return out, o_buf[:, : -(-N // bn), :]


def linear_ln(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: str = "none",
              residual: Optional[torch.Tensor] = None, lna: Optional[tuple] = None, lnr: Optional[tuple] = None,
              out_stats: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
              tile_cfg: int = -1) -> torch.Tensor:
    """GEMM with the deferred-LayerNorm epilogues (bf16; ``gemm_ln.hip``).

    * ``lna=(stats, colsum, bias_f32, D, eps)``: x holds RAW rows whose LayerNorm
      is folded into w (w = W * gamma, colsum = w.float().sum(1), bias_f32 =
      b + W @ beta); ``stats`` [M, 2] f32 = per-row (sum, sum of squares).
      y = act(LN(x) @ W.T + b); ``bias`` must be None.  ``stats=None``: the
      GEMM computes x's row statistics itself in its main loop (no producer
      pass) and, if ``out_stats`` is given, STORES them there (for a later
      ``lnr`` of the same rows) -- ``out_stats`` needs no zeroing in this mode.
    * ``lnr=(stats, gamma, beta, D, eps)``: ``residual`` holds raw rows and is
      added as LayerNorm(residual) (normalised on load).
    * ``out_stats`` [M, 2] f32: += per-row (sum, sum of squares) of the stored y
      (must be zeroed by the caller before the first producer writes it).
    """
    _check(x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16, "linear_ln: bf16 on the GPU")
    _check(w.dim() == 2 and w.is_contiguous(), "linear_ln: w must be a contiguous [N, K] matrix")
    N, K = w.shape
    _check(x.dim() == 2 and x.stride(1) == 1 and x.shape[1] == K, "linear_ln: x must be a 2-D [M, K] (row-strided) view")
    M, lda = x.shape[0], x.stride(0)
    _check(K % 8 == 0 and lda % 8 == 0 and N % 4 == 0 and _aligned(x) and _aligned(w), "linear_ln: alignment")
    _check(act != "swiglu", "linear_ln: no swiglu")
    self_stats = lna is not None and lna[0] is None
    if self_stats:
        mode = LN_LNA | LN_SELF
        _check(lnr is None, "linear_ln: lna with in-kernel statistics takes no lnr")
    else:
        mode = (LN_LNA if lna is not None else 0) | (LN_LNR if lnr is not None else 0) | \
            (LN_STATS if out_stats is not None else 0)
    _check(mode in (LN_LNA, LN_STATS, LN_LNR | LN_STATS, LN_LNR, LN_LNA | LN_SELF),
           "linear_ln: modes are lna, out_stats, lnr, lnr + out_stats, or lna with in-kernel statistics")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    _check(out.is_contiguous() and out.shape == (M, N), "linear_ln: bad out")
    if bias is not None:
        _check(bias.is_contiguous() and bias.numel() == N and bias.dtype == x.dtype, "linear_ln: bad bias")
    ldr = 0
    if residual is not None:
        _check(residual.dim() == 2 and residual.shape == (M, N) and residual.stride(1) == 1
               and residual.stride(0) % 4 == 0 and residual.dtype == x.dtype and _aligned(residual, 8),
               "linear_ln: bad residual")
        ldr = residual.stride(0)
    a_st = a_cs = a_b = r_st = r_g = r_b = o_st = None
    a_ld = r_ld = o_ld = 0
    a_inv = r_inv = 0.0
    eps = 0.0
    if lna is not None:
        a_st, a_cs, a_b, d, eps = lna
        a_ld = 0 if a_st is None else _stats_ld(a_st, M, "lna")
        _check(a_cs.dtype == torch.float32 and a_cs.numel() == N and a_cs.is_contiguous()
               and a_b.dtype == torch.float32 and a_b.numel() == N and a_b.is_contiguous(), "linear_ln: bad lna vectors")
        a_inv = 1.0 / d
    if lnr is not None:
        _check(residual is not None, "linear_ln: lnr needs the residual")
        r_st, r_g, r_b, d, eps_r = lnr
        r_ld = _stats_ld(r_st, M, "lnr")
        _check(r_g.numel() == N and r_b.numel() == N and r_g.dtype == x.dtype and r_b.dtype == x.dtype
               and r_g.is_contiguous() and r_b.is_contiguous(), "linear_ln: bad lnr gamma/beta")
        _check(lna is None or eps_r == eps, "linear_ln: one eps")
        r_inv, eps = 1.0 / d, eps_r
    if out_stats is not None:
        o_ld = _stats_ld(out_stats, M, "out")
    args = (x.data_ptr(), lda, w.data_ptr(), K, out.data_ptr(), N, _ptr(bias), _ptr(residual), ldr, M, N, K, 1.0,
            ACT_CODE[act], mode, _ptr(a_st), a_ld, _ptr(a_cs), _ptr(a_b), _ptr(r_st), r_ld, _ptr(r_g), _ptr(r_b),
            _ptr(out_stats), o_ld, float(a_inv), float(r_inv), float(eps))
    fn = _ops().gemm_tn_ln
    if tile_cfg < 0:
        key = ("gemm_ln", x.dtype, M, N, K, lda, act, mode)
        tuned = key in _TUNE
        tile_cfg = _tuned_cfg(key, lambda c: fn(*args, _stream(), c), range(NUM_LN_TILE_CFGS))
        if not tuned and mode & LN_STATS and not torch.cuda.is_current_stream_capturing():
            out_stats.zero_()        # the tuning launches accumulated into it
    fn(*args, _stream(), int(tile_cfg))
    return out


LN_OUT = 16
_LNOUT_ERR: Dict[int, torch.Tensor] = {}


def _lnout_err(dev: torch.device) -> torch.Tensor:
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _LNOUT_ERR:
        _LNOUT_ERR[i] = torch.zeros(1, device=dev, dtype=torch.int32)
    return _LNOUT_ERR[i]


def ln_out_error(device=None, reset: bool = True) -> bool:
    """True if a ``linear_residual_ln`` row-panel wait timed out on ``device``
    since the last reset (its output is then wrong; the kernel never hangs)."""
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    e = _lnout_err(dev)
    bad = bool(e.item())
    if reset and bad:
        e.zero_()
    return bad


def linear_residual_ln(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, residual: torch.Tensor,
                       gamma: torch.Tensor, beta: torch.Tensor, eps: float, stats_ws: torch.Tensor,
                       panel_ws: torch.Tensor, out: Optional[torch.Tensor] = None, tile_cfg: int = -1) -> torch.Tensor:
    """y = LayerNorm(x @ w.T + bias + residual) * gamma + beta in ONE GEMM (bf16;
    gemm_core.h EPI_LNOUT): the blocks of a row panel reduce the row statistics
    through ``stats_ws`` (f32 [M, 2]) and ``panel_ws`` (int32, >= M entries),
    which must be ZERO at launch (one use per zeroing: models/bert.py zeroes a
    forward's workspaces in its embedding kernel).  The post-LN transformer's
    o-proj -> LN1 and FFN-down -> LN2 without a LayerNorm kernel or the pre-LN
    activation round trip."""
    _check(x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == x.dtype, "linear_residual_ln: bf16 on the GPU")
    _check(w.dim() == 2 and w.is_contiguous(), "linear_residual_ln: w must be a contiguous [N, K] matrix")
    N, K = w.shape
    _check(x.dim() == 2 and x.stride(1) == 1 and x.shape[1] == K, "linear_residual_ln: x must be a 2-D [M, K] view")
    M, lda = x.shape[0], x.stride(0)
    _check(K % 8 == 0 and lda % 8 == 0 and N % 8 == 0 and _aligned(x) and _aligned(w), "linear_residual_ln: alignment")
    _check(bias.is_contiguous() and bias.numel() == N and bias.dtype == x.dtype, "linear_residual_ln: bad bias")
    _check(residual.dim() == 2 and residual.shape == (M, N) and residual.stride(1) == 1 and residual.stride(0) % 8 == 0
           and residual.dtype == x.dtype and _aligned(residual), "linear_residual_ln: bad residual")
    for v in (gamma, beta):
        _check(v.is_contiguous() and v.numel() == N and v.dtype == x.dtype and _aligned(v), "linear_residual_ln: gamma/beta")
    _check(stats_ws.dtype == torch.float32 and stats_ws.is_contiguous() and stats_ws.numel() >= 2 * M
           and _aligned(stats_ws, 8), "linear_residual_ln: stats_ws must be contiguous f32 [M, 2]")
    _check(panel_ws.dtype == torch.int32 and panel_ws.is_contiguous() and panel_ws.numel() >= M,
           "linear_residual_ln: panel_ws must be contiguous int32 with >= M entries")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    _check(out.is_contiguous() and out.shape == (M, N) and _aligned(out), "linear_residual_ln: bad out")
    err = _lnout_err(x.device)
    fn = _ops().gemm_tn_ln

    def launch(c):
        fn(x.data_ptr(), lda, w.data_ptr(), K, out.data_ptr(), N, bias.data_ptr(), residual.data_ptr(),
           residual.stride(0), M, N, K, 1.0, 0, LN_OUT, 0, 0, 0, 0, 0, 0, gamma.data_ptr(), beta.data_ptr(),
           stats_ws.data_ptr(), 2, 0.0, 1.0 / N, float(eps), _stream(), int(c), panel=panel_ws.data_ptr(),
           err=err.data_ptr())

    if tile_cfg < 0:
        key = ("gemm_lnout", M, N, K, lda)
        tuned = key in _TUNE
        tile_cfg = _tuned_cfg(key, launch, range(NUM_LN_TILE_CFGS))
        if not tuned and not torch.cuda.is_current_stream_capturing():
            stats_ws.zero_()         # the tuning launches used (and left) the workspaces
            panel_ws.zero_()
    launch(tile_cfg)
    return out


def linear_rowln_supported(M: int, N: int, K: int) -> bool:
    """Shapes the full-row GEMM + LayerNorm kernel (``gemm_rowln.hip``) takes."""
    return N == 768 and K % 32 == 0 and M > 0


def pack_rowln_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] weight -> the k-tile-major [K/32, N, 32] layout ``linear_rowln`` reads
    (each 32-wide k-step of all N rows contiguous).  Done once per weight."""
    N, K = w.shape
    _check(K % 32 == 0, "pack_rowln_weight: K must be a multiple of 32")
    return w.reshape(N, K // 32, 32).permute(1, 0, 2).contiguous()


def linear_rowln(x: torch.Tensor, wp: torch.Tensor, bias: torch.Tensor, residual: torch.Tensor,
                 gamma: torch.Tensor, beta: torch.Tensor, eps: float,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = LayerNorm(x @ w.T + bias + residual) * gamma + beta (bf16, N = 768) in ONE
    kernel whose 64-row blocks own whole output rows (``gemm_rowln.hip``): the row
    statistics never leave the block -- no workspace, no zeroing, no cross-block
    wait, no LayerNorm launch.  ``wp`` = ``pack_rowln_weight(w)``.  The post-LN
    transformer's o-proj -> LN1 and FFN-down -> LN2."""
    _check(x.is_cuda and x.dtype == torch.bfloat16 and wp.dtype == x.dtype, "linear_rowln: bf16 on the GPU")
    _check(wp.dim() == 3 and wp.shape[2] == 32 and wp.is_contiguous(),
           "linear_rowln: wp must be pack_rowln_weight(w), [K/32, N, 32]")
    N, K = wp.shape[1], wp.shape[0] * 32
    _check(x.dim() == 2 and x.stride(1) == 1 and x.shape[1] == K, "linear_rowln: x must be a 2-D [M, K] view")
    M, lda = x.shape[0], x.stride(0)
    _check(linear_rowln_supported(M, N, K), f"linear_rowln: unsupported shape M={M} N={N} K={K}")
    _check(lda % 8 == 0 and _aligned(x) and _aligned(wp), "linear_rowln: x / w rows must be 16-byte aligned")
    _check(bias.is_contiguous() and bias.numel() == N and bias.dtype == x.dtype and _aligned(bias, 8),
           "linear_rowln: bad bias")
    _check(residual.dim() == 2 and residual.shape == (M, N) and residual.stride(1) == 1
           and residual.stride(0) % 4 == 0 and residual.dtype == x.dtype and _aligned(residual, 8),
           "linear_rowln: bad residual")
    for v in (gamma, beta):
        _check(v.is_contiguous() and v.numel() == N and v.dtype == x.dtype and _aligned(v, 8), "linear_rowln: gamma/beta")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    _check(out.dim() == 2 and out.shape == (M, N) and out.stride(1) == 1 and out.stride(0) % 4 == 0
           and _aligned(out, 8), "linear_rowln: bad out")
    _ops().gemm_rowln(x.data_ptr(), lda, wp.data_ptr(), bias.data_ptr(), residual.data_ptr(), residual.stride(0),
                      gamma.data_ptr(), beta.data_ptr(), out.data_ptr(), out.stride(0), M, N, K, float(eps), _stream())
    return out


def linear_residual_ln_ref(x, w, bias, residual, gamma, beta, eps=1e-12):
    y = x.float() @ w.float().t() + bias.float() + residual.float()
    return F.layer_norm(y, (y.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def fold_ln_weights(w: torch.Tensor, b: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor):
    """(w', colsum, bias_f32) for ``linear_ln(lna=...)``: LN(x) @ w.T + b ==
    rstd * (x @ w'.T - mean * colsum) + bias_f32 with w' = w * gamma."""
    wf = w.float()
    w2 = (wf * gamma.float()[None, :]).to(w.dtype).contiguous()
    return w2, w2.float().sum(1).contiguous(), (b.float() + wf @ beta.float()).contiguous()


def linear_ln_ref(x, w, bias=None, act="none", residual=None, ln_x=None, ln_res=None, eps=1e-12):
    """fp32 reference of linear_ln in terms of the UNFOLDED LayerNorms:
    act(LN_x(x) @ w.T + bias + LN_res(residual)); ln_* = (gamma, beta) or None."""
    xf = x.float()
    if ln_x is not None:
        xf = F.layer_norm(xf, (xf.shape[-1],), ln_x[0].float(), ln_x[1].float(), eps)
    y = xf @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if residual is not None:
        rf = residual.float()
        if ln_res is not None:
            rf = F.layer_norm(rf, (rf.shape[-1],), ln_res[0].float(), ln_res[1].float(), eps)
        y = y + rf
    return _act_ref(y, act)


def _act_ref(y: torch.Tensor, act: str) -> torch.Tensor:
    if act == "gelu":
        return F.gelu(y)
    if act == "gelu_tanh":
        return F.gelu(y, approximate="tanh")
    if act == "relu":
        return F.relu(y)
    if act == "tanh":
        return torch.tanh(y)
    if act == "silu":
        return F.silu(y)
    if act == "sigmoid":
        return torch.sigmoid(y)
    return y


def linear_ref(x, w, bias=None, act="none", residual=None, out_dtype=None, alpha=1.0):
    y = alpha * (x.float() @ w.float().t())
    if bias is not None:
        y = y + bias.float()
    if act == "swiglu":
        g, u = y[..., 0::2], y[..., 1::2]
        y = F.silu(g) * u
        if residual is not None:
            y = y + residual.float()
    else:
        if residual is not None:
            y = y + residual.float()
        y = _act_ref(y, act)
    return y.to(out_dtype or x.dtype)


# ---------------------------------------------------------------------------
# Norms
# ---------------------------------------------------------------------------
def _norm(x, gamma, beta, eps, residual, residual_out, mode):
    _check(x.is_cuda and x.dtype in (torch.bfloat16, torch.float16), "norm: bad x")
    D = x.shape[-1]
    if x.is_contiguous():
        rows, ldx = x.numel() // D, D
    else:
        # a 2-D row-strided view (e.g. the [CLS] rows): read in place
        _check(x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 4 == 0 and _aligned(x, 8)
               and residual is None, "norm: x must be contiguous or a 2-D row-strided view without residual")
        rows, ldx = x.shape[0], x.stride(0)
    _check(D % 4 == 0 and D <= 8192, "norm: D must be a multiple of 4, <= 8192")
    _check(gamma.numel() == D and gamma.dtype == x.dtype, "norm: bad gamma")
    if beta is not None:
        _check(beta.numel() == D and beta.dtype == x.dtype, "norm: bad beta")
    if residual is not None:
        _check(residual.shape == x.shape and residual.is_contiguous() and residual.dtype == x.dtype, "norm: bad residual")
    if residual_out is not None:
        _check(residual_out.shape == x.shape and residual_out.is_contiguous(), "norm: bad residual_out")
    y = torch.empty(x.shape, device=x.device, dtype=x.dtype)
    _ops().norm_fwd(DTYPE_CODE[x.dtype], mode, x.data_ptr(), _ptr(residual), _ptr(residual_out),
                    gamma.data_ptr(), _ptr(beta), y.data_ptr(), rows, D, ldx, float(eps), _stream())
    return y


def layer_norm(x, gamma, beta, eps=1e-12, residual=None, residual_out=None):
    """LayerNorm(x [+ residual]) (optionally also writing x + residual)."""
    return _norm(x, gamma, beta, eps, residual, residual_out, 0)


def rms_norm(x, gamma, eps=1e-5, residual=None, residual_out=None):
    return _norm(x, gamma, None, eps, residual, residual_out, 1)


def layer_norm_ref(x, gamma, beta, eps=1e-12, residual=None):
    xf = x.float() + (residual.float() if residual is not None else 0)
    return F.layer_norm(xf, (x.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def rms_norm_ref(x, gamma, eps=1e-5, residual=None):
    xf = x.float() + (residual.float() if residual is not None else 0)
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()).to(x.dtype)


def embed_ln(ids, word, pos, typ, gamma, beta, eps=1e-12, types=None, zero_stats=None):
    """BERT embeddings: LN(word[ids] + pos[t % S] + type[types or 0]); ids [B, S] int32.
    ``zero_stats`` [..., B*S, 2] f32 (contiguous): also zeroed (the deferred-LN
    row statistics of the folded forward), saving a fill kernel."""
    _check(ids.dtype == torch.int32 and ids.is_contiguous() and ids.dim() == 2, "embed_ln: ids must be [B, S] int32")
    B, S = ids.shape
    D = word.shape[1]
    _check(pos.shape[0] >= S and pos.shape[1] == D and typ.shape[1] == D, "embed_ln: table shapes")
    _check(D % 256 == 0, "embed_ln: hidden size must be a multiple of 256")
    if types is not None:
        _check(types.dtype == torch.int32 and types.shape == ids.shape and types.is_contiguous(), "embed_ln: bad types")
    zn = 0
    if zero_stats is not None:
        _check(zero_stats.dtype == torch.float32 and zero_stats.is_contiguous() and zero_stats.shape[-1] == 2
               and zero_stats.shape[-2] == B * S, "embed_ln: zero_stats must be [..., B*S, 2] f32")
        zn = zero_stats.numel() // (2 * B * S)
    y = torch.empty(B * S, D, device=ids.device, dtype=word.dtype)
    _ops().embed_ln_fwd(DTYPE_CODE[word.dtype], ids.data_ptr(), _ptr(types), word.data_ptr(), pos.data_ptr(),
                        typ.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), B * S, S, D,
                        word.shape[0], float(eps), _ptr(zero_stats), zn, B * S, _stream())
    return y


def embed_ln_ref(ids, word, pos, typ, gamma, beta, eps=1e-12, types=None):
    B, S = ids.shape
    idl = ids.long().clamp(0, word.shape[0] - 1)
    x = word.float()[idl] + pos.float()[:S][None] + typ.float()[(types.long() if types is not None else torch.zeros_like(idl))]
    return F.layer_norm(x, (word.shape[1],), gamma.float(), beta.float(), eps).to(word.dtype).reshape(B * S, -1)


def seq_lens(ids: torch.Tensor, pad_id: int = 0) -> torch.Tensor:
    """int32 [B]: number of non-pad ids per row of ``ids`` [B, S] int32 (min 1)."""
    _check(ids.is_cuda and ids.dtype == torch.int32 and ids.dim() == 2 and ids.is_contiguous(), "seq_lens: ids")
    B, S = ids.shape
    lens = torch.empty(B, device=ids.device, dtype=torch.int32)
    _ops().seq_lens(ids.data_ptr(), B, S, int(pad_id), lens.data_ptr(), _stream())
    return lens


def seq_lens_ref(ids, pad_id=0):
    return (ids != pad_id).sum(dim=1, dtype=torch.int32).clamp_(min=1)


# ---------------------------------------------------------------------------
# Attention
# ---------------------------------------------------------------------------
def attention(qkv: torch.Tensor, B: int, S: int, H: int, Hkv: int, D: int, lens: Optional[torch.Tensor] = None,
              causal: bool = False, scale: Optional[float] = None, out: Optional[torch.Tensor] = None,
              q_off: int = 0, k_off: Optional[int] = None, v_off: Optional[int] = None) -> torch.Tensor:
    """Fused MHA / GQA on the packed projection output qkv [B*S, ld] (q | k | v)."""
    _check(qkv.is_cuda and qkv.dtype in (torch.bfloat16, torch.float16) and qkv.dim() == 2 and qkv.stride(1) == 1,
           "attention: bad qkv")
    _check(qkv.shape[0] == B * S, "attention: qkv rows must be B*S")
    _check(D in (64, 128), "attention: head dim must be 64 or 128")
    _check(H % Hkv == 0, "attention: H % Hkv")
    k_off = H * D if k_off is None else k_off
    v_off = (H + Hkv) * D if v_off is None else v_off
    ld = qkv.stride(0)
    _check(max(q_off + H * D, k_off + Hkv * D, v_off + Hkv * D) <= qkv.shape[1], "attention: offsets exceed row")
    _check(ld % 8 == 0 and q_off % 8 == 0 and k_off % 8 == 0 and v_off % 8 == 0 and _aligned(qkv), "attention: alignment")
    if lens is not None:
        _check(lens.dtype == torch.int32 and lens.numel() == B and lens.is_cuda, "attention: lens must be int32 [B]")
    if out is None:
        out = torch.empty(B * S, H * D, device=qkv.device, dtype=qkv.dtype)
    _check(out.is_contiguous() and out.shape == (B * S, H * D), "attention: bad out")
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    _ops().attn_fwd(DTYPE_CODE[qkv.dtype], qkv.data_ptr(), ld, q_off, k_off, v_off, B, H, Hkv, S, D, _ptr(lens), int(causal),
                    out.data_ptr(), H * D, float(scale), _stream())
    return out


NUM_QKV_ATTN_CFGS = 5   # qkv_attention.hip: 8 waves (4x2) x 3 stages, 8 (4x2) x 2, 4 x 2, 8 (2x4) x 2, two sequences per block (S == 128)
QKV_ATTN_MAX_S = 128


def pack_qkv_heads(w: torch.Tensor, b: torch.Tensor, H: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """[q | k | v] projection rows (nn.Linear [3*H*D, K] layout) -> head-major
    [H*3*D, K]: rows h*3D + [0,D) = q_h, [D,2D) = k_h, [2D,3D) = v_h (and the
    bias likewise) -- the operand layout of ``qkv_attention``."""
    N, K = w.shape
    _check(N % (3 * H) == 0 and b.numel() == N, "pack_qkv_heads: rows must be 3*H*D")
    D = N // (3 * H)
    wp = w.view(3, H, D, K).transpose(0, 1).reshape(N, K).contiguous()
    bp = b.view(3, H, D).transpose(0, 1).reshape(N).contiguous()
    return wp, bp


def pack_qkv_vec(v: torch.Tensor, H: int) -> torch.Tensor:
    """A per-output-row vector of the [q | k | v] projection (bias, folded
    colsum / bias) in ``pack_qkv_heads`` order."""
    N = v.numel()
    _check(N % (3 * H) == 0, "pack_qkv_vec: length must be 3*H*D")
    return v.view(3, H, N // (3 * H)).transpose(0, 1).reshape(N).contiguous()


def qkv_attention_supported(S: int, H: int, D: int, K: int) -> bool:
    return 1 <= S <= QKV_ATTN_MAX_S and D == 64 and K % 8 == 0


def qkv_attention(x: torch.Tensor, w_packed: torch.Tensor, b_packed: Optional[torch.Tensor], B: int, S: int, H: int,
                  lens: Optional[torch.Tensor] = None, scale: Optional[float] = None,
                  out: Optional[torch.Tensor] = None, cfg: int = -1, lna: Optional[tuple] = None,
                  stats_out: Optional[torch.Tensor] = None, key_ids: Optional[tuple] = None,
                  a_stats: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused QKV projection + bidirectional attention (qkv_attention.hip):
    ctx [B*S, H*64] = MHA(x @ W^T + b) for S <= 128, head dim 64, with the
    projection weight in ``pack_qkv_heads`` layout.  The [B*S, 3*H*64] QKV
    activation is never materialised.

    Key lengths: ``lens`` (int32 [B], e.g. ``seq_lens``) or ``key_ids=(ids,
    pad_id)`` -- the kernel counts each sequence's non-pad tokens itself
    (right padding, as ``seq_lens``), so no lengths kernel runs.

    ``lna=(colsum, bias_f32, eps)`` (packed order, f32): x holds RAW rows whose
    LayerNorm is folded into ``w_packed`` (``fold_ln_weights`` then packing);
    the kernel computes each row's statistics itself and, with ``stats_out``
    [B*S, 2] f32, stores (sum, sum of squares) for a later ``linear_ln(lnr=...)``.
    ``b_packed`` must then be None.  ``a_stats`` [B*S, P, 2] f32 (P <= 8, row-
    strided view): the producer's per-N-tile partial statistics of x
    (``linear_ln(..., pstats=True)``) -- the kernel sums them instead of
    computing statistics in its main loop."""
    _check(x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.dim() == 2 and x.stride(1) == 1,
           "qkv_attention: x must be a 2-D [B*S, K] (row-strided) bf16/f16 view")
    N, K = w_packed.shape
    _check(w_packed.dtype == x.dtype and w_packed.is_contiguous(), "qkv_attention: weight dtype and layout")
    cs = bf = None
    eps = 0.0
    if lna is not None:
        cs, bf, eps = lna
        _check(b_packed is None, "qkv_attention: the folded form takes its bias from lna")
        _check(all(v.dtype == torch.float32 and v.is_contiguous() and v.numel() == N and _aligned(v) for v in (cs, bf)),
               "qkv_attention: lna colsum / bias must be contiguous f32 [H*192]")
        if stats_out is not None:
            _check(stats_out.dtype == torch.float32 and stats_out.is_contiguous() and stats_out.shape == (B * S, 2),
                   "qkv_attention: stats_out must be contiguous f32 [B*S, 2]")
    else:
        _check(b_packed is not None and b_packed.dtype == x.dtype and b_packed.is_contiguous()
               and b_packed.numel() == N and _aligned(b_packed, 8), "qkv_attention: bias dtype / layout")
        _check(stats_out is None, "qkv_attention: stats_out needs lna")
    _check(x.shape == (B * S, K), f"qkv_attention: x must be [B*S, K] = [{B * S}, {K}], got {tuple(x.shape)}")
    _check(N == H * 192, "qkv_attention: packed weight must be [H*3*64, K]")
    _check(qkv_attention_supported(S, H, 64, K), "qkv_attention: S <= 128, head dim 64, K % 8 == 0")
    _check(x.stride(0) % 8 == 0 and _aligned(x) and _aligned(w_packed), "qkv_attention: alignment")
    if lens is not None:
        _check(lens.dtype == torch.int32 and lens.numel() == B and lens.is_cuda, "qkv_attention: lens must be int32 [B]")
    kid, pad = None, 0
    if key_ids is not None:
        kid, pad = key_ids
        _check(lens is None, "qkv_attention: pass lens or key_ids, not both")
        _check(kid.dtype == torch.int32 and kid.is_cuda and kid.is_contiguous() and tuple(kid.shape) == (B, S),
               "qkv_attention: key_ids must be contiguous int32 [B, S] on the GPU")
    if out is None:
        out = torch.empty(B * S, H * 64, device=x.device, dtype=x.dtype)
    _check(out.is_contiguous() and out.shape == (B * S, H * 64) and _aligned(out), "qkv_attention: bad out")
    scale = 1.0 / 8.0 if scale is None else scale
    args = (DTYPE_CODE[x.dtype], x.data_ptr(), x.stride(0), w_packed.data_ptr(), _ptr(b_packed), B, S, H, K,
            _ptr(lens), out.data_ptr(), H * 64, float(scale))
    a_ld = a_parts = 0
    if a_stats is not None:
        _check(lna is not None and stats_out is None, "qkv_attention: a_stats needs lna and no stats_out")
        a_ld, a_parts = _pstats_layout(a_stats, B * S, "qkv_attention a_stats")
        _check(a_parts <= 8, "qkv_attention: at most 8 partials per row")
    extra = (_ptr(cs), _ptr(bf), _ptr(stats_out), float(eps), _ptr(kid), int(pad), _ptr(a_stats), a_ld, a_parts)
    fn = _ops().qkv_attn_fwd
    if cfg < 0:
        key = ("qkv_attn", x.dtype, B, S, H, K, x.stride(0), lna is not None) + (("pstats",) if a_stats is not None else ())
        cfg = _tuned_cfg(key, lambda c: fn(*args, c, _stream(), *extra), range(NUM_QKV_ATTN_CFGS))
    fn(*args, int(cfg), _stream(), *extra)
    return out


def qkv_attention_ref(x, w, b, B, S, H, lens=None, scale=None):
    """Unfused fp32 reference with the UNPACKED [q | k | v] weight; the projection
    is rounded to x's dtype like the two-kernel path."""
    qkv = F.linear(x.float(), w.float(), b.float()).to(x.dtype)
    return attention_ref(qkv, B, S, H, H, w.shape[0] // (3 * H), lens=lens, scale=scale)


def attention_ref(qkv, B, S, H, Hkv, D, lens=None, causal=False, scale=None, q_off=0, k_off=None, v_off=None):
    k_off = H * D if k_off is None else k_off
    v_off = (H + Hkv) * D if v_off is None else v_off
    x = qkv.float()
    q = x[:, q_off:q_off + H * D].reshape(B, S, H, D).transpose(1, 2)
    k = x[:, k_off:k_off + Hkv * D].reshape(B, S, Hkv, D).transpose(1, 2)
    v = x[:, v_off:v_off + Hkv * D].reshape(B, S, Hkv, D).transpose(1, 2)
    if Hkv != H:
        k = k.repeat_interleave(H // Hkv, dim=1)
        v = v.repeat_interleave(H // Hkv, dim=1)
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    s = (q @ k.transpose(-1, -2)) * scale
    keys = torch.arange(S, device=qkv.device)
    mask = torch.zeros(B, 1, S, S, dtype=torch.bool, device=qkv.device)
    if lens is not None:
        mask |= (keys[None, None, None, :] >= lens.long()[:, None, None, None])
    if causal:
        mask |= keys[None, None, None, :] > keys[None, None, :, None]
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    o = (p @ v).transpose(1, 2).reshape(B * S, H * D)
    return o.to(qkv.dtype)


# ---------------------------------------------------------------------------
# Heads / misc
# ---------------------------------------------------------------------------
def softmax_topk(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    _check(logits.is_cuda and logits.dtype == torch.float32 and logits.dim() == 2 and logits.is_contiguous(),
           "softmax_topk: logits must be contiguous f32 [B, C]")
    B, C = logits.shape
    _check(C <= 4096 and 1 <= k <= min(16, C), "softmax_topk: C <= 4096 and 1 <= k <= 16")
    probs = torch.empty(B, k, device=logits.device, dtype=torch.float32)
    idx = torch.empty(B, k, device=logits.device, dtype=torch.int32)
    _ops().softmax_topk(logits.data_ptr(), B, C, k, probs.data_ptr(), idx.data_ptr(), _stream())
    return probs, idx


def softmax_topk_packed(logits: torch.Tensor, k: int) -> torch.Tensor:
    """softmax + top-k written as the serving output row [k probs | k class ids
    as f32] ([B, 2k]) by the kernel itself (no cat / cast kernels)."""
    _check(logits.is_cuda and logits.dtype == torch.float32 and logits.dim() == 2 and logits.is_contiguous(),
           "softmax_topk: logits must be contiguous f32 [B, C]")
    B, C = logits.shape
    _check(C <= 4096 and 1 <= k <= min(16, C), "softmax_topk: C <= 4096 and 1 <= k <= 16")
    out = torch.empty(B, 2 * k, device=logits.device, dtype=torch.float32)
    _ops().softmax_topk(logits.data_ptr(), B, C, k, out.data_ptr(), 0, _stream())
    return out


def softmax_topk_ref(logits, k):
    p = torch.softmax(logits.float(), dim=-1)
    v, i = torch.topk(p, k, dim=-1)
    return v, i.to(torch.int32)


def rope_tables(max_pos: int, D: int, theta: float = 500000.0, device=None):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_(qkv, cos, sin, B, S, H, Hkv, D, q_off=0, k_off=None, pos_offset=0):
    """In-place rotary embedding of the q and k heads of qkv [B*S, ld]."""
    _check(qkv.is_cuda and qkv.dtype == torch.bfloat16 and qkv.dim() == 2 and qkv.stride(1) == 1, "rope: bad qkv")
    _check(cos.dtype == torch.float32 and cos.shape[1] == D // 2 and cos.shape[0] >= S + pos_offset, "rope: bad tables")
    k_off = H * D if k_off is None else k_off
    _ops().rope(qkv.data_ptr(), qkv.stride(0), q_off, k_off, H, Hkv, D, S, cos.data_ptr(), sin.data_ptr(),
                B * S, pos_offset, _stream())
    return qkv


def rope_ref(qkv, cos, sin, B, S, H, Hkv, D, q_off=0, k_off=None, pos_offset=0):
    k_off = H * D if k_off is None else k_off
    x = qkv.float().clone()
    pos = (torch.arange(B * S, device=qkv.device) % S) + pos_offset
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]

    def rot(a):
        a1, a2 = a[..., : D // 2], a[..., D // 2:]
        return torch.cat([a1 * c - a2 * s, a2 * c + a1 * s], dim=-1)

    x[:, q_off:q_off + H * D] = rot(x[:, q_off:q_off + H * D].reshape(-1, H, D)).reshape(-1, H * D)
    x[:, k_off:k_off + Hkv * D] = rot(x[:, k_off:k_off + Hkv * D].reshape(-1, Hkv, D)).reshape(-1, Hkv * D)
    return x.to(qkv.dtype)


def gather_rows(src_ptrs: torch.Tensor, n: int, rows: int, row_bytes: int, dst: torch.Tensor):
    _ops().gather_rows(src_ptrs.data_ptr(), n, rows, row_bytes, dst.data_ptr(), _stream())


def image_to_nhwc(img_u8: torch.Tensor, Cp: int = 8) -> torch.Tensor:
    """uint8 [N, H, W, 3] -> normalised f16 [N, H, W, Cp] (ImageNet mean/std)."""
    _check(img_u8.is_cuda and img_u8.dtype == torch.uint8 and img_u8.is_contiguous() and img_u8.shape[-1] == 3, "image_to_nhwc: bad input")
    N, H, W, _ = img_u8.shape
    out = torch.empty(N, H, W, Cp, device=img_u8.device, dtype=torch.float16)
    _ops().image_to_nhwc(img_u8.data_ptr(), N, H * W, Cp, out.data_ptr(), _stream())
    return out


def image_to_s2d(img_u8: torch.Tensor, zero: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 [N, H, W, 3] -> normalised f16 space-to-depth [N, H/2, W/2, 16]
    (channel (dy*2+dx)*3 + c = pixel (2i+dy, 2j+dx) channel c; 12..15 zero).
    ``zero``: a split-K workspace (``splitk_workspace(..., zeroed=False)``) whose
    counter header the same kernel zeroes -- no separate memset per forward."""
    _check(img_u8.is_cuda and img_u8.dtype == torch.uint8 and img_u8.is_contiguous() and img_u8.shape[-1] == 3,
           "image_to_s2d: bad input")
    N, H, W, _ = img_u8.shape
    _check(H % 2 == 0 and W % 4 == 0, "image_to_s2d: H must be even and W a multiple of 4")
    out = torch.empty(N, H // 2, W // 2, 16, device=img_u8.device, dtype=torch.float16)
    zb = 0
    if zero is not None:
        _check(zero.is_cuda and zero.dtype == torch.uint8 and zero.numel() >= SPLITK_HEADER and _aligned(zero),
               "image_to_s2d: zero must be a split-K workspace")
        zb = SPLITK_HEADER
    _ops().image_to_s2d(img_u8.data_ptr(), N, H, W, out.data_ptr(), _ptr(zero), zb, _stream())
    return out


def stem_s2d_pool(img_u8: torch.Tensor, w_s2d: torch.Tensor, bias: torch.Tensor,
                  zero: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The ResNet stem in one kernel (ops/csrc/cnn_stem.hip): uint8 [N, H, W, 3]
    -> normalise -> space-to-depth -> 4x4 conv with ``w_s2d`` [64, 4, 4, 16]
    (``stem_weight_s2d``) + bias + ReLU -> 3x3 / stride-2 max-pool (pad 1) ->
    f16 [N, H/4, W/4, 64].  H, W multiples of 32.  ``zero``: a split-K workspace
    whose counter header the kernel zeroes on the side."""
    _check(img_u8.is_cuda and img_u8.dtype == torch.uint8 and img_u8.is_contiguous() and img_u8.shape[-1] == 3,
           "stem_s2d_pool: bad image")
    N, H, W, _ = img_u8.shape
    _check(H % 32 == 0 and W % 32 == 0, "stem_s2d_pool: H and W must be multiples of 32")
    _check(w_s2d.shape == (64, 4, 4, 16) and w_s2d.dtype == torch.float16 and w_s2d.is_contiguous()
           and bias.numel() == 64 and bias.dtype == torch.float16 and _aligned(w_s2d), "stem_s2d_pool: bad weights")
    out = torch.empty(N, H // 4, W // 4, 64, device=img_u8.device, dtype=torch.float16)
    zb = 0
    if zero is not None:
        _check(zero.is_cuda and zero.dtype == torch.uint8 and zero.numel() >= SPLITK_HEADER and _aligned(zero),
               "stem_s2d_pool: zero must be a split-K workspace")
        zb = SPLITK_HEADER
    _ops().stem_s2d_pool(img_u8.data_ptr(), N, H, W, w_s2d.data_ptr(), bias.data_ptr(), out.data_ptr(), _ptr(zero),
                         zb, _stream())
    return out


def image_to_s2d_ref(img_u8):
    x = image_to_nhwc_ref(img_u8, 3).float()                       # [N, H, W, 3]
    N, H, W, _ = x.shape
    x = x.view(N, H // 2, 2, W // 2, 2, 3).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 12)
    return torch.cat([x, torch.zeros(N, H // 2, W // 2, 4, device=x.device)], -1).half()


def stem_weight_s2d(w: torch.Tensor) -> torch.Tensor:
    """7x7 stride-2 pad-3 conv weights [K, 7, 7, 3] -> the equivalent 4x4 stride-1
    pad-2 conv on the space-to-depth input, [K, 4, 4, 16]: input row 2(p-2+bi)+dy
    is tap r = 2*bi + dy - 1 of output row p (taps outside 0..6 are zero)."""
    K = w.shape[0]
    out = torch.zeros(K, 4, 4, 16, dtype=w.dtype, device=w.device)
    for bi in range(4):
        for bj in range(4):
            for dy in range(2):
                for dx in range(2):
                    r, c = 2 * bi + dy - 1, 2 * bj + dx - 1
                    if 0 <= r < 7 and 0 <= c < 7:
                        ch = (dy * 2 + dx) * 3
                        out[:, bi, bj, ch:ch + 3] = w[:, r, c, :3]
    return out.contiguous()


def image_to_nhwc_ref(img_u8, Cp=8):
    mean = torch.tensor([0.485, 0.456, 0.406], device=img_u8.device)
    std = torch.tensor([0.229, 0.224, 0.225], device=img_u8.device)
    x = (img_u8.float() / 255.0 - mean) / std
    pad = torch.zeros(*x.shape[:-1], Cp - 3, device=x.device)
    return torch.cat([x, pad], -1).half()


# ---------------------------------------------------------------------------
# Convolution family (NHWC f16)
# ---------------------------------------------------------------------------
# RDB_CONV1X1_GEMM=0 keeps 1x1 convolutions off the dense `linear` tiles
_CONV1X1_GEMM = os.environ.get("RDB_CONV1X1_GEMM", "1") != "0"
# RDB_CONV_SPLITK=0: no split-K candidates
_CONV_SPLITK = os.environ.get("RDB_CONV_SPLITK", "1") != "0"
# RDB_GEMM_SPLITK=0: no split-K candidates for the dense GEMM (linear)
_GEMM_SPLITK = os.environ.get("RDB_GEMM_SPLITK", "1") != "0"
# RDB_GEMM_DEEP=0: no DEEP (one block per CU, many LDS stages) tile candidates
_GEMM_DEEP = os.environ.get("RDB_GEMM_DEEP", "1") != "0"
# Encoded conv tile choices (what the tuner / tile tables store):
#   cfg                  4-wave tile cfg (0..12) of the implicit-GEMM conv kernel
#   cfg | splits << 8    the same tile, split-K over `splits` workgroups per tile
#   CONV_LINEAR | cfg    (1x1 / stride 1) the dense GEMM `linear` on tile cfg (0..25)
#   ... | DEEP           tiles 0, 1, 2, 3, 9, 10 with one block per CU and up to 8 LDS stages
CONV_LINEAR = 1 << 16
#   CONV_PP | v [| splits << 8]   (R x S / strided convs, C % BK == 0, with bias) the
#                        8-wave ping-pong kernel with the im2col operand, tile v (conv.hip)
CONV_PP = 1 << 17
_CONV_PP_BM = (256, 128, 256, 256, 128)          # conv.hip kConvPPBM / BN / BK
_CONV_PP_BN = (128, 256, 128, 64, 128)
_CONV_PP_BK = (64, 64, 32, 64, 32)
# RDB_CONV_PP=0: no ping-pong conv candidates
_CONV_PP = os.environ.get("RDB_CONV_PP", "1") != "0"
#   CONV_HALO | v        (3x3, stride 1, pad 1, C % 64 == 0, with bias) the halo-tile kernel,
#                        tile v (conv_halo.hip): one LDS patch feeds all 9 taps
CONV_HALO = 1 << 18
_CONV_HALO_BM = (256, 112, 112, 64, 224, 224, 64, 128, 256, 256, 64, 64)    # conv_halo.hip kHaloBM / kHaloBN
_CONV_HALO_BN = (64, 64, 64, 64, 64, 128, 64, 32, 64, 64, 128, 64)
_CONV_HALO_RW = (6, 7, 8)          # persistent resident-weight tiles: no residual, ReLU / none (stride 1)
_CONV_HALO_SK = (2, 3, 4, 5, 9, 10, 11)   # two-patch-buffer streamed tiles: split-K over the 64-channel blocks
# RDB_CONV_HALO=0: no halo-tile conv candidates
_CONV_HALO = os.environ.get("RDB_CONV_HALO", "1") != "0"
DEEP = 1 << 12                        # gemm_core.h kDeepFlag: one block per CU, up to 8 LDS stages
_DEEP_TILES = (0, 1, 2, 3, 9, 10, 6, 7)
_DEEP_BIG = (6, 7)                    # 256x128 / 128x256: one block per CU at any grid size
_DEEP_MAX_BLOCKS = 320                # DEEP candidates only where the grid is ~one block per CU
SPLITK_HEADER = 65536                 # gemm_core.h kSplitKHeader (tile arrival counters)
SPLITK_WS_BYTES = 40 << 20            # one forward's split-K workspace (ops.splitk_workspace)
_SPLITS = (2, 3, 4, 6, 8)
_PP_SPLITK_TILES = (19, 21)           # ping-pong tiles with a split-K instantiation (BK 64, gemm_core.h splitk_epi)
_TILE_BM = (128, 64, 128, 64, 128, 192, 256, 128, 128, 64, 128, 256, 128)   # gemm_core.h kTileBM/BN, 4-wave tiles
_TILE_BN = (128, 128, 64, 64, 192, 128, 128, 256, 144, 96, 96, 144, 48)
_tune_ws: Dict[int, torch.Tensor] = {}
_priv_ws: Dict[tuple, torch.Tensor] = {}
_cap_ws_local = threading.local()    # .ws: the split-K workspace of the capture running on this thread


@contextlib.contextmanager
def capture_splitk_workspace(ws: Optional[torch.Tensor]):
    """Graph captures inside this block give their split-K launches (those
    without a caller workspace) ``ws`` instead of a memset graph-pool workspace per
    launch.  ``ws`` (``splitk_workspace``, zeroed counters) must be used only by
    graphs that never run concurrently -- the engine keeps one per compute stream.
    Thread-local: a live capture on another thread is unaffected."""
    prev = getattr(_cap_ws_local, "ws", None)
    _cap_ws_local.ws = ws
    try:
        yield ws
    finally:
        _cap_ws_local.ws = prev


def splits_of(c: int) -> int:
    """Split-K factor of an encoded tile choice (0 / 1: not split).  The factor is
    the 4-bit field at bit 8 (gemm_core.h decodes ``(cfg >> 8) & 15``): the DEEP
    flag (bit 12), CONV_LINEAR (bit 16) and CONV_PP (bit 17) are not part of it;
    a CONV_LINEAR choice is never split."""
    return 0 if c < 0 or (c & CONV_LINEAR) else (c >> 8) & 15


def _private_splitk_ws(device, need: int) -> torch.Tensor:
    """The split-K workspace a launch without a caller workspace uses: one per
    (device, stream), grown on demand, so a forward that passes none pays no
    allocation or counter memset per call.  Split-K launches leave the counters
    zero, so consecutive launches on one stream may share it (two streams never do).
    Inside a graph capture it is the workspace the capturing code installed with
    ``capture_splitk_workspace`` (the engine: one per compute stream, shared by the
    graphs replayed on that stream, which run in stream order and leave the
    counters zero -- no memset node at all), else a fresh one from the graph's own
    pool zeroed by a memset node per launch (never cached: a cached one would be
    shared by graphs replayed concurrently on different streams, and would keep
    the capture pool alive past the graph)."""
    need = max(SPLITK_HEADER, int(need))
    if torch.cuda.is_current_stream_capturing():
        ws = getattr(_cap_ws_local, "ws", None)
        if ws is not None and ws.numel() >= need:
            return ws
        return splitk_workspace(device, need)
    key = (str(device), _stream())
    ws = _priv_ws.get(key)
    if ws is None or ws.numel() < need:
        ws = _priv_ws[key] = splitk_workspace(device, max(need, SPLITK_WS_BYTES))
    return ws


def splitk_workspace(device, nbytes: int = SPLITK_WS_BYTES, zeroed: bool = True) -> torch.Tensor:
    """A split-K workspace: zeroed tile counters + f32 partial tiles.  Every
    split-K launch leaves the counters zero again, so one workspace serves the
    consecutive convolutions of a forward; two launches that may overlap (two
    streams) need two workspaces.  ``zeroed=False``: the caller zeroes the
    counter header itself before the first split-K launch (``image_to_s2d(zero=)``)."""
    ws = torch.empty(nbytes, device=device, dtype=torch.uint8)
    if zeroed:
        ws[:SPLITK_HEADER].zero_()
    return ws


def _conv_pp_candidates(M: int, K_out: int, Kg: int, C: int):
    """Ping-pong conv tiles (CONV_PP) for an im2col conv: every tile whose BK
    divides C, split-K where the grid is under ~one block per CU."""
    out = []
    if K_out % 8:
        return out
    for v in range(len(_CONV_PP_BM)):
        bm, bn, bk = _CONV_PP_BM[v], _CONV_PP_BN[v], _CONV_PP_BK[v]
        if C % bk:
            continue
        tiles = -(-M // bm) * -(-K_out // bn)
        out.append(CONV_PP | v)
        if not _CONV_SPLITK or tiles >= 256:
            continue
        nk = Kg // bk
        for sp in _SPLITS + (12,):
            kper = -(-nk // sp)
            eff = -(-nk // kper)
            if eff < 2 or kper < 3 or tiles * eff > 1024:
                continue
            if SPLITK_HEADER + tiles * eff * bm * bn * 4 > SPLITK_WS_BYTES:
                continue
            out.append(CONV_PP | v | (sp << 8))
    return out


def conv_halo_candidates(N: int, H: int, W: int, C: int, K: int, R: int, S: int, stride: int, pad: int, P: int,
                         Q: int, has_bias: bool, has_res: bool = False, act: str = "relu"):
    """Halo-tile 3x3 tiles (CONV_HALO | v [| splits << 8]) whose rows fit the image
    (conv_halo.hip ``conv_halo_tiles_s``): 3x3 convs with pad 1, stride 1 or 2, the full
    output, a bias; the one-patch-buffer tiles only for a single 64-channel block
    (C == 64), the resident-weight tiles only at stride 1; split-K where the tile
    grid leaves CUs idle."""
    if not (_CONV_HALO and has_bias and R == 3 and S == 3 and stride in (1, 2) and pad == 1
            and (P, Q) == ((H - 1) // stride + 1, (W - 1) // stride + 1) and C % 64 == 0 and K % 8 == 0):
        return []
    rw_ok = not has_res and act in ("relu", "none")
    out = []
    for v in range(len(_CONV_HALO_BM)):
        tiles = _ops().conv_halo_tiles_s(v, N, H, W, C, K, stride)
        if tiles <= 0 or (v in _CONV_HALO_RW and not rw_ok):
            continue
        out.append(CONV_HALO | v)
        if v not in _CONV_HALO_SK or not _CONV_SPLITK or tiles >= 256:
            continue
        # split-K where the tile grid leaves CUs idle (stages 3 / 4 of ResNet-50 at small batch)
        ncb = C // 64
        for sp in (2, 3, 4, 8):
            cpb = -(-ncb // sp)
            eff = -(-ncb // cpb)
            if eff < 2 or eff != sp or tiles * eff > 1024:
                continue
            if _ops().conv_halo_ws_bytes(v, N, H, W, C, K, sp, stride) > SPLITK_WS_BYTES:
                continue
            out.append(CONV_HALO | v | (sp << 8))
    return out


def _conv_candidates(M: int, K_out: int, Kg: int, one_by_one: bool, C: int = 0, has_bias: bool = False):
    """Tile choices for a conv of output [M, K_out] over a Kg-long reduction:
    every 4-wave tile; split-K where the tile grid leaves CUs idle (< 2 blocks
    per CU) and each split keeps >= 4 K-steps; the dense GEMM tiles for 1x1;
    the ping-pong conv tiles for the im2col convs (with a bias)."""
    cands = list(range(NUM_CONV_TILE_CFGS))
    nk = -(-Kg // 64)

    def tiles_of(c):
        return -(-M // _TILE_BM[c]) * -(-K_out // _TILE_BN[c])

    if _GEMM_DEEP:
        cands += [c | DEEP for c in _DEEP_TILES if (c in _DEEP_BIG or tiles_of(c) <= _DEEP_MAX_BLOCKS) and nk >= 4]
    if _CONV_SPLITK:
        for c in range(NUM_CONV_TILE_CFGS):
            tiles = tiles_of(c)
            if tiles >= 512:
                continue
            for sp in _SPLITS:
                kper = -(-nk // sp)
                eff = -(-nk // kper)
                if eff < 2 or kper < 4 or tiles * eff > 2048:
                    continue
                if SPLITK_HEADER + tiles * eff * _TILE_BM[c] * _TILE_BN[c] * 4 > SPLITK_WS_BYTES:
                    continue
                cands.append(c | (sp << 8))
                if _GEMM_DEEP and c in _DEEP_TILES and tiles * eff <= _DEEP_MAX_BLOCKS and kper >= 4:
                    cands.append(c | (sp << 8) | DEEP)
    if one_by_one and _CONV1X1_GEMM and K_out % 8 == 0:
        cands += [CONV_LINEAR | c for c in _gemm_candidates(M, K_out, Kg)]
    if not one_by_one and has_bias and _CONV_PP:
        cands += _conv_pp_candidates(M, K_out, Kg, C)
    return cands


def conv2d_nhwc(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, stride: int = 1,
                pad: int = 0, act: str = "none", residual: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, tile_cfg: int = -1, out_hw: Optional[tuple] = None,
                workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [N, H, W, C] f16, w [K, R, S, C] f16 (BN folded), bias [K]; fused residual + act.
    ``out_hw`` = (P, Q) computes only the first P x Q outputs (an asymmetric pad:
    the space-to-depth stem pads 2 on top / left and 1 on the bottom / right).
    ``workspace`` (``splitk_workspace``): used when the chosen tile is split-K;
    without one a split-K choice allocates its own (one extra memset)."""
    _check(x.is_cuda and x.dtype == torch.float16 and x.is_contiguous() and x.dim() == 4, "conv2d: bad x")
    _check(w.dtype == torch.float16 and w.is_contiguous() and w.dim() == 4, "conv2d: bad w")
    N, H, W, C = x.shape
    K, R, S, C2 = w.shape
    _check(C == C2 and C % 8 == 0, f"conv2d: channel mismatch/alignment {C} vs {C2}")
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - S) // stride + 1
    if out_hw is not None:
        _check(0 < out_hw[0] <= P and 0 < out_hw[1] <= Q, "conv2d: out_hw larger than the padded output")
        P, Q = int(out_hw[0]), int(out_hw[1])
    if out is None:
        out = torch.empty(N, P, Q, K, device=x.device, dtype=torch.float16)
    _check(out.shape == (N, P, Q, K) and out.is_contiguous(), "conv2d: bad out")
    if bias is not None:
        _check(bias.numel() == K and bias.dtype == torch.float16, "conv2d: bad bias")
    if residual is not None:
        _check(residual.shape == (N, P, Q, K) and residual.is_contiguous() and residual.dtype == torch.float16, "conv2d: bad residual")
    _check(_aligned(x) and _aligned(w), "conv2d: alignment")
    M, Kg = N * P * Q, R * S * C
    one_by_one = R == 1 and S == 1 and stride == 1 and pad == 0
    fn = _ops().conv2d_nhwc
    args = (x.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(), N, H, W, C, K, R, S,
            stride, pad, P, Q, ACT_CODE[act])

    def launch(c: int, ws: Optional[torch.Tensor]) -> None:
        if c >= 0 and c & CONV_LINEAR:
            _ops().gemm_tn(DTYPE_CODE[torch.float16], DTYPE_CODE[torch.float16], x.data_ptr(), C, w.data_ptr(), C,
                           out.data_ptr(), K, _ptr(bias), _ptr(residual), K if residual is not None else 0, M, K, C,
                           1.0, ACT_CODE[act], _stream(), c & ~CONV_LINEAR)
            return
        sp = splits_of(c)
        if sp > 1 and ws is None:
            need = _ops().conv_halo_ws_bytes(c & 255, N, H, W, C, K, sp, stride) if c & CONV_HALO else \
                _ops().conv_splitk_bytes(M, K, c & ~0xF00, sp)
            ws = _private_splitk_ws(x.device, int(need))
        fn(*args, _stream(), int(c), _ptr(ws), 0 if ws is None else ws.numel())

    if tile_cfg < 0:
        key = ("conv", N, H, W, C, K, R, S, stride, pad, act, bias is not None, residual is not None) + \
            ((P, Q) if out_hw is not None else ())

        def tune_launch(c: int) -> None:
            # tuning launches may overlap on side streams: one workspace per stream
            ws = None
            if splits_of(c) > 1:
                sid = _stream()
                ws = _tune_ws.get(sid)
                if ws is None:
                    ws = _tune_ws[sid] = splitk_workspace(x.device)
            launch(c, ws)
        tile_cfg = _tuned_cfg(key, tune_launch, _conv_candidates(M, K, Kg, one_by_one, C, bias is not None) +
                              conv_halo_candidates(N, H, W, C, K, R, S, stride, pad, P, Q, bias is not None,
                                                   residual is not None, act))
    launch(int(tile_cfg), workspace)
    return out


def conv2d_nhwc_ref(x, w, bias=None, stride=1, pad=0, act="none", residual=None):
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(),
                 bias.float() if bias is not None else None, stride=stride, padding=pad)
    y = y.permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual.float()
    return _act_ref(y, act).to(torch.float16)


def dwconv_nhwc(x, w, bias, stride=1, pad=1, act="none"):
    """Depthwise conv: x [N, H, W, C], w [R, R, C], bias [C]."""
    _check(x.is_cuda and x.dtype == torch.float16 and x.is_contiguous(), "dwconv: bad x")
    N, H, W, C = x.shape
    R = w.shape[0]
    _check(w.shape == (R, R, C) and w.is_contiguous() and bias.numel() == C and C % 8 == 0, "dwconv: bad w/bias")
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - R) // stride + 1
    out = torch.empty(N, P, Q, C, device=x.device, dtype=torch.float16)
    _ops().dwconv_nhwc(x.data_ptr(), w.data_ptr(), bias.data_ptr(), out.data_ptr(), N, H, W, C, R, stride, pad, P, Q,
                       ACT_CODE[act], _stream())
    return out


def dwconv_nhwc_ref(x, w, bias, stride=1, pad=1, act="none"):
    C = x.shape[-1]
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(2, 0, 1).unsqueeze(1).float(), bias.float(),
                 stride=stride, padding=pad, groups=C)
    return _act_ref(y.permute(0, 2, 3, 1), act).to(torch.float16)


def maxpool_nhwc(x, k=3, stride=2, pad=1):
    _check(x.is_cuda and x.dtype == torch.float16 and x.is_contiguous() and x.shape[-1] % 8 == 0, "maxpool: bad x")
    N, H, W, C = x.shape
    P = (H + 2 * pad - k) // stride + 1
    Q = (W + 2 * pad - k) // stride + 1
    out = torch.empty(N, P, Q, C, device=x.device, dtype=torch.float16)
    _ops().maxpool_nhwc(x.data_ptr(), out.data_ptr(), N, H, W, C, k, stride, pad, P, Q, _stream())
    return out


def maxpool_nhwc_ref(x, k=3, stride=2, pad=1):
    return F.max_pool2d(x.permute(0, 3, 1, 2).float(), k, stride, pad).permute(0, 2, 3, 1).half()


def avgpool_nhwc(x):
    _check(x.is_cuda and x.dtype == torch.float16 and x.is_contiguous() and x.shape[-1] % 8 == 0, "avgpool: bad x")
    N, H, W, C = x.shape
    out = torch.empty(N, C, device=x.device, dtype=torch.float16)
    _ops().avgpool_nhwc(x.data_ptr(), out.data_ptr(), N, H * W, C, _stream())
    return out


def avgpool_nhwc_ref(x):
    return x.float().mean(dim=(1, 2)).half()


def shuffle_remap(a: torch.Tensor, b: torch.Tensor, ch: int, split: bool, ld1: int, ld2: int = 0):
    """ShuffleNetV2 concat(a, b) + channel_shuffle(groups=2) [+ split] in one pass.

    a, b: [..., >=ch] f16 (x1 / branch output, possibly channel-padded views with
    unit stride in the last dim).  Returns one tensor [..., ld1] (``split=False``,
    2*ch real channels) or two tensors [..., ld1], [..., ld2] (the next unit's
    halves, ch real channels each); padded channels are zero."""
    _check(a.is_cuda and a.dtype == torch.float16 and b.dtype == torch.float16, "shuffle_remap: f16 cuda tensors")
    _check(a.stride(-1) == 1 and b.stride(-1) == 1 and a.shape[:-1] == b.shape[:-1], "shuffle_remap: bad views")
    lead = a.shape[:-1]
    pixels = 1
    for d in lead:
        pixels *= d
    lda = a.stride(-2) if a.dim() > 1 else a.shape[-1]
    ldb = b.stride(-2) if b.dim() > 1 else b.shape[-1]
    _check(a.dim() < 2 or all(a.stride(i) == a.stride(i + 1) * a.shape[i + 1] for i in range(a.dim() - 2)),
           "shuffle_remap: a must be a channel slice of a contiguous tensor")
    _check(b.dim() < 2 or all(b.stride(i) == b.stride(i + 1) * b.shape[i + 1] for i in range(b.dim() - 2)),
           "shuffle_remap: b must be a channel slice of a contiguous tensor")
    o1 = torch.empty(*lead, ld1, device=a.device, dtype=torch.float16)
    o2 = torch.empty(*lead, ld2, device=a.device, dtype=torch.float16) if split else None
    _ops().shuffle_remap(a.data_ptr(), lda, b.data_ptr(), ldb, ch, pixels, o1.data_ptr(), ld1, _ptr(o2), ld2,
                         int(split), _stream())
    return (o1, o2) if split else o1


def shuffle_remap_ref(a, b, ch, split, ld1, ld2=0):
    cat = torch.cat([a[..., :ch], b[..., :ch]], dim=-1)
    lead = cat.shape[:-1]
    sh = cat.reshape(*lead, 2, ch).transpose(-1, -2).reshape(*lead, 2 * ch)

    def pad(t, ld):
        out = torch.zeros(*lead, ld, device=t.device, dtype=t.dtype)
        out[..., :t.shape[-1]] = t
        return out
    if split:
        return pad(sh[..., :ch], ld1), pad(sh[..., ch:], ld2)
    return pad(sh, ld1)


def se_scale(x: torch.Tensor, s: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Squeeze-excitation scaling: x [N, H, W, C] * s [N, C] (f16)."""
    _check(x.is_cuda and x.dtype == torch.float16 and x.is_contiguous() and x.dim() == 4, "se_scale: bad x")
    N, H, W, C = x.shape
    _check(s.shape == (N, C) and s.is_contiguous() and s.dtype == torch.float16, "se_scale: bad s")
    out = torch.empty_like(x) if out is None else out
    _ops().se_scale(x.data_ptr(), s.data_ptr(), out.data_ptr(), N, H * W, C, _stream())
    return out


def se_scale_ref(x, s):
    return (x.float() * s.float()[:, None, None, :]).to(torch.float16)


# ---------------------------------------------------------------------------
# Per-block stamps of the diagnostic kernel build (ops/csrc/common.h
# RDB_STAMP_*; ``python -m ray_dynamic_batching_amd._build --variant stamps
# -D RDB_BLOCK_STAMPS``, loaded with RDB_OPS_SO).  bench/stamp_timeline.py turns
# the records into co-residency / CU-time of the UN-profiled serving bench.
# ---------------------------------------------------------------------------
_V4_BUILT = None


def _v4_tiles_built() -> bool:
    """The 4-wave VGPR-staged tiles (cfg 26..28) are part of the opt-in
    RDB_EXPERIMENTAL_KERNELS build only."""
    global _V4_BUILT
    if _V4_BUILT is None:
        try:
            _V4_BUILT = experimental_kernels_built()
        except Exception:  # noqa: BLE001 -- no kernel library (CPU host): not built
            _V4_BUILT = False
    return _V4_BUILT


def experimental_kernels_built() -> bool:
    """Whether the loaded kernel library carries the opt-in variants that lost
    their A/Bs (stream-K, row-LayerNorm, LNOUT / staged-LN epilogues): built only
    with ``python -m ray_dynamic_batching_amd._build --variant experimental -D
    RDB_EXPERIMENTAL_KERNELS`` and loaded with RDB_OPS_SO (ops/csrc/common.h)."""
    f = getattr(_ops(), "experimental_kernels_built", None)
    return bool(f and f())


def stamps_built() -> bool:
    """Whether the loaded kernel library is the RDB_BLOCK_STAMPS diagnostic build."""
    f = getattr(_ops(), "stamps_built", None)
    return bool(f and f())


class BlockStamps:
    """Device buffer the instrumented kernels write one record per block to:
    [t_begin, t_end, meta, where] u64 (common.h).  ``cap`` records at most; the
    counter keeps counting past it (``dropped``)."""

    def __init__(self, cap: int = 1 << 22, device="cuda"):
        _check(stamps_built(), "BlockStamps needs the RDB_BLOCK_STAMPS kernel build (RDB_OPS_SO=<variant .so>)")
        self.cap = int(cap)
        self.buf = torch.zeros(self.cap * 4, dtype=torch.int64, device=device)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        _ops().stamps_set(self.buf.data_ptr(), self.count.data_ptr(), self.cap)

    def reset(self) -> None:
        torch.cuda.synchronize()
        self.count.zero_()
        torch.cuda.synchronize()

    def read(self):
        """The records written since the last reset, as an [n, 4] uint64 array."""
        import numpy as np

        torch.cuda.synchronize()
        n = min(int(self.count.item()), self.cap)
        return self.buf[: n * 4].view(n, 4).cpu().numpy().view(np.uint64)

    @property
    def dropped(self) -> int:
        return max(0, int(self.count.item()) - self.cap)

    def close(self) -> None:
        torch.cuda.synchronize()
        _ops().stamps_set(0, 0, 0)
