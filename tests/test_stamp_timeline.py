"""bench/stamp_timeline.py on synthetic stamp records (no GPU)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
import stamp_timeline as st  # noqa: E402


def rec(t0, t1, fam, tile, grid, packet, xcc, cu):
    meta = (fam << 56) | (tile << 40) | grid
    hw = (packet << 32) | (xcc << 16) | (cu << 8)
    return [t0, t1, meta, hw]


def test_two_overlapping_launches_on_shared_cus():
    # launch A (gemm_pp tile 19, 2 blocks) on CUs 0 and 1 over [0, 100];
    # launch B (qkv_attn, 2 blocks) on CU 1 over [50, 150] and CU 2 over [50, 150]
    r = np.array([rec(1000, 1100, 1, 19, 2, 7, 0, 0), rec(1000, 1100, 1, 19, 2, 7, 0, 1),
                  rec(1050, 1150, 3, 1, 2, 9, 0, 1), rec(1050, 1150, 3, 1, 2, 9, 1, 2)], dtype=np.uint64)
    s = st.summarize(r, n_cus=4)
    assert s["launches"] == 2 and s["cus_seen"] == 3
    assert s["wall_us"] == 1.5 and s["kernel_sum_us"] == 2.0        # 150 ticks wall, 200 ticks of spans
    assert abs(s["overlap"] - 0.25) < 1e-9
    k = {x["kernel"].split("[")[0]: x for x in s["kernels"]}
    # on CU 1 the two blocks share [50, 100]: each gets half of those 50 ticks
    assert k["gemm_pp"]["cu_us_per_launch"] == 1.8                   # 100 + 75 ticks
    assert k["qkv_attn"]["cu_us_per_launch"] == 1.8
    assert abs(k["gemm_pp"]["co_resident_frac"] - 0.25) < 1e-3        # 50 of 200 block-ticks
    # busy CU time: CU0 100 + CU1 150 + CU2 100 ticks = 3.5 us over 4 CUs x 1.5 us
    assert s["cu_busy_us"] == 3.5 and abs(s["machine_util"] - 350 / 600) < 1e-4


def test_reused_packet_slot_splits_into_launches():
    r = np.array([rec(0 + 10, 100, 4, 0, 1, 3, 0, 0), rec(10000, 10100, 4, 0, 1, 3, 0, 0)], dtype=np.uint64)
    s = st.summarize(r, n_cus=1)
    assert s["launches"] == 2 and s["kernels"][0]["launches"] == 2
