"""CPU tests of the profiling helpers: the GEMM tile-table save/load that lets
counter passes replay identical kernels, and the rocprofv3 --pmc summarizer
(on a synthetic counter CSV of the rocprofv3 csv layout)."""
import csv
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_tuning_table_roundtrip(tmp_path):
    from ray_dynamic_batching_amd import ops

    saved = dict(ops._TUNE)
    try:
        ops._TUNE.clear()
        k1 = ("gemm", torch.bfloat16, 4096, 768, 768, 768, "none", True, True)
        k2 = ("gemm_ln", torch.bfloat16, 4096, 3072, 768, 768, "gelu", 1)
        ops._TUNE[k1], ops._TUNE[k2] = 9, 15
        p = str(tmp_path / "t.json")
        ops.save_tuning(p)
        ops._TUNE.clear()
        assert ops.load_tuning(p) == 2
        assert ops._TUNE == {k1: 9, k2: 15}
    finally:
        ops._TUNE.clear()
        ops._TUNE.update(saved)


def _write_pass(d, counters, rows):
    os.makedirs(d, exist_ok=True)
    cols = ["Dispatch_Id", "Grid_Size", "Workgroup_Size", "Kernel_Name", "Counter_Name", "Counter_Value",
            "Start_Timestamp", "End_Timestamp"]
    with open(os.path.join(d, "p_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for did, name, grid, dur_ns, vals in rows:
            for c in counters:
                w.writerow(dict(Dispatch_Id=did, Grid_Size=grid, Workgroup_Size=256, Kernel_Name=name,
                                Counter_Name=c, Counter_Value=vals[c], Start_Timestamp=1000,
                                End_Timestamp=1000 + dur_ns))


def test_pmc_summary_window_and_metrics(tmp_path):
    gemm = "_ZN3rdb16mfma_gemm_kernelIDF16bDF16bLi128ELi144ENS_11DenseLoaderELb1ELb0ELi4ELi4ELi0EEEvv"
    marker = "rdb::seq_lens_kernel(int const*, int, int, int*)"
    sq = ["SQ_INSTS_MFMA", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"]
    rows = []
    did = 0
    for fwd in range(3):   # the first forward (tuning / warmup) must be windowed out
        did += 1
        rows.append((did, marker, 2048, 2000, {c: 0 for c in sq}))
        did += 1
        rows.append((did, gemm, 131072, 20000 if fwd else 99000,
                     {"SQ_INSTS_MFMA": 884736, "SQ_LDS_BANK_CONFLICT": 10, "SQ_LDS_IDX_ACTIVE": 1000}))
    _write_pass(str(tmp_path / "sq"), sq, rows)
    _write_pass(str(tmp_path / "fetch"), ["FETCH_SIZE"], [(r[0], r[1], r[2], r[3], {"FETCH_SIZE": 100.0}) for r in rows])
    out = str(tmp_path / "s.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "bench", "pmc_summary.py"), str(tmp_path / "sq"),
                    str(tmp_path / "fetch"), "--marker", "seq_lens_kernel", "--forwards", "2", "-o", out],
                   check=True, capture_output=True)
    d = json.load(open(out))
    g = [k for k in d["kernels"] if k["kernel"].startswith("rdb::mfma_gemm_kernel<128,144>")][0]
    assert g["dispatches"] == 2 and abs(g["avg_us"] - 20.0) < 1e-6
    assert abs(g["mfma_tflops"] - 884736 * 16384 / 20e-6 / 1e12) < 0.1
    assert g["lds_bank_conflict_frac"] == 0.01 and g["fetch_bytes"] == 2 * 100 * 1024
    assert abs(d["kernel_us_per_forward_profiled"] - 22.0) < 1e-6
