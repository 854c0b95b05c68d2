"""Config 5 with live re-planning on the GPU (bench/colocation_replan_bench.py):
ResNet-50 + BERT-base on engine executors while their rates ramp; measured
arrival rates drive SLOScheduler.check_and_update (293-project/src/scheduler.py:
763-904, ramp of test_scheduler.py:57-96).  Across every re-plan -- batch /
duty changes and, with two executors, model moves (load + capture beside the
serving sessions, drain, retire, free) -- no request fails."""
import json
import os
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("policy", ["duty", "priority"])
def test_replan_under_ramp_no_failed_requests(tmp_path, policy):
    sys.path.insert(0, os.path.join(_ROOT, "bench"))
    import colocation_replan_bench as crb

    out = tmp_path / "replan.json"
    crb.main(["--slots", "2", "--policy", policy, "--load", "0.3:0.5,0.7:0.4,0.6:0.2,0.3:0.6",
              "--phase-s", "2.0", "--batches", "1,4,16,32", "--profile-dir", str(tmp_path / "prof"),
              "--json-out", str(out)])
    d = json.loads(out.read_text())
    assert len(d["replans"]) >= 2, d["replans"]                 # the initial plan + at least one re-plan
    for m, t in d["totals"].items():
        assert t["errors"] == 0, (m, t)
        assert t["completed"] > 0
    for row in d["results"]:
        for m, r in row["models"].items():
            assert r["errors"] == 0 and r["served_rps"] > 0.5 * r["offered_rps"], (row["phase"], m, r)
