"""Test-result logging (reference: scheduler.py:46-86 TestResultLogger):
metrics JSON, schedule-change CSV, node-state text dumps under
<base_dir>/<timestamp>/."""
from __future__ import annotations

import csv
import json
from datetime import datetime
from pathlib import Path
from typing import Dict, List


class ResultLogger:
    def __init__(self, base_dir: str = "test_results"):
        self.test_dir = Path(base_dir) / datetime.now().strftime("%Y%m%d_%H%M%S_%f")
        self.test_dir.mkdir(parents=True, exist_ok=True)

    def log_metrics(self, name: str, metrics: dict) -> Path:
        p = self.test_dir / f"{name}_metrics.json"
        p.write_text(json.dumps(metrics, indent=2, default=str))
        return p

    def log_changes(self, name: str, changes: List[dict]) -> Path:
        p = self.test_dir / f"{name}_changes.csv"
        if changes:
            keys = sorted({k for c in changes for k in c})
            with open(p, "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=keys)
                w.writeheader()
                w.writerows(changes)
        return p

    def log_node_state(self, name: str, nodes: Dict[str, list], timestamp: str) -> Path:
        p = self.test_dir / f"{name}_nodes.txt"
        with open(p, "a") as f:
            f.write(f"\nNode state at {timestamp}\n" + "=" * 50 + "\n")
            for label, ns in nodes.items():
                f.write(f"\n{label}\n")
                for i, n in enumerate(ns):
                    f.write(f"Node {i + 1}:\n")
                    f.write((n.describe() if hasattr(n, "describe") else str(n)) + "\n")
        return p
