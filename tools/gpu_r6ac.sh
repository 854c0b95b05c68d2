#!/bin/bash
# Round 6: TP replicas through serve.run with hipGraphs ON, rehearsed on one GPU (xGMI all-reduce
# captured in the bucket graphs, grid capped, no line-up barrier): world 2, then world 8, then the
# line-up rehearsal (now on the xGMI all-reduce over the gloo host group).
set -o pipefail
O=gpurun_out/r6ac2
mkdir -p $O
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 330 $P "tests/test_serve_tp_gpu.py::test_llama_tp_through_serve_graphs_one_gpu[2]" > $O/w2.log 2>&1 || { tail -40 $O/w2.log; for d in /tmp/rdb_serve_*; do cp -r $d $O/ 2>/dev/null; done; tail -40 $O/rdb_serve_*/*.log; exit 1; }
tail -3 $O/w2.log
timeout -k 10 330 $P "tests/test_serve_tp_gpu.py::test_llama_tp_through_serve_graphs_one_gpu[8]" > $O/w8.log 2>&1 || { tail -40 $O/w8.log; for d in /tmp/rdb_serve_*; do cp -r $d $O/ 2>/dev/null; done; tail -40 $O/rdb_serve_*/*.log; exit 1; }
tail -3 $O/w8.log
timeout -k 10 330 $P "tests/test_serve_tp_gpu.py::test_llama_tp8_through_serve_matches_tp1" > $O/lineup.log 2>&1 || { tail -40 $O/lineup.log; exit 1; }
tail -3 $O/lineup.log
timeout -k 10 330 $P "tests/test_tp8_gpu.py" > $O/tp8.log 2>&1 || { tail -40 $O/tp8.log; exit 1; }
tail -3 $O/tp8.log
