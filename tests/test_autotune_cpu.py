"""In-context tile selection (ops.tune_in_context): coordinate descent over the
near-tied candidates of each GEMM shape, driven by a whole-forward timer.
Pure-Python logic, no GPU: the timer is a fake cost model."""
from ray_dynamic_batching_amd import ops


def test_tune_in_context_keeps_only_real_gains():
    k1, k2, k3 = ("gemm", 1), ("gemm", 2), ("gemm", 3)
    saved = dict(ops._TUNE), dict(ops._TUNE_TOP)
    try:
        ops._TUNE.update({k1: 9, k2: 8, k3: 4})
        # isolated ranking said 9 / 8 / 4; in context cfg 12 is 10 % faster for k1,
        # k2's alternative is only 0.5 % faster (noise), k3 has no runner-up
        ops._TUNE_TOP.update({k1: [9, 12], k2: [8, 15], k3: [4]})
        cost = {(k1, 9): 40.0, (k1, 12): 30.0, (k2, 8): 20.0, (k2, 15): 19.5, (k3, 4): 10.0}
        calls = []

        def time_forward():
            calls.append(1)
            return sum(cost[(k, ops._TUNE[k])] for k in (k1, k2, k3))

        changed = ops.tune_in_context(time_forward, keys=[k1, k2, k3], min_gain=0.02)
        assert changed == {k1: (9, 12)}
        assert ops._TUNE[k1] == 12 and ops._TUNE[k2] == 8 and ops._TUNE[k3] == 4
        assert len(calls) == 3          # baseline + one alternative each for k1, k2
    finally:
        ops._TUNE.clear()
        ops._TUNE.update(saved[0])
        ops._TUNE_TOP.clear()
        ops._TUNE_TOP.update(saved[1])


def test_record_tuning_keys_collects_unique_keys():
    with ops.record_tuning_keys() as keys:
        ops._KEY_LOG.append(("a",))
        assert ops._KEY_LOG is keys
    assert keys == [("a",)] and ops._KEY_LOG is None
