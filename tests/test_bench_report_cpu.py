"""bench.py's report helpers on synthetic inputs: the steady-state summary a run that never agrees
carries, merges by source and device-time shares (item 7)."""
import bench


def _state(n, locked, depth, fexp_rate, bad):
    return [{"round": 100 * i, "disagreeing": bad, "hosts_locked": locked, "mean_fifo_depth": depth,
             "max_fifo_depth": 2 * depth, "false_expiries": fexp_rate * 100 * i, "ae_exchanges": i,
             "queue_drops": 0} for i in range(1, n + 1)]


def test_steady_state_of_a_stationary_run():
    ss = bench.steady_state(_state(40, 900, 500.0, 7, 1234), 1000)
    assert ss["hosts_locked_frac"] == 0.9 and ss["disagreeing_min"] == 1234
    assert ss["false_expiries_per_round"] == 7.0 and ss["push_pull_exchanges_per_round"] == 0.01
    assert all(abs(v) < 1e-9 for v in ss["drift_q3_to_q4"].values())
    assert ss["rounds"] == [2000, 4000] and ss["queue_drops"] == 0


def test_steady_state_reports_drift():
    st = _state(40, 900, 500.0, 7, 1234)
    for r in st:
        r["mean_fifo_depth"] = float(r["round"])  # a queue that keeps growing
    ss = bench.steady_state(st, 1000)
    assert ss["drift_q3_to_q4"]["mean_fifo_depth"] > 0.2
    assert bench.steady_state(st[:3], 1000) is None  # too few samples


def test_merges_by_source_and_time_share():
    st0 = dict(gossip_merges=10, ae_merges=100, local_merges=1, lock_drained=0)
    st1 = dict(gossip_merges=60, ae_merges=400, local_merges=5, lock_drained=20)
    m = bench.merges_by_source(st0, st1)
    assert m == {"gossip_packets": 30, "lock_pipeline_drained": 20, "push_pull": 300, "owner_local": 4}
    sh = bench.device_time_share({"storm": {"ms": 9.0}, "merge": {"ms": 1.0}})
    assert sh == {"storm": 0.9, "merge": 0.1} and list(sh) == ["storm", "merge"]
    assert bench.device_time_share({}) is None
    assert bench.expiry_report(dict(expired=3, false_expiries=2), dict(expired=10, false_expiries=8)) == \
        {"expired": 7, "false_expiries": 6}
