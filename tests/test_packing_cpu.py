"""Byte-limited packPacket in the round model, on the CPU oracle.

services_delegate.go:186-223: every packet holds whole messages whose encoded lengths plus the
per-message overhead sum to at most the limit; a message that does not fit stays pending.
"""
import numpy as np

from sidecar_amd.abi import INIT_OWN, Engine, default_params


def _engine(lib, limit, cap=32, static=None):
    p = default_params(lib, n_hosts=48, n_services=8, init_mode=INIT_OWN, limit_bytes=limit,
                       overhead_bytes=3, packet_cap=cap, ae_period_rounds=0, churn_ppm=50000,
                       queue_cap=2048)
    e = Engine(p, lib=lib)
    if static is not None:
        e.set_static_bytes(0, 48, static)
    return e


def test_packets_respect_byte_limit(oracle_lib):
    rnd = np.random.default_rng(3)
    static = rnd.integers(100, 500, size=48 * 8).astype(np.uint16)
    e = _engine(oracle_lib, 1398, static=static)
    for _ in range(30):
        e.run_rounds(1)
        for host in range(48):
            # the round's own calls already ran; one more explicit call must also fit the limit
            r = e.get_broadcasts_bytes(host, 3, 1398)
            if r:
                assert sum(b + 3 for b in e.message_bytes(r)) <= 1398
    st = e.stats()
    assert st["packets"] > 0 and st["cap_cuts"] == 0
    # a 1398-byte packet of >=123-byte messages (100 static + 22 + 1) holds at most 11
    assert st["records_sent"] <= 11 * st["packets"]


def test_record_cap_cut_counted(oracle_lib):
    """packet_cap smaller than what the byte limit admits: the cut is reported, never silent."""
    e = _engine(oracle_lib, 1398, cap=2)
    e.run_rounds(20)
    assert e.stats()["cap_cuts"] > 0


def test_record_mode_unchanged(oracle_lib):
    """limit_bytes = 0 keeps BASELINE's record cap: no byte accounting at all."""
    e = _engine(oracle_lib, 0)
    e.run_rounds(20)
    st = e.stats()
    assert st["bytes_sent"] == 0 and st["cap_cuts"] == 0 and st["records_sent"] > 0
