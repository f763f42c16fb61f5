"""HIP full-state JSON codec vs the CPU oracle: LocalState bytes, Decode results and
MergeRemoteState effects must be identical, over valid peer documents (rewritten, edge records)
and the documents the reference's Decode rejects."""
import pytest

from sidecar_amd.abi import INIT_EMPTY, INIT_OWN, INIT_WARM, Engine, default_params
from sidecar_amd.codec import synthetic_names
from tests.codec_docs import fixture_names, reference_fixture_state, variants
from tests.parity import assert_same

pytestmark = pytest.mark.gpu

SCEN = {
    "h12_s4_own": dict(n_hosts=12, n_services=4, init_mode=INIT_OWN, ae_period_rounds=5, churn_ppm=100000),
    "h9_s3_odd": dict(n_hosts=9, n_services=3, init_mode=INIT_OWN, ae_period_rounds=4, churn_ppm=200000),
    "h40_s16_storm": dict(n_hosts=40, n_services=16, init_mode=INIT_WARM, ae_period_rounds=10,
                          partition_start=0, partition_end=20, storm_round=3, queue_cap=1024),
    "h7_s64": dict(n_hosts=7, n_services=64, init_mode=INIT_EMPTY, ae_period_rounds=6, churn_ppm=300000),
    "h33_s1": dict(n_hosts=33, n_services=1, init_mode=INIT_OWN, ae_period_rounds=3),
}


def pair(oracle_lib, gx_lib, kw, rounds, names_seed=5):
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    g.run_rounds(rounds)
    o.run_rounds(rounds)
    nm = synthetic_names(kw["n_hosts"], kw["n_services"], seed=names_seed)
    g.set_names(nm)
    o.set_names(nm)
    return g, o


@pytest.mark.parametrize("name", sorted(SCEN))
def test_gpu_local_state_json_equals_oracle(oracle_lib, gx_lib, name):
    kw = SCEN[name]
    g, o = pair(oracle_lib, gx_lib, kw, 27)
    for v in range(kw["n_hosts"]):
        assert g.local_state_json(v) == o.local_state_json(v), (name, v)
    assert_same(g, o, name)  # set_names also set the packPacket static bytes


def _cmp_decode(g, o, doc, what):
    rg, recg, dsg = g.decode_state_json(doc)
    ro, reco, dso = o.decode_state_json(doc)
    assert rg == ro, (what, rg, ro, dsg, dso)
    dsg.pop("error_at")
    dso.pop("error_at")
    if ro == 0:
        assert recg == reco, what
        assert dsg == dso, what
    else:
        assert recg == [], what


def test_gpu_decode_equals_oracle_on_variants(oracle_lib, gx_lib):
    kw = SCEN["h40_s16_storm"]
    g, o = pair(oracle_lib, gx_lib, kw, 31)
    for v in (0, 21, 39):
        base = o.local_state_json(v)
        for name, doc, ok in variants(base, seed=v):
            _cmp_decode(g, o, doc, f"view {v} {name}")


def test_gpu_decodes_reference_fixture_records(oracle_lib, gx_lib):
    kw = dict(n_hosts=2, n_services=2, init_mode=INIT_EMPTY)
    g = Engine(default_params(gx_lib, **kw), lib=gx_lib)
    o = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    g.set_names(fixture_names())
    o.set_names(fixture_names())
    _cmp_decode(g, o, reference_fixture_state(), "services_delegate_test.go fixtures")
    assert g.decode_state_json(reference_fixture_state())[2]["records"] == 3


@pytest.mark.parametrize("name", ["h12_s4_own", "h40_s16_storm", "h7_s64"])
def test_gpu_merge_remote_state_json_equals_oracle(oracle_lib, gx_lib, name):
    kw = SCEN[name]
    src_g, src_o = pair(oracle_lib, gx_lib, kw, 40)
    kw2 = dict(kw, seed=1234)
    g, o = pair(oracle_lib, gx_lib, kw2, 9)
    H = kw["n_hosts"]
    g.add_listener(1 % H, 7, 5000)
    o.add_listener(1 % H, 7, 5000)
    for v_src, v_dst in ((0, 1 % H), (H - 1, 2 % H), (3 % H, 3 % H), (1 % H, 1 % H)):
        doc = src_o.local_state_json(v_src)
        assert src_g.local_state_json(v_src) == doc
        rg, dg = g.merge_remote_state_json(v_dst, doc)
        ro, do = o.merge_remote_state_json(v_dst, doc)
        assert rg == ro == 0
        assert_same(g, o, f"{name} merge {v_src}->{v_dst}")
        assert [e.tup() for e in g.drain_listener(1 % H, 7)] == [e.tup() for e in o.drain_listener(1 % H, 7)]
    g.run_rounds(15)
    o.run_rounds(15)
    assert_same(g, o, f"{name} after merges + rounds")


def test_gpu_codec_1024x16(oracle_lib, gx_lib):
    kw = dict(n_hosts=1024, n_services=16, init_mode=INIT_WARM, ae_period_rounds=10, partition_start=0,
              partition_end=30, storm_round=4, queue_cap=4096)
    g, o = pair(oracle_lib, gx_lib, kw, 12)
    for v in (0, 777):
        doc = o.local_state_json(v)
        assert g.local_state_json(v) == doc
        _cmp_decode(g, o, doc, f"1024x16 view {v}")
    doc = o.local_state_json(900)
    assert g.merge_remote_state_json(5, doc)[0] == o.merge_remote_state_json(5, doc)[0] == 0
    assert_same(g, o, "1024x16 merge")


def test_gpu_decode_fuzz_equals_oracle(oracle_lib, gx_lib):
    """Seeded byte mutations (flip, insert, delete, duplicate a span) of valid states: the GPU parser
    accepts exactly what the oracle accepts and decodes the same records."""
    import random
    kw = SCEN["h12_s4_own"]
    g, o = pair(oracle_lib, gx_lib, kw, 19)
    rng = random.Random(2024)
    alphabet = b'{}[]:,"\\ u0123456789abcdefnulltrue-.eE+Z\n\t'
    base = [o.local_state_json(v) for v in range(kw["n_hosts"])]
    n_ok = 0
    for i in range(300):
        doc = bytearray(rng.choice(base))
        for _ in range(rng.randint(1, 3)):
            p = rng.randrange(len(doc))
            m = rng.randrange(4)
            if m == 0:
                doc[p] = rng.choice(alphabet)
            elif m == 1:
                doc.insert(p, rng.choice(alphabet))
            elif m == 2:
                del doc[p]
            else:
                q = min(len(doc), p + rng.randint(1, 40))
                doc[p:p] = doc[p:q]
        rg, recg, dsg = g.decode_state_json(bytes(doc))
        ro, reco, dso = o.decode_state_json(bytes(doc))
        assert rg == ro, (i, bytes(doc), dsg, dso)
        if ro == 0:
            n_ok += 1
            assert recg == reco, i
            dsg.pop("error_at")
            dso.pop("error_at")
            assert dsg == dso, i
    assert 0 < n_ok < 300
