"""Full-state JSON codec on the CPU oracle, pinned to the reference's own JSON.

- The Python restatement of ffjson's Service encoder (sidecar_amd/codec.py) reproduces the
  services_delegate_test.go:15-20 records byte for byte, so its string escaping, RFC3339Nano time
  format and field order are the reference's.
- The oracle's LocalState JSON equals an independent Python assembly of the same document
  (encoding/json map-key order, ffjson Server/ServicesState layout) and parses with json.loads.
- The oracle's decoder reads the reference's own fixture records; Encode -> Decode round trips
  (services_state_test.go:102-115) and junk is refused (:110-115).
- MergeRemoteState(JSON) equals Merge of the same records through the binary ABI.
"""
import json

import numpy as np
import pytest

from sidecar_amd.abi import GX_EINVAL, INIT_OWN, INIT_WARM, Engine, default_params
from sidecar_amd.codec import (go_json_string, json_time, parse_rfc3339, rfc3339nano, service_json,
                               synthetic_names)
from tests.codec_docs import (FIXTURE_FIELDS, FIXTURE_RECORDS, fixture_names, reference_fixture_state,
                              variants)
from tests.parity import snapshot


def test_service_json_reproduces_reference_fixtures():
    for rec, (sid, name, image, created, host, ports, updated) in zip(FIXTURE_RECORDS, FIXTURE_FIELDS):
        got = service_json(sid, name, image, parse_rfc3339(created), host, ports, parse_rfc3339(updated), "", 0,
                           proxy_mode_field=False)
        assert got == rec
    assert [len(r) for r in FIXTURE_RECORDS] == [225, 225, 214]  # services_delegate_test.go GetBroadcasts cases


def test_go_string_escaping():
    assert go_json_string("a<b>&\"\\") == b'"a\\u003cb\\u003e\\u0026\\"\\\\"'
    assert go_json_string("\n\r\t\x01") == b'"\\n\\r\\t\\u0001"'
    assert go_json_string(" x ") == b'"\\u2028x\\u2029"'
    assert go_json_string(b"\xff") == b'"\\ufffd"'
    assert go_json_string("héllo") == '"héllo"'.encode()


@pytest.mark.parametrize("ns", [0, 1, 10, 100_000_000, 1_700_000_000_000_000_000, 1_425_431_566_669_648_453,
                                2**61 - 1])
def test_time_roundtrip(ns):
    assert parse_rfc3339(rfc3339nano(ns)) == ns
    assert json_time(ns)[0:1] == b'"'


def _engine(lib, H=12, S=4, rounds=25, **kw):
    p = dict(n_hosts=H, n_services=S, init_mode=INIT_OWN, ae_period_rounds=5, churn_ppm=100000)
    p.update(kw)
    e = Engine(default_params(lib, **p), lib=lib)
    e.run_rounds(rounds)
    e.set_names(synthetic_names(H, S, seed=3))
    return e


def python_state_json(e, names, view):
    """The ServicesState JSON assembled independently: encoding/json map-key order, ffjson layout
    (catalog/services_state_ffjson.go:334-375, 771-803), Service = pre + Updated + post + Status."""
    row = e.read_views(view, view + 1)[0]
    times = e.server_times(view)
    vlc = int(e.last_changed(view, view + 1)[0])
    S = e.S
    servers = []
    for o in sorted(range(e.H), key=lambda o: names.hosts[o]):
        ents = []
        for j in sorted(range(S), key=lambda j: names.ids[o * S + j]):
            r = o * S + j
            w = int(row[r])
            if w & 7 == 7:
                continue
            ents.append(go_json_string(names.ids[r]) + b":" + names.pre[r] + json_time(e.word_time(w)) + names.post[r] +
                        str(w & 7).encode() + b"}")
        if not ents:
            continue
        hk = go_json_string(names.hosts[o])
        servers.append(hk + b':{"Name":' + hk + b',"Services":{' + b",".join(ents) + b'},"LastUpdated":' +
                       json_time(int(times[o, 0])) + b',"LastChanged":' + json_time(int(times[o, 1])) + b"}")
    return (b'{"Servers":{' + b",".join(servers) + b'},"LastChanged":' + json_time(vlc) + b',"ClusterName":' +
            go_json_string(names.cluster_name) + b',"Hostname":' + go_json_string(names.hosts[view]) + b"}")


@pytest.mark.parametrize("S", [1, 3, 16])
def test_oracle_encoder_matches_independent_assembly(oracle_lib, S):
    e = _engine(oracle_lib, H=9, S=S)
    names = synthetic_names(9, S, seed=3)
    for v in range(9):
        j = e.local_state_json(v)
        assert j == python_state_json(e, names, v)
        d = json.loads(j)
        assert set(d) == {"Servers", "LastChanged", "ClusterName", "Hostname"}


def test_oracle_decodes_reference_fixture_records(oracle_lib):
    e = Engine(default_params(oracle_lib, n_hosts=2, n_services=2, init_mode=0), lib=oracle_lib)
    e.set_names(fixture_names())
    rc, recs, ds = e.decode_state_json(reference_fixture_state())
    assert rc == 0, ds
    t1 = parse_rfc3339("2015-03-04T01:12:32.630357657Z")
    t2 = parse_rfc3339("2015-03-04T01:12:46.669648453Z")
    assert recs == [(t1, 0, 0, 0), (t2, 1, 0, 0), (t2, 1, 1, 0)]
    assert ds["services"] == 3 and ds["records"] == 3 and ds["unknown"] == 0 and ds["invalid"] == 0


def test_encode_decode_roundtrip_and_junk(oracle_lib):
    # services_state_test.go:102-115: Encode() generates JSON that Decode() reads; junk is an error
    e = _engine(oracle_lib)
    for v in (0, 5, 11):
        j = e.local_state_json(v)
        rc, recs, ds = e.decode_state_json(j)
        assert rc == 0
        row = e.read_views(v, v + 1)[0]
        names = synthetic_names(e.H, e.S, seed=3)
        want = []
        for o in sorted(range(e.H), key=lambda o: names.hosts[o]):
            for s in sorted(range(e.S), key=lambda s: names.ids[o * e.S + s]):
                w = int(row[o * e.S + s])
                if w & 7 != 7:
                    want.append((e.word_time(w), o, s, w & 7))
        assert recs == want
    rc, recs, ds = e.decode_state_json(b"asdf")
    assert rc == GX_EINVAL and recs == [] and ds["error_at"] >= 0


def test_merge_remote_state_json_equals_binary_merge(oracle_lib):
    src = _engine(oracle_lib, rounds=30)
    a = _engine(oracle_lib, rounds=7, seed=99)
    b = _engine(oracle_lib, rounds=7, seed=99)
    n_merged = 0
    for v_src, v_dst in ((3, 4), (0, 11), (7, 7)):
        j = src.local_state_json(v_src)
        rc, ds = a.merge_remote_state_json(v_dst, j)
        assert rc == 0
        _, recs, _ = src.decode_state_json(j)
        recs.sort(key=lambda t: (t[1] * src.S + t[2]))  # Merge in key order
        b.merge_remote_state(v_dst, [(h, sv, ts, st) for ts, h, sv, st in recs])
        n_merged += 1
        sa, sb = snapshot(a), snapshot(b)
        # a full remote state is streamed like gx_merge (ae_slots); the record API streams none
        assert sa["stats"].pop("ae_slots") == sb["stats"].pop("ae_slots") + n_merged * a.H * a.S
        for k in sa:
            eq = np.array_equal(sa[k], sb[k]) if isinstance(sa[k], np.ndarray) else sa[k] == sb[k]
            assert eq, (k, v_src, v_dst)


def test_variants_accept_reject(oracle_lib):
    e = _engine(oracle_lib, rounds=12, init_mode=INIT_WARM)
    base = e.local_state_json(2)
    for name, doc, ok in variants(base):
        rc, recs, ds = e.decode_state_json(doc)
        assert (rc == 0) == ok, (name, rc, ds)
        if name == "edge_records":
            # status 7 is invalid; 2050 is inside the engine's window (stored exactly); the
            # pre-1970 and missing (zero time.Time) Updated clamp to the window's start
            assert ds["unknown"] == 2 and ds["invalid"] == 1, ds
            times = [t for t, _, _, _ in recs]
            assert parse_rfc3339("2050-01-01T00:00:00Z") in times
            assert times.count(e.epoch) == 2 and e.epoch > 0
        if name in ("pretty", "ascii_escaped", "escaped_names"):
            assert recs == e.decode_state_json(base)[1], name
        if name == "shuffled_keys":  # document order changes with the key order
            assert sorted(recs) == sorted(e.decode_state_json(base)[1])


def test_names_rejects_duplicates(oracle_lib):
    from sidecar_amd.codec import Names
    e = Engine(default_params(oracle_lib, n_hosts=2, n_services=2, init_mode=0), lib=oracle_lib)
    nm = fixture_names()
    bad = Names("c", ["a", "a"], nm.ids, nm.pre, nm.post)
    with pytest.raises(Exception):
        e.set_names(bad)
    bad = Names("c", ["a", "b"], ["x", "x", "y", "z"], nm.pre, nm.post)
    with pytest.raises(Exception):
        e.set_names(bad)
