"""ServicesState JSON documents for the codec tests: valid states produced by the
encoder and rewritten the ways a real peer's JSON may differ (whitespace, key order and case,
unknown fields, nulls, escapes, duplicate fields), edge records (unknown names, invalid status,
far-future and pre-1970 times) and documents the reference's Decode rejects.

`reference_fixture_state()` wraps the three gossip records of services_delegate_test.go:15-20
(the reference's own JSON, written before ProxyMode existed) into a state document.
"""
import json
import random

from sidecar_amd.codec import Names, go_json_string, service_fragments

# services_delegate_test.go:15-20 (byte for byte)
FIXTURE_RECORDS = [
    b'{"ID":"d419fa7ad1a7","Name":"/dockercon-6adfe629eebc91","Image":"nginx:latest","Created":"2015-02-25T19:04:46Z","Hostname":"docker2","Ports":[{"Type":"tcp","Port":10234}],"Updated":"2015-03-04T01:12:46.669648453Z","Status":0}',
    b'{"ID":"deadbeefabba","Name":"/dockercon-6c01869525db08","Image":"nginx:latest","Created":"2015-02-25T19:04:46Z","Hostname":"docker2","Ports":[{"Type":"tcp","Port":10234}],"Updated":"2015-03-04T01:12:46.669648453Z","Status":0}',
    b'{"ID":"1b3295bf300f","Name":"/romantic_brown","Image":"0415448f2cc2","Created":"2014-10-02T23:58:48Z","Hostname":"docker1","Ports":[{"Type":"tcp","Port":9494}],"Updated":"2015-03-04T01:12:32.630357657Z","Status":0}',
]
FIXTURE_FIELDS = [  # (ID, Name, Image, Created, Hostname, Ports, Updated) of the fixtures
    ("d419fa7ad1a7", "/dockercon-6adfe629eebc91", "nginx:latest", "2015-02-25T19:04:46Z", "docker2", [("tcp", 10234)],
     "2015-03-04T01:12:46.669648453Z"),
    ("deadbeefabba", "/dockercon-6c01869525db08", "nginx:latest", "2015-02-25T19:04:46Z", "docker2", [("tcp", 10234)],
     "2015-03-04T01:12:46.669648453Z"),
    ("1b3295bf300f", "/romantic_brown", "0415448f2cc2", "2014-10-02T23:58:48Z", "docker1", [("tcp", 9494)],
     "2015-03-04T01:12:32.630357657Z"),
]


def fixture_names():
    """A 2-host x 2-service catalog naming the fixture records: docker1 = host 0, docker2 = host 1."""
    ids = ["1b3295bf300f", "unused-svc-01", "d419fa7ad1a7", "deadbeefabba"]
    hosts = ["docker1", "docker2"]
    pre, post = [], []
    for r, sid in enumerate(ids):
        a, b = service_fragments(sid, "/x", "img", 0, hosts[r // 2], None, "")
        pre.append(a)
        post.append(b)
    return Names("default", hosts, ids, pre, post)


def reference_fixture_state():
    """{"Servers":{docker1:{...},docker2:{...}}} around the services_delegate_test.go records."""
    d1 = b'"docker1":{"Name":"docker1","Services":{"1b3295bf300f":' + FIXTURE_RECORDS[2] + b'}}'
    d2 = (b'"docker2":{"Name":"docker2","Services":{"d419fa7ad1a7":' + FIXTURE_RECORDS[0] +
          b',"deadbeefabba":' + FIXTURE_RECORDS[1] + b'}}')
    return b'{"Servers":{' + d1 + b',' + d2 + b'},"ClusterName":"default","Hostname":"docker1"}'


def _shuffle_keys(o, rng):
    if isinstance(o, dict):
        items = list(o.items())
        rng.shuffle(items)
        return {k: _shuffle_keys(v, rng) for k, v in items}
    if isinstance(o, list):
        return [_shuffle_keys(v, rng) for v in o]
    return o


def _services(doc):
    for srv in (doc.get("Servers") or {}).values():
        for sv in (srv.get("Services") or {}).values():
            yield sv


def variants(base: bytes, seed: int = 7):
    """(name, bytes, expect_ok) rewrites of a valid encoder output."""
    rng = random.Random(seed)
    d = json.loads(base)
    out = [("canonical", base, True)]
    out.append(("pretty", json.dumps(d, indent=2).encode(), True))
    out.append(("ascii_escaped", json.dumps(d, ensure_ascii=True, separators=(", ", " : ")).encode(), True))
    out.append(("shuffled_keys", json.dumps(_shuffle_keys(d, rng)).encode(), True))
    # unknown fields with nested values, key case variants
    d2 = json.loads(base)
    d2["Extra"] = {"a": [1, 2, {"b": None}], "c": "x"}
    for srv in d2["Servers"].values():
        srv["Unknown"] = [[], {}, [1.5e3, True, False, None]]
        for sv in srv["Services"].values():
            sv["id"] = sv.pop("ID")
            sv["STATUS"] = sv.pop("Status")
            sv["extra_field"] = {"nested": {"deep": [1, 2, 3]}}
            break
    out.append(("unknown_fields_case", json.dumps(d2).encode(), True))
    # duplicate struct fields: the last wins (raw text surgery keeps the duplicates)
    txt = base.decode()
    i = txt.find('"Updated":')
    if i >= 0:
        j = txt.find('"', i + 11)
        dup = txt[:i] + '"Updated":"2001-01-01T00:00:00Z",' + txt[i:]
        out.append(("dup_field_last_wins", dup.encode(), True))
    k = txt.find('"Servers":')
    if k >= 0:
        out.append(("dup_servers_field", (txt[:k] + '"Servers":{"zz":{"Name":"zz","Services":{}}},' + txt[k:]).encode(), True))
        out.append(("servers_null_last", (txt[:-1] + ',"Servers":null}').encode(), True))
    # nulls where the Go types allow them
    d3 = json.loads(base)
    first = True
    for srv in d3["Servers"].values():
        if first:
            srv["Services"] = None
            first = False
        for sv in (srv["Services"] or {}).values():
            sv["Ports"] = None
            sv["Name"] = None
            sv["Created"] = None
    d3["LastChanged"] = None
    out.append(("nulls", json.dumps(d3).encode(), True))
    # \u escapes inside hostnames and IDs (decoded before the names lookup)
    d4 = json.loads(base)
    for sv in _services(d4):
        sv["Hostname"] = sv["Hostname"]
    s4 = json.dumps(d4)
    s4 = s4.replace('"Hostname": "ip-', '"Hostname": "\\u0069p-', 3)
    out.append(("escaped_names", s4.encode(), True))
    # edge records: unknown host / id, status out of range, far future, pre-1970, zero time
    d5 = json.loads(base)
    svs = list(_services(d5))
    if len(svs) >= 6:
        svs[0]["Hostname"] = "no-such-host"
        svs[1]["ID"] = "no-such-id"
        svs[2]["Status"] = 7
        svs[3]["Updated"] = "2050-01-01T00:00:00Z"
        svs[4]["Updated"] = "1969-12-31T23:59:59.5Z"
        del svs[5]["Updated"]
    out.append(("edge_records", json.dumps(d5).encode(), True))
    d6 = json.loads(base)
    svs = list(_services(d6))
    if len(svs) >= 3:
        svs[0]["Updated"] = "2023-11-14T23:13:20.123+01:00"
        svs[1]["Updated"] = "2023-11-14T22:13:20.1234567891Z"
        svs[2]["Status"] = -1
    out.append(("offsets_long_fraction", json.dumps(d6).encode(), True))
    # rejected documents
    bad = []
    if svs:
        d7 = json.loads(base)
        next(iter(_services(d7)))["Status"] = 1.0
        bad.append(("float_status", json.dumps(d7).encode()))
        d7 = json.loads(base)
        next(iter(_services(d7)))["Status"] = "0"
        bad.append(("string_status", json.dumps(d7).encode()))
        d7 = json.loads(base)
        next(iter(_services(d7)))["Updated"] = "yesterday"
        bad.append(("bad_time", json.dumps(d7).encode()))
        d7 = json.loads(base)
        next(iter(_services(d7)))["Created"] = "2015-02-30T00:00:00Z"
        bad.append(("bad_created_day", json.dumps(d7).encode()))
        d7 = json.loads(base)
        next(iter(_services(d7)))["Ports"] = {"Type": "tcp"}
        bad.append(("ports_object", json.dumps(d7).encode()))
        d7 = json.loads(base)
        next(iter(_services(d7)))["Ports"] = [{"Type": "tcp", "Port": "80"}]
        bad.append(("port_string", json.dumps(d7).encode()))
        d7 = json.loads(base)
        next(iter(_services(d7)))["Hostname"] = 5
        bad.append(("hostname_number", json.dumps(d7).encode()))
        d7 = json.loads(base)
        next(iter(_services(d7)))["Status"] = 2 ** 63
        bad.append(("status_overflow", json.dumps(d7).encode()))
    d8 = json.loads(base)
    if d8["Servers"]:
        key = next(iter(d8["Servers"]))
        d8["Servers"][key] = None
        bad.append(("null_server", json.dumps(d8).encode()))
    t = base.decode()
    m = t.find(':{"Name":')
    if m > 0:
        q = t.rfind('"', 0, t.rfind('"', 0, m))
        hostkey = t[q:m]
        nxt = t.find('},"', t.find('"LastChanged"', m))
        # a second server under the same map key
        bad.append(("dup_server_key", (t[:12] + hostkey + ':{"Name":"x","Services":{}},' + t[12:]).encode()))
    # the same record twice (two server entries holding one service)
    d9 = json.loads(base)
    if d9["Servers"]:
        key = next(iter(d9["Servers"]))
        d9["Servers"]["zzz-copy"] = d9["Servers"][key]
        bad.append(("dup_record", json.dumps(d9).encode()))
    bad += [
        ("junk", b"asdf"), ("empty", b""), ("ws_only", b"  \n"), ("null_doc", b"null"), ("array_doc", b"[]"),
        ("number_doc", b"42"), ("trailing_garbage", base + b"x"), ("two_values", base + b" {}"),
        ("unclosed", base[:-1]), ("truncated", base[: len(base) // 2]), ("extra_close", base + b"}"),
        ("trailing_comma", b'{"Servers":{},}'), ("missing_colon", b'{"Servers" {}}'),
        ("bad_escape", b'{"Hostname":"a\\x"}'), ("raw_control", b'{"Hostname":"a\x01b"}'),
        ("bad_literal", b'{"Servers":nul}'), ("bad_number", b'{"X":01}'), ("leading_plus", b'{"X":+1}'),
        ("unterminated_string", b'{"Servers":{"a'), ("colon_in_array", b'{"X":[1:2]}'),
        ("deep", b'{"X":' + b"[" * 20 + b"]" * 20 + b"}"),
        ("mismatch", b'{"X":[1,2}}'), ("servers_array", b'{"Servers":[]}'),
        ("services_array", b'{"Servers":{"h":{"Services":[]}}}'), ("name_object", b'{"Servers":{"h":{"Name":{}}}}'),
        ("cluster_number", b'{"ClusterName":1}'), ("key_not_string", b'{1:2}'),
    ]
    good = [("empty_state", b"{}", True), ("ws_state", b' \t{ "Servers" : { } }\n', True),
            ("servers_null", b'{"Servers":null}', True),
            ("server_no_services", b'{"Servers":{"h":{"Name":"h"}}}', True),
            ("deep_ok", b'{"X":' + b"[" * 14 + b"]" * 14 + b"}", True),
            ("unicode_keys", '{"Servers":{"héllo ":{"Name":"x","Services":{}}}}'.encode(), True)]
    return out + good + [(n, b, False) for n, b in bad]


def go_string(s) -> bytes:
    return go_json_string(s)
