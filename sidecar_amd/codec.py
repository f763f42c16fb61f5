"""Host side of the full-state JSON codec: the strings a caller hands to
``gx_set_names``.

The engine stores records as (owner, service) indices; the codec needs each record's static JSON
once. A Go host gets it from ``svc.Encode()`` (ffjson, service/service_ffjson.go:370-436); this
module restates that encoder for the Python mirror and the tests:

  Service JSON = {"ID":s,"Name":s,"Image":s,"Created":t,"Hostname":s,"Ports":[{"Type":s,"Port":n,
                 "ServicePort":n,"IP":s},...]|null,"Updated":t,"ProxyMode":s,"Status":n}

with strings escaped like encoding/json (HTML-safe: the Services map goes through encoding/json's
compaction, which escapes <, > and & whatever ffjson wrote) and times as time.Time.MarshalJSON
(quoted RFC3339Nano, UTC). ``pre`` is everything before the Updated value, ``post`` everything
between it and the Status value.
"""
from __future__ import annotations

import datetime as _dt
import re
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

_HEX = "0123456789abcdef"
_PLAIN = re.compile(rb"[\x20-\x21\x23-\x25\x27-\x3b\x3d\x3f-\x5b\x5d-\x7e]*")


def go_json_string(s) -> bytes:
    """encoding/json encodeState.string(s, escapeHTML=true), Go 1.13."""
    b = s.encode() if isinstance(s, str) else bytes(s)
    if _PLAIN.fullmatch(b):  # nothing to escape
        return b'"' + b + b'"'
    out = bytearray(b'"')
    i = 0
    n = len(b)
    while i < n:
        c = b[i]
        if c < 0x80:
            if c >= 0x20 and c not in (0x22, 0x5C, 0x3C, 0x3E, 0x26):
                out.append(c)
            elif c in (0x22, 0x5C):
                out += b"\\" + bytes([c])
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            else:
                out += ("\\u00" + _HEX[c >> 4] + _HEX[c & 15]).encode()
            i += 1
            continue
        r, sz = _utf8_rune(b, i)
        if (r == 0xFFFD and sz == 1) or r in (0x2028, 0x2029):
            out += {0xFFFD: b"\\ufffd", 0x2028: b"\\u2028", 0x2029: b"\\u2029"}[r]
        else:
            out += b[i:i + sz]
        i += sz
    out += b'"'
    return bytes(out)


def _utf8_rune(b: bytes, i: int) -> Tuple[int, int]:
    """utf8.DecodeRune: (rune, size), invalid -> (0xFFFD, 1)."""
    c = b[i]
    n = len(b) - i
    cont = lambda k: n > k and (b[i + k] & 0xC0) == 0x80  # noqa: E731
    if 0xC2 <= c <= 0xDF and cont(1):
        return ((c & 0x1F) << 6) | (b[i + 1] & 0x3F), 2
    if 0xE0 <= c <= 0xEF and cont(1) and cont(2):
        r = ((c & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F)
        if r >= 0x800 and not (0xD800 <= r <= 0xDFFF):
            return r, 3
    if 0xF0 <= c <= 0xF4 and cont(1) and cont(2) and cont(3):
        r = ((c & 0x07) << 18) | ((b[i + 1] & 0x3F) << 12) | ((b[i + 2] & 0x3F) << 6) | (b[i + 3] & 0x3F)
        if 0x10000 <= r <= 0x10FFFF:
            return r, 4
    return 0xFFFD, 1


def rfc3339nano(ns: int) -> str:
    """time.Time.Format(RFC3339Nano) of a UTC instant given in ns since the epoch (>= 0)."""
    secs, frac = divmod(int(ns), 1_000_000_000)
    t = _dt.datetime(1970, 1, 1) + _dt.timedelta(seconds=secs)
    s = t.strftime("%Y-%m-%dT%H:%M:%S")
    if frac:
        s += ("." + f"{frac:09d}").rstrip("0")
    return s + "Z"


def json_time(ns: int) -> bytes:
    return b'"' + rfc3339nano(ns).encode() + b'"'


def parse_rfc3339(s: str) -> int:
    """ns since the epoch of an RFC3339 time with a 'Z' or +hh:mm offset (test helper)."""
    main, _, rest = s.partition(".") if "." in s[19:20] else (s[:19], "", s[19:])
    if _ == ".":
        digits = ""
        k = 0
        while k < len(rest) and rest[k].isdigit():
            digits += rest[k]
            k += 1
        frac = int((digits + "000000000")[:9])
        tz = rest[k:]
    else:
        frac = 0
        tz = rest
    t = _dt.datetime.strptime(main, "%Y-%m-%dT%H:%M:%S")
    off = 0
    if tz != "Z":
        sign = -1 if tz[0] == "-" else 1
        off = sign * (int(tz[1:3]) * 3600 + int(tz[4:6]) * 60)
    secs = (t - _dt.datetime(1970, 1, 1)).days * 86400 + (t - _dt.datetime(1970, 1, 1)).seconds - off
    return secs * 1_000_000_000 + frac


def service_json(ID, Name, Image, Created_ns, Hostname, Ports: Optional[Sequence], Updated_ns, ProxyMode,
                 Status: int, proxy_mode_field: bool = True) -> bytes:
    """Service.MarshalJSON (service/service_ffjson.go:370-436). Ports: None (null) or a list of
    (Type, Port, ServicePort, IP). proxy_mode_field=False gives the older layout of the
    services_delegate_test.go fixtures, which predate ProxyMode (and Port's ServicePort/IP)."""
    pre, post = service_fragments(ID, Name, Image, Created_ns, Hostname, Ports, ProxyMode, proxy_mode_field)
    return pre + json_time(Updated_ns) + post + str(int(Status)).encode() + b"}"


def _ports_json(Ports, full_port: bool) -> bytes:
    if Ports is None:
        return b"null"
    parts = []
    for p in Ports:
        typ, port, sport, ip = (tuple(p) + (0, ""))[:4] if len(p) < 4 else tuple(p)
        s = b'{"Type":' + go_json_string(typ) + b',"Port":' + str(int(port)).encode()
        if full_port:
            s += b',"ServicePort":' + str(int(sport)).encode() + b',"IP":' + go_json_string(ip)
        parts.append(s + b"}")
    return b"[" + b",".join(parts) + b"]"


def service_fragments(ID, Name, Image, Created_ns, Hostname, Ports, ProxyMode,
                      proxy_mode_field: bool = True) -> Tuple[bytes, bytes]:
    """(pre, post) of a Service's JSON around its Updated value (include/gx.h gx_names)."""
    pre = (b'{"ID":' + go_json_string(ID) + b',"Name":' + go_json_string(Name) + b',"Image":' +
           go_json_string(Image) + b',"Created":' + json_time(Created_ns) + b',"Hostname":' +
           go_json_string(Hostname) + b',"Ports":' + _ports_json(Ports, proxy_mode_field) + b',"Updated":')
    post = (b',"ProxyMode":' + go_json_string(ProxyMode) if proxy_mode_field else b"") + b',"Status":'
    return pre, post


class Names:
    """The gx_names tables of a cluster: hostnames, service IDs and Service JSON fragments."""

    def __init__(self, cluster_name, hosts: Sequence, ids: Sequence, pre: Sequence[bytes], post: Sequence[bytes]):
        enc = lambda x: x.encode() if isinstance(x, str) else bytes(x)  # noqa: E731
        self.cluster_name = enc(cluster_name)
        self.hosts = [enc(h) for h in hosts]
        self.ids = [enc(i) for i in ids]
        self.pre = list(pre)
        self.post = list(post)

    @staticmethod
    def _blob(items):
        off = np.zeros(len(items) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64) if items else []
        return b"".join(items), off


def synthetic_names(H: int, S: int, seed: int = 1, cluster: str = "default") -> Names:
    """Sidecar-looking names for a simulated cluster: Docker-style 12-hex IDs, container names,
    images, one TCP port each, ProxyMode "http" (services_delegate_test.go:15-20 style)."""
    rng = np.random.default_rng(seed)
    hosts = [f"ip-10-{(o >> 16) & 255}-{(o >> 8) & 255}-{o & 255}.cluster.local" for o in range(H)]
    created0 = 1_424_891_086_000_000_000  # 2015-02-25T19:04:46Z
    hx = rng.integers(0, 2**48, size=H * S)
    cr = rng.integers(0, 86_400, size=H * S)
    ids, pre, post = [], [], []
    images = ["nginx:latest", "redis:5", "gossip/api:1.4.2", "0415448f2cc2"]
    for o in range(H):
        for j in range(S):
            r = o * S + j
            sid = f"{int(hx[r]):012x}"
            ports = [("tcp", 10000 + j, 8000 + j, f"10.{(o >> 8) & 255}.{o & 255}.{j}")]
            a, b = service_fragments(sid, f"/svc-{o}-{j}", images[(o + j) % len(images)],
                                     created0 + int(cr[r]) * 1_000_000_000, hosts[o], ports, "http")
            ids.append(sid)
            pre.append(a)
            post.append(b)
    return Names(cluster, hosts, ids, pre, post)
