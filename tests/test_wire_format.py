"""The push-pull wire formats of gx.h, checked by an independent Python reading of the spec: the
digests, who leads each differing block, the lead blocks (run-length coded rows) and the return
blocks ("own word" bits and the follower's words), against the rows both sides held when the
push-pull phase began (taken from an unsharded engine driven phase by phase in lockstep)."""
import numpy as np
import pytest

from sidecar_amd.abi import Engine, default_params
from sidecar_amd.dist import LocalShards
from tests.test_shards_cpu import SCEN

M64 = (1 << 64) - 1
ABSENT = 7
BLK = 512


def dig_hash(w: int, i: int) -> int:
    x = w ^ (i << 40) ^ i
    lo, hi = x & 0xFFFFFFFF, (x >> 32) & 0xFFFFFFFF
    a = ((lo ^ (((hi << 16) | (hi >> 16)) & 0xFFFFFFFF)) * 0x85EBCA6B) & 0xFFFFFFFF
    b = ((hi ^ (a >> 15)) * 0xC2B2AE35) & 0xFFFFFFFF
    a = ((a ^ (b >> 13)) * 0x27D4EB2F) & 0xFFFFFFFF
    a ^= a >> 16
    b = ((b ^ (a >> 11)) * 0x165667B1) & 0xFFFFFFFF
    b ^= b >> 15
    return (a << 32) | b


def lead_literals(words):
    return sum(1 for i, w in enumerate(words) if i == 0 or w != words[i - 1])


def digest(row, b):
    lo, hi = b * BLK, min(len(row), (b + 1) * BLK)
    s0 = s1 = 0
    for i in range(lo, hi):
        h = dig_hash(int(row[i]), i)
        s0 = (s0 + h) & M64
        s1 = (s1 + (h ^ (h >> 29))) & M64
    L = lead_literals([int(w) for w in row[lo:hi]])
    return s0, (s1 & ((1 << 54) - 1)) | (L << 54)


def decode(buf, off, own_words):
    """One encoded block at buf[off:]: (words, own mask bits, bytes used)."""
    om = np.frombuffer(buf, dtype=np.uint64, count=8, offset=off)
    nm = np.frombuffer(buf, dtype=np.uint64, count=8, offset=off + 64)
    n_lit = sum(bin(int(x)).count("1") for x in nm)
    lits = np.frombuffer(buf, dtype=np.uint64, count=n_lit, offset=off + 128)
    out, own, rank = [], [], -1
    for i in range(BLK):
        if (int(nm[i >> 6]) >> (i & 63)) & 1:
            rank += 1
        o = (int(om[i >> 6]) >> (i & 63)) & 1
        own.append(o)
        out.append(own_words[i] if o else int(lits[rank]))
    return out, own, 128 + 8 * n_lit


def stale(w, now, p):
    return (w >> 3) < now - p.tombstone_lifespan_ns - p.stale_fudge_ns


def own_ok(x, y, now, p):
    """gx.h "return": merging y into x acts like merging x into x."""
    xa, ya = (x & 7) == ABSENT, (y & 7) == ABSENT
    if xa or ya:
        return xa and ya
    if stale(y, now, p):
        return stale(x, now, p)
    return not stale(x, now, p) and (y >> 3) <= (x >> 3)


def block_words(row, b):
    lo = b * BLK
    w = [int(x) for x in row[lo:lo + BLK]]
    return w + [0] * (BLK - len(w))


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def rng4(seed, stream, a, b, c):
    h = mix64(seed ^ ((stream * 0xD1B54A32D192ED03) & M64))
    for x in (a, b, c):
        h = mix64(h ^ x)
    return h


def feistel(key, q, m):
    b = 0
    while (1 << b) < m:
        b += 1
    hb = max(1, (b + 1) // 2)
    hmask = (1 << hb) - 1
    x = q
    while True:
        L, Rr = x >> hb, x & hmask
        for i in range(4):
            F = mix64(key ^ (i << 32) ^ Rr) & hmask
            L, Rr = Rr, L ^ F
        x = (L << hb) | Rr
        if x < m:
            return x


def ae_pairs(p, rnd):
    """Push-pull pairs of a round in pair order t (gx_oracle.c ae_pairs)."""
    H = p.n_hosts
    split = p.partition_start <= rnd < p.partition_end and not p.fd_enable
    groups = [(0, H // 2), (H // 2, H - H // 2)] if split else [(0, H)]
    out = []
    for base, m in groups:
        key = rng4(p.seed, 7, rnd, base, 0)
        out += [(base + feistel(key, t, m), base + feistel(key, t + 1, m)) for t in range(0, m - 1, 2)]
    return out


def leads(Va, Vb, b, R, a_first):
    """Block b differs and side a leads it (fewer literals; ties: the pair's first host)."""
    if digest(Va, b) == digest(Vb, b):
        return False
    n = min(BLK, R - b * BLK)
    la, lb = lead_literals(block_words(Va, b)[:n]), lead_literals(block_words(Vb, b)[:n])
    return la < lb or (la == lb and a_first)


def parse_lead(buf):
    buf, off, out = bytes(buf), 0, []
    while off < len(buf):
        t, host, n_lead, _ = (int(x) for x in np.frombuffer(buf, dtype=np.uint32, count=4, offset=off))
        off += 16
        blocks = []
        for _ in range(n_lead):
            words, own, used = decode(buf, off, [0] * BLK)
            blocks.append((words, own))
            off += used
        out.append((t, host, blocks))
    return out


@pytest.mark.parametrize("lock_model", [0, 1])
@pytest.mark.parametrize("name", ["storm", "blocks3", "blocks_ragged"])
def test_push_pull_messages_follow_the_spec(oracle_lib, name, lock_model):
    kw = dict(SCEN[name], lock_model=lock_model)
    whole = Engine(default_params(oracle_lib, **kw), lib=oracle_lib)
    sh = LocalShards(oracle_lib, 2, **kw)
    sh.trace_ae = True
    sh.skip_locked = False  # the whole exchange even when every host is locked (its digests are checked)
    p = whole.params
    R = whole.H * whole.S
    nblk = (R + BLK - 1) // BLK
    checked = {"lead": 0, "ret": 0, "digest": 0}
    for _ in range(3 * p.ae_period_rounds + 1):
        rnd, ae = whole.round, whole.is_ae_round()
        # the ServicesState lock this round (gx.h lock_model): a pair with a locked side does not
        # run, so it ships no lead or return blocks; each digest's word 3 bit 1 is its side's lock
        locked = [h.locked_at(rnd) for h in whole.hosts()]
        runs = lambda a, b: not (p.lock_model and (locked[a] or locked[b]))  # noqa: E731
        whole.round_send()
        whole.round_merge()
        V = whole.read_views().reshape(whole.H, R).astype(np.uint64) if ae else None
        now = whole.now() - whole.epoch  # slot time (the words are epoch-relative)
        whole.ae_merge()
        whole.round_end()
        n_trace = len(sh.ae_trace)
        sh.run_rounds(1)
        if not ae or len(sh.ae_trace) == n_trace:
            continue
        pairs = ae_pairs(p, rnd)
        dig_in, lead_in, ret_in = sh.ae_trace[-1]
        for buf in dig_in:  # each received digest is its sender row's, per the spec
            buf, step = bytes(buf), 16 + 16 * nblk
            for off in range(0, len(buf), step):
                t, host, nb, w3 = (int(x) for x in np.frombuffer(buf, dtype=np.uint32, count=4, offset=off))
                assert nb == nblk and host in pairs[t] and (w3 >> 1) & 1 == locked[host]
                d = np.frombuffer(buf, dtype=np.uint64, count=2 * nblk, offset=off + 16)
                for b in range(nblk):  # a side that holds the lock (lock_model = 1) sends zero digests
                    want = (0, 0) if p.lock_model and locked[host] else digest(V[host], b)
                    assert (int(d[2 * b]), int(d[2 * b + 1])) == want
                    checked["digest"] += 1
        for lbuf, rbuf in zip(lead_in, ret_in):  # one inbox per shard (G = 2: one source)
            msgs = parse_lead(lbuf)
            for t, host, blocks in msgs:  # lead blocks: the sender's own rows, coded
                a, b_ = pairs[t]
                partner = b_ if host == a else a
                led = [b for b in range(nblk) if runs(a, b_) and leads(V[host], V[partner], b, R, host == a)]
                assert len(led) == len(blocks), (t, led)
                for b, (words, own) in zip(led, blocks):
                    n = min(BLK, R - b * BLK)
                    assert words[:n] == block_words(V[host], b)[:n]
                    assert own == [int(i >= n) for i in range(BLK)]
                    checked["lead"] += 1
            # return segment: a u64 size per pair, then the answers to this shard's lead blocks
            rbuf = bytes(rbuf)
            sizes = np.frombuffer(rbuf, dtype=np.uint64, count=len(msgs), offset=0)
            off = 8 * len(msgs)
            for k, sz in enumerate(sizes):
                t, host, n_ret, _ = (int(x) for x in np.frombuffer(rbuf, dtype=np.uint32, count=4, offset=off))
                a, b_ = pairs[t]
                leader = b_ if host == a else a  # the receiving side, which led these blocks
                cnts = np.frombuffer(rbuf, dtype=np.uint32, count=n_ret, offset=off + 16)
                q = off + 16 + 4 * (n_ret + (n_ret & 1))
                led = [b for b in range(nblk) if runs(a, b_) and leads(V[leader], V[host], b, R, leader == a)]
                assert len(led) == n_ret
                for j, b in enumerate(led):
                    x, y = block_words(V[leader], b), block_words(V[host], b)
                    words, own, used = decode(rbuf, q, x)
                    assert (used - 128) // 8 == int(cnts[j])
                    for i in range(min(BLK, R - b * BLK)):
                        if own[i]:
                            assert own_ok(x[i], y[i], now, p), (t, b, i)
                        else:
                            assert words[i] == y[i] and not own_ok(x[i], y[i], now, p), (t, b, i)
                    q += used
                    checked["ret"] += 1
                assert q == off + int(sz)
                off += int(sz)
            assert off == len(rbuf)
        assert np.array_equal(np.concatenate([e.read_views() for e in sh.engines]), whole.read_views())
    # with the lock modelled, these storms leave (almost) every pair with a locked side
    assert (lock_model or (checked["lead"] > 0 and checked["ret"] > 0)) and checked["digest"] > 0, checked
