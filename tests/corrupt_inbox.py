"""A received packet slot that fails validation (gx.h packet wire format: key < H * K naming a
sender on another shard, no key twice in a round, receiver owned by the receiving shard, len <=
packet_cap, n_fd <= fd_msg_cap, record keys < R) is refused with GX_EINVAL by both engines: the
oracle at gx_inbox_unpack, the HIP engine (which skips the slot on the device and flags it) at the
next call that waits. Shared by the CPU and GPU tests."""
import numpy as np
import torch

from sidecar_amd.abi import GxError
from sidecar_amd.dist import LocalShards, _ptr

KW = dict(n_hosts=16, n_services=4, fanout=3, init_mode=1, queue_cap=256, packet_cap=8, churn_ppm=200000)
FIELDS = {"key": 0, "receiver": 1, "len": 2, "local_key": 0, "rec_key": 6, "dup": 0}
CASES = sorted(FIELDS)


def _warm(lib, device):
    """Two shards after a few rounds (packets in flight), each past its send phase."""
    sh = LocalShards(lib, 2, device=str(device), **KW)
    sh.run_rounds(3)
    for s in sh.shards:
        s.e.round_send()
    return sh.shards


def bad_value(field, p, words, slot_words):
    """The corrupted word: an out-of-range key, a receiver on the sending shard, an oversized
    length, the key of a sender on the receiving shard (shard 1 = hosts [H/2, H)), a record key
    >= R, or the first slot's key repeated in the second slot."""
    H = p.n_hosts
    return {"key": H * p.fanout, "receiver": 0, "len": p.packet_cap + 1, "local_key": (H // 2) * p.fanout,
            "rec_key": H * p.n_services, "dup": int(words[0])}[field]


def run(lib, device, field):
    """Two shards of KW; shard 0's packets for shard 1 with one header field of the first slot
    corrupted. Returns the rc path: 'ok' or 'einval'."""
    shards = _warm(lib, device)
    sizes = shards[0].e.outbox_bytes()
    assert sizes[1] > 0
    buf = shards[0].pack(sizes, lambda ptr, n: shards[0].e.outbox_pack(ptr, n))
    seg = buf[int(sizes[0]):int(sizes[0]) + int(sizes[1])].clone()
    words = seg.view(torch.int32) if seg.numel() % 4 == 0 else None
    assert words is not None
    slot_words = (16 + 16 * shards[1].e.params.packet_cap) // 4
    at = FIELDS[field] + (slot_words if field == "dup" else 0)  # dup: the second slot takes the first's key
    assert at < words.numel()
    words[at] = bad_value(field, shards[1].e.params, words, slot_words)
    e = shards[1].e
    try:
        e.inbox_unpack(_ptr(seg), seg.numel())
        e.round_merge()
        e.stats()  # waits: the HIP engine reports the flagged slot here
    except GxError as x:
        assert "rc=-22" in str(x), x
        return "einval"
    return "ok"


def run_valid(lib, device):
    """The same exchange without corruption goes through."""
    shards = _warm(lib, device)
    sizes = shards[0].e.outbox_bytes()
    buf = shards[0].pack(sizes, lambda ptr, n: shards[0].e.outbox_pack(ptr, n))
    seg = buf[int(sizes[0]):int(sizes[0]) + int(sizes[1])].clone()
    shards[1].e.inbox_unpack(_ptr(seg), seg.numel())
    shards[1].e.round_merge()
    return shards[1].e.stats()["gossip_merges"]
