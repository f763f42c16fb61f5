"""memberlist's messages behind a blocked packet handler (gx.h fd_handoff_shared) on the HIP engine
against the oracle, bit for bit: catalog views, host states, queue digests, server times, every
counter (fd_handoff_queued / fd_handoff_drops included), every host's member list, its handoff
queue count (gx_fd_host.hq_len) and the memberlist broadcast queues. Upstream memberlist at the fork's
date queues alive / suspect / dead messages on the same handoff channel as user messages, drained by
one packetHandler goroutine; a NotifyMsg blocked on the catalog lock stops it (parity unpinned: the
fork is absent). Schedules: departures detected by the failure detector with the lock on, small
pipelines that fill (lock_buffer 60-100), a partition with churn, GossipMessages 4."""
import pytest

from sidecar_amd.abi import INIT_OWN, INIT_WARM
from tests.test_gpu_fd import compare

pytestmark = pytest.mark.gpu

BASE = dict(n_hosts=64, n_services=8, fd_enable=1, depart_round=3, depart_ppm=100000, ae_period_rounds=10,
            queue_cap=4096, fd_handoff_shared=1)
SCENARIOS = {
    "depart_warm": dict(init_mode=INIT_WARM),
    "depart_own": dict(init_mode=INIT_OWN),
    "depart_own_buf80": dict(init_mode=INIT_OWN, lock_buffer=80),
    "depart_gm4_buf100": dict(init_mode=INIT_OWN, gossip_messages=4, lock_buffer=100),
    "partition_churn_buf60": dict(n_hosts=96, n_services=4, init_mode=INIT_OWN, depart_round=-1, depart_ppm=0,
                                  partition_start=5, partition_end=40, churn_ppm=50000, lock_buffer=60),
    "depart_own_readers": dict(init_mode=INIT_OWN, lock_buffer=80, lock_readers=1),
}


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_fd_handoff_parity(gx_lib, oracle_lib, name):
    kw = dict(BASE)
    kw.update(SCENARIOS[name])
    compare(gx_lib, oracle_lib, kw, 200, chunks=(1, 6, 33, 60))
