"""Helpers to compare two engines (HIP vs oracle) bit for bit."""
import numpy as np


def host_tuples(e):
    return [tuple(getattr(h, f) for f, _ in h._fields_) for h in e.hosts()]


def server_times(e, max_views=512):
    """Server.LastUpdated/LastChanged of every owner, for up to max_views of the engine's views
    (evenly spaced), plus state.LastChanged of all of them."""
    n = e.hi - e.lo
    pick = range(e.lo, e.hi) if n <= max_views else np.linspace(e.lo, e.hi - 1, max_views).astype(int)
    return np.stack([e.server_times(int(v)) for v in pick]), e.last_changed()


def snapshot(e, views=True):
    s = {"hosts": host_tuples(e), "digests": e.digests(), "stats": e.stats()}
    if views:
        s["views"] = e.read_views()
        s["times"], s["last_changed"] = server_times(e)
    return s


def assert_same(a, b, what=""):
    sa, sb = snapshot(a), snapshot(b)
    assert sa["stats"] == sb["stats"], f"{what}: stats differ\n{_dict_diff(sa['stats'], sb['stats'])}"
    if not np.array_equal(sa["views"], sb["views"]):
        diff = np.argwhere(sa["views"] != sb["views"])
        raise AssertionError(f"{what}: {len(diff)} view slots differ, first {diff[:5].tolist()}")
    assert sa["hosts"] == sb["hosts"], f"{what}: host states differ at {_first_diff(sa['hosts'], sb['hosts'])}"
    if not np.array_equal(sa["digests"], sb["digests"]):
        bad = np.nonzero(sa["digests"] != sb["digests"])[0]
        raise AssertionError(f"{what}: queue digests differ for hosts {bad[:10].tolist()}")
    if not np.array_equal(sa["last_changed"], sb["last_changed"]):
        bad = np.nonzero(sa["last_changed"] != sb["last_changed"])[0]
        raise AssertionError(f"{what}: state.LastChanged differs for views {bad[:10].tolist()}")
    if not np.array_equal(sa["times"], sb["times"]):
        diff = np.argwhere(sa["times"] != sb["times"])
        raise AssertionError(f"{what}: {len(diff)} server times differ, first (view#, owner, field) {diff[:5].tolist()}")


def _dict_diff(a, b):
    return {k: (a[k], b.get(k)) for k in a if a[k] != b.get(k)}


def _first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i, x, y
    return None
