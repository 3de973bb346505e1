"""Consumer side of the drop notifications and the metrics map (no GPU):
pkg/monitor's DropNotify decoding of the oracle's records, and the
Prometheus labels SyncMetricsMap derives from cilium_metrics."""
import numpy as np

import golden_io as G
import oracle as O
from cilium_amd import _lib as L
from cilium_amd import metricsmap, monitor
from cilium_amd.datapath import host_only


def test_decode_oracle_records():
    g = G.Golden("c2_egress_v4")
    o = O.Oracle(g.tables)
    act, ver, ide, nt = o.classify(g.headers, g.mode, g.ep_lxc, want_notify=True)
    rec, idx = o.drop_notify(g.headers, g.mode, g.ep_lxc, ver, ide, nt)
    ev = monitor.decode_records(rec)
    assert len(ev) == len(rec) > 0
    for e, r in zip(ev[:200], rec[:200]):
        assert e.type == monitor.CILIUM_NOTIFY_DROP
        assert (e.sub_type, e.source, e.hash, e.dst_id) == \
            (r["subtype"], r["source"], r["hash"], r["dst_id"])
    e = next(e for e in ev if e.sub_type == 133)
    assert monitor.drop_reason(e.sub_type) == "Policy denied (L3)"
    assert e.dump_info().startswith("xx drop (Policy denied (L3)) flow 0x")
    assert "DROP: " in e.dump_verbose()
    assert monitor.drop_reason(250) == "250"


def test_prometheus_labels_from_metrics_map():
    dp = host_only()
    fd = metricsmap.open_map(dp)
    rows = [(0, 1, 10, 1000), (0, 2, 5, 500), (133, 1, 7, 700),
            (133, 2, 1, 60), (140, 1, 2, 120), (137, 3, 4, 240)]
    for reason, d, c, b in rows:
        key = bytes([reason, d]) + bytes(6)
        dp.update_element(fd, key, np.array([c, b], np.uint64).tobytes())
    got = metricsmap.prometheus_counters(dp, fd)
    assert got == {("forward", "INGRESS"): 10, ("forward", "EGRESS"): 5,
                   ("drop", "Policy denied (L3)", "INGRESS"): 7,
                   ("drop", "Policy denied (L3)", "EGRESS"): 1,
                   ("drop", "Missed tail call", "INGRESS"): 2,
                   ("drop", "CT: Unknown L4 protocol", "UNKNOWN"): 4}
    assert L.CFC_DEVICE_NONE == -1
