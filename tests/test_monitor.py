"""Consumer side of the monitor records and the metrics map (no GPU):
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


def test_decode_reference_events():
    """The reference's own perf-ring records (read from cilium_events when
    the fixture was made) through the TraceNotify / DropNotify decoders
    (datapath_trace.go:28-40, 96-150, 175-195): fields, observation points,
    connection states, the text and JSON forms."""
    g = G.Golden("ct_seq_egress_v4")
    ev = monitor.decode_events(g.ev.tobytes())
    assert len(ev) == len(g.ev)
    tr = [e for e in ev if isinstance(e, monitor.TraceNotify)]
    dr = [e for e in ev if isinstance(e, monitor.DropNotify)]
    assert len(tr) == int((g.ev["type"] == 4).sum()) > 0 and len(dr) > 0
    for e, r in zip(ev, g.ev):
        assert (e.type, e.hash, e.orig_len, e.src_label, e.dst_label, e.ifindex) == \
            (r["type"], r["hash"], r["len_orig"], r["src_label"], r["dst_label"], r["ifindex"])
        if r["type"] == 4:
            assert (e.obs_point, e.dst_id, e.reason) == \
                (r["subtype"], r["w6"] & 0xFFFF, (r["w6"] >> 16) & 0xFF)
    states = {monitor.conn_state(e.reason) for e in tr}
    assert {"new", "established", "reply"} <= states
    t = next(e for e in tr if e.obs_point == 0)   # TRACE_TO_LXC
    assert t.dump_info().startswith(f"-> endpoint {t.dst_id} flow {t.hash:#x} identity ")
    assert f"to-endpoint: {t.orig_len} bytes ({t.cap_len} captured)" in t.dump_verbose()
    v = t.to_verbose()
    assert v["type"] == "trace" and v["observationPoint"] == "to-endpoint"
    assert v["traceSummary"] == f"-> endpoint {t.dst_id}" and "cpu" not in v
    assert monitor.obs_point(42) == "42" and monitor.conn_state(9) == "9"
    d = dr[0].to_verbose(cpu_prefix="CPU 01: ")
    assert d["type"] == "drop" and d["reason"] == monitor.drop_reason(dr[0].sub_type)
    assert d["cpu"] == "CPU 01: " and d["mark"] == f"{dr[0].hash:#x}"
