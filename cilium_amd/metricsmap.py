"""Mirror of pkg/maps/metricsmap (metricsmap.go): read cilium_metrics.

Key {u8 reason; u8 dir; u16 reserved[3]}, value {u64 count; u64 bytes}
(bpf/lib/common.h:195-206); reason 0 = forwarded, >0 = -DROP_*; dir
1 ingress, 2 egress.  The map is PERCPU_HASH in the reference; here the
GPU is the single "CPU" (cfc_num_possible_cpus() == 1).
"""
from __future__ import annotations

import struct

from .datapath import Datapath

MapName = "cilium_metrics"     # metricsmap.go:42
MaxEntries = 65536
BPF_MAP_TYPE_PERCPU_HASH = 5
DirIngress, DirEgress = 1, 2


def open_map(dp: Datapath):
    fd, _ = dp.open_or_create_map(MapName, BPF_MAP_TYPE_PERCPU_HASH, 8, 16,
                                  MaxEntries, 0)
    return fd


def dump(dp: Datapath, fd=None):
    """{(reason, dir): (count, bytes)} summed over CPUs (SyncMetricsMap,
    metricsmap.go:170-206)."""
    if fd is None:
        fd = open_map(dp)
    out = {}
    for k in dp.keys(fd):
        v = dp.lookup_element(fd, k)
        reason, d = k[0], k[1] & 3
        out[(reason, d)] = struct.unpack_from("<QQ", v)
    return out


def dump_rows(dp: Datapath):
    """sorted rows (reason, dir, count, bytes) like the golden fixtures."""
    return sorted((r, d, c, b) for (r, d), (c, b) in dump(dp).items())


_DIRECTION = {0: "UNKNOWN", 1: "INGRESS", 2: "EGRESS"}   # metricsmap.go:60-64


def direction(d: int) -> str:
    """Key.Direction (metricsmap.go:82-90)."""
    return _DIRECTION[d] if d in (DirIngress, DirEgress) else _DIRECTION[0]


def prometheus_counters(dp: Datapath, fd=None):
    """What SyncMetricsMap feeds Prometheus (metricsmap.go:142-206):
    {("drop", reason text, direction): count} for Key.IsDrop() entries
    (metrics.DropCount) and {("forward", direction): count} for forwards
    (metrics.ForwardCount); entries mapping to the same labels add up."""
    from .monitor import drop_reason
    out = {}
    for (reason, d), (count, _bytes) in dump(dp, fd).items():
        if reason:
            lab = ("drop", drop_reason(reason), direction(d))
        else:
            lab = ("forward", direction(d))
        out[lab] = out.get(lab, 0) + count
    return out
