"""pkg/maps/ctmap's garbage-collection API over the engine's CT maps.

GCFilter mirrors struct GCFilter (pkg/maps/ctmap/ctmap.go:163-182) and GC()
ctmap.GC (:339-350): RemoveExpired deletes entries whose lifetime is below
Time (GC fills Time from the datapath clock, as the reference reads
bpf.GetMtime), ValidIPs scrubs entries with neither address in the set,
MatchIPs removes entries with either address in it (doFiltering,
:303-325).  EnableConntrackGC's periodic loop (pkg/endpointmanager/
conntrack.go:96-125) is gc_all() on a clock the caller advances.
The work runs in libcfc (cfc_ct_gc): IPv4 entries on the device CT table."""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass, field

# conntrack-garbage-collector-interval (daemon/main.go:367) and its floor
# (pkg/endpointmanager/conntrack.go:30)
GC_INTERVAL_DEFAULT = 60
MIN_GC_INTERVAL = 5
# ctmap.go:78-80
MAX_TIME = 0xFFFFFFFF


def _ip_bytes(ip) -> bytes:
    if isinstance(ip, (bytes, bytearray)):
        return bytes(ip)
    return ipaddress.ip_address(ip).packed


@dataclass
class GCFilter:
    remove_expired: bool = False
    time: int = 0
    valid_ips: set | None = None    # None: no ValidIPs filter
    match_ips: set | None = None    # None: no MatchIPs filter
    stats: dict = field(default_factory=dict)


def GC(dp, fd: int, flt: GCFilter, now: int | None = None) -> int:
    """ctmap.GC(m, filter): with RemoveExpired, Time is the datapath clock
    (`now`, else the clock the datapath runs at: bpf.GetMtime) -> entries
    deleted (gcStats.deleted)."""
    if flt.remove_expired:
        flt.time = int(dp.clock if now is None else now) & 0xFFFFFFFF
    return _do_gc(dp, fd, flt)


def _do_gc(dp, fd: int, flt: GCFilter) -> int:
    """doGC with the filter as given (Flush: Time = MAX_TIME)"""
    st = dp.ct_gc(fd, flt.time, flt.remove_expired,
                  None if flt.valid_ips is None else [_ip_bytes(i) for i in flt.valid_ips],
                  None if flt.match_ips is None else [_ip_bytes(i) for i in flt.match_ips])
    flt.stats = st
    return int(st["deleted"])


def gc_all(dp, now: int, valid_ips=None) -> int:
    """One pass of EnableConntrackGC's loop over every CT map (global and
    local): RemoveExpired at `now`, plus ValidIPs on the initial scan."""
    return GC(dp, -1, GCFilter(remove_expired=True, valid_ips=valid_ips), now)


def flush(dp, fd: int) -> int:
    """(*Map).Flush (ctmap.go:352-360): every entry goes."""
    return _do_gc(dp, fd, GCFilter(remove_expired=True, time=MAX_TIME))
