"""Consumer side of the monitor records: what pkg/monitor does with a
`struct drop_notify` / `struct trace_notify` sample from the cilium_events
perf ring, applied to the records cfc_drop_notify_v4/v6 and
cfc_monitor_events_v4/v6 return.

  * `DropNotify` — pkg/monitor/datapath_drop.go:28-40, 32 little-endian
    bytes, identical to include/cfc.h `cfc_drop_notify`.
  * `drop_reason` — DropReason (datapath_drop.go:80-86) over the reason
    table `errors` (:42-78), which names bpf/lib/common.h's DROP_* codes.
  * `dump_info` / `dump_verbose` — the `cilium monitor` text lines
    (DumpInfo :89-93, DumpVerbose :96-110); the connection summary of the
    captured payload is the caller's (the batch carries no payload).
  * `TraceNotify` — datapath_trace.go:28-40 (include/cfc.h
    `cfc_trace_notify`): observation points, connection states, its
    DumpInfo / DumpVerbose lines and the JSON form (`to_verbose`,
    TraceNotifyToVerbose).
  * `decode_events` — a cfc_monitor_events buffer, drop and trace records
    told apart by the type byte, as the monitor's dispatch on the message
    type does.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

DROP_NOTIFY_LEN = 32           # DropNotifyLen (datapath_drop.go:24)
CILIUM_NOTIFY_DROP = 1         # bpf/lib/common.h:211

_REASONS = {
    0: "Success", 2: "Invalid packet", 130: "Invalid source mac",
    131: "Invalid destination mac", 132: "Invalid source ip",
    133: "Policy denied (L3)", 134: "Invalid packet",
    135: "CT: Truncated or invalid header", 136: "CT: Missing TCP ACK flag",
    137: "CT: Unknown L4 protocol", 138: "CT: Can't create entry from packet",
    139: "Unsupported L3 protocol", 140: "Missed tail call",
    141: "Error writing to packet", 142: "Unknown L4 protocol",
    143: "Unknown ICMPv4 code", 144: "Unknown ICMPv4 type",
    145: "Unknown ICMPv6 code", 146: "Unknown ICMPv6 type",
    147: "Error retrieving tunnel key", 148: "Error retrieving tunnel options",
    149: "Invalid Geneve option", 150: "Unknown L3 target address",
    151: "Not a local target address", 152: "No matching local container found",
    153: "Error while correcting L3 checksum",
    154: "Error while correcting L4 checksum", 155: "CT: Map insertion failed",
    156: "Invalid IPv6 extension header", 157: "IP fragmentation not supported",
    158: "Service backend not found", 159: "Policy denied (L4)",
    160: "No tunnel/encapsulation endpoint (datapath BUG!)",
    161: "Failed to insert into proxymap", 162: "Policy denied (CIDR)",
}


def drop_reason(reason: int) -> str:
    """DropReason: the table's text, else the number."""
    return _REASONS.get(reason, str(reason))


@dataclass
class DropNotify:
    type: int
    sub_type: int
    source: int
    hash: int
    orig_len: int
    cap_len: int
    src_label: int
    dst_label: int
    dst_id: int
    ifindex: int

    _FMT = "<BBHIIIIIII"

    @classmethod
    def decode(cls, raw: bytes) -> "DropNotify":
        """binary.Read(LittleEndian) of one record (monitor's decoder)."""
        if len(raw) < DROP_NOTIFY_LEN:
            raise ValueError(f"drop notify needs {DROP_NOTIFY_LEN} bytes")
        return cls(*struct.unpack_from(cls._FMT, raw))

    def dump_info(self, summary: str = "") -> str:
        return (f"xx drop ({drop_reason(self.sub_type)}) flow {self.hash:#x} to "
                f"endpoint {self.dst_id}, identity {self.src_label}->"
                f"{self.dst_label}: {summary}")

    def dump_verbose(self, prefix: str = "", ifname: str | None = None) -> str:
        s = (f"{prefix} MARK {self.hash:#x} FROM {self.source} DROP: "
             f"{self.orig_len} bytes, reason {drop_reason(self.sub_type)}, "
             f"to ifindex {ifname if ifname is not None else self.ifindex}")
        if self.src_label or self.dst_label:
            s += f", identity {self.src_label}->{self.dst_label}"
        if self.dst_id:
            s += f", to endpoint {self.dst_id}"
        return s

    def to_verbose(self, cpu_prefix: str = "", ifname: str | None = None) -> dict:
        """DropNotifyToVerbose (datapath_drop.go:135-166): the JSON object
        `cilium monitor -o json` prints (empty strings left out)."""
        d = {"cpu": cpu_prefix, "type": "drop", "mark": f"{self.hash:#x}",
             "ifindex": ifname if ifname is not None else str(self.ifindex),
             "reason": drop_reason(self.sub_type), "source": self.source,
             "bytes": self.orig_len, "srcLabel": self.src_label,
             "dstLabel": self.dst_label, "dstID": self.dst_id}
        return {k: v for k, v in d.items() if v != ""}


def decode_records(buf) -> list[DropNotify]:
    """A packed array of records (bytes, numpy or a host copy of the tensor
    cfc_drop_notify_v4/v6 filled) -> DropNotify list, in order."""
    raw = bytes(memoryview(buf).cast("B"))
    if len(raw) % DROP_NOTIFY_LEN:
        raise ValueError("not a whole number of drop_notify records")
    return [DropNotify.decode(raw[i:i + DROP_NOTIFY_LEN])
            for i in range(0, len(raw), DROP_NOTIFY_LEN)]


CILIUM_NOTIFY_TRACE = 4        # bpf/lib/common.h:214
TRACE_NOTIFY_LEN = 32          # TraceNotifyLen (datapath_trace.go:22-23)

# observation points and forwarding reasons (datapath_trace.go:43-85)
TRACE_OBS_POINTS = {0: "to-endpoint", 1: "to-proxy", 2: "to-host", 3: "to-stack",
                    4: "to-overlay", 5: "from-endpoint", 6: "from-proxy",
                    7: "from-host", 8: "from-stack", 9: "from-overlay"}
TRACE_REASONS = {0: "new", 1: "established", 2: "reply", 3: "related"}


def obs_point(p: int) -> str:
    return TRACE_OBS_POINTS.get(p, str(p))


def conn_state(reason: int) -> str:
    return TRACE_REASONS.get(reason, str(reason))


@dataclass
class TraceNotify:
    type: int
    obs_point: int
    source: int
    hash: int
    orig_len: int
    cap_len: int
    src_label: int
    dst_label: int
    dst_id: int
    reason: int
    pad: int
    ifindex: int

    _FMT = "<BBHIIIIIHBBI"

    @classmethod
    def decode(cls, raw: bytes) -> "TraceNotify":
        if len(raw) < TRACE_NOTIFY_LEN:
            raise ValueError(f"trace notify needs {TRACE_NOTIFY_LEN} bytes")
        return cls(*struct.unpack_from(cls._FMT, raw))

    def trace_summary(self) -> str:
        """traceSummary (datapath_trace.go:96-121)."""
        return {0: f"-> endpoint {self.dst_id}", 1: "-> proxy", 2: "-> host from",
                3: "-> stack", 4: "-> overlay", 5: f"<- endpoint {self.source}",
                6: "<- proxy", 7: "<- host", 8: "<- stack",
                9: "<- overlay"}.get(self.obs_point, "unknown trace")

    def dump_info(self, ifname: str | None = None, summary: str = "") -> str:
        """DumpInfo (:124-128)."""
        return (f"{self.trace_summary()} flow {self.hash:#x} identity {self.src_label}->"
                f"{self.dst_label} state {conn_state(self.reason)} ifindex "
                f"{ifname if ifname is not None else self.ifindex}: {summary}")

    def dump_verbose(self, prefix: str = "", ifname: str | None = None) -> str:
        """DumpVerbose (:131-150), without the payload dissection."""
        s = (f"{prefix} MARK {self.hash:#x} FROM {self.source} {obs_point(self.obs_point)}: "
             f"{self.orig_len} bytes ({self.cap_len} captured), state "
             f"{conn_state(self.reason)}")
        if self.ifindex:
            s += f", interface {ifname if ifname is not None else self.ifindex}"
        if self.src_label or self.dst_label:
            s += f", identity {self.src_label}->{self.dst_label}"
        if self.dst_id:
            s += f", to endpoint {self.dst_id}"
        return s

    def to_verbose(self, cpu_prefix: str = "", ifname: str | None = None) -> dict:
        """TraceNotifyToVerbose (:175-195): the JSON object `cilium monitor
        -o json` prints (empty strings left out, as omitempty does)."""
        d = {"cpu": cpu_prefix, "type": "trace", "mark": f"{self.hash:#x}",
             "ifindex": ifname if ifname is not None else str(self.ifindex),
             "state": conn_state(self.reason),
             "observationPoint": obs_point(self.obs_point),
             "traceSummary": self.trace_summary(), "source": self.source,
             "bytes": self.orig_len, "srcLabel": self.src_label,
             "dstLabel": self.dst_label, "dstID": self.dst_id}
        return {k: v for k, v in d.items() if v != "" or k in ("observationPoint",
                                                               "traceSummary")}


def decode_events(buf) -> list:
    """A cfc_monitor_events buffer -> DropNotify / TraceNotify list, in
    order (the type byte picks the record kind)."""
    raw = bytes(memoryview(buf).cast("B"))
    if len(raw) % TRACE_NOTIFY_LEN:
        raise ValueError("not a whole number of 32-byte monitor records")
    out = []
    for i in range(0, len(raw), TRACE_NOTIFY_LEN):
        r = raw[i:i + TRACE_NOTIFY_LEN]
        if r[0] == CILIUM_NOTIFY_DROP:
            out.append(DropNotify.decode(r))
        elif r[0] == CILIUM_NOTIFY_TRACE:
            out.append(TraceNotify.decode(r))
        else:
            raise ValueError(f"record {i // TRACE_NOTIFY_LEN}: unknown type {r[0]}")
    return out
