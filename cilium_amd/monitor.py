"""Consumer side of the drop notifications: what pkg/monitor does with a
`struct drop_notify` sample from the cilium_events perf ring, applied to the
records cfc_drop_notify_v4/v6 return.

  * `DropNotify` — pkg/monitor/datapath_drop.go:28-40, 32 little-endian
    bytes, identical to include/cfc.h `cfc_drop_notify`.
  * `drop_reason` — DropReason (datapath_drop.go:80-86) over the reason
    table `errors` (:42-78), which names bpf/lib/common.h's DROP_* codes.
  * `dump_info` / `dump_verbose` — the `cilium monitor` text lines
    (DumpInfo :89-93, DumpVerbose :96-110); the connection summary of the
    captured payload is the caller's (the batch carries no payload).
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


def decode_records(buf) -> list[DropNotify]:
    """A packed array of records (bytes, numpy or a host copy of the tensor
    cfc_drop_notify_v4/v6 filled) -> DropNotify list, in order."""
    raw = bytes(memoryview(buf).cast("B"))
    if len(raw) % DROP_NOTIFY_LEN:
        raise ValueError("not a whole number of drop_notify records")
    return [DropNotify.decode(raw[i:i + DROP_NOTIFY_LEN])
            for i in range(0, len(raw), DROP_NOTIFY_LEN)]
