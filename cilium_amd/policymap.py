"""Mirror of pkg/maps/policymap (policymap.go, trafficdirection.go).

Same key/value byte layouts as the reference:
  PolicyKey   {u32 Identity; u16 DestPort (network order); u8 Nexthdr;
               u8 TrafficDirection}                       policymap.go:64-69
  PolicyEntry {u16 ProxyPort (network order); u16 pad[3]; u64 Packets;
               u64 Bytes}                                  policymap.go:73-80
backed by a `cilium_policy_<endpoint id>` map of the Datapath context.
"""
from __future__ import annotations

import dataclasses
import struct

from .datapath import Datapath

MapName = "cilium_policy_"          # policymap.go:33
MaxEntries = 16384                  # policymap.go:37
BPF_MAP_TYPE_HASH = 1
Ingress, Egress = 0, 1              # trafficdirection.go:20-29


def _htons(x):
    return ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)


@dataclasses.dataclass(frozen=True)
class PolicyKey:
    Identity: int
    DestPort: int          # network byte order (as stored)
    Nexthdr: int
    TrafficDirection: int

    def pack(self) -> bytes:
        return struct.pack("<IHBB", self.Identity, self.DestPort, self.Nexthdr,
                           self.TrafficDirection)

    @classmethod
    def unpack(cls, b: bytes):
        return cls(*struct.unpack("<IHBB", b))

    def GetIdentity(self):
        return self.Identity

    def GetPort(self):                       # policymap.go:124 (host order)
        return _htons(self.DestPort)

    def GetProto(self):
        return self.Nexthdr

    def GetDirection(self):
        return self.TrafficDirection

    def ToHost(self):                        # policymap.go:140
        return dataclasses.replace(self, DestPort=_htons(self.DestPort))

    def ToNetwork(self):                     # policymap.go:152
        return dataclasses.replace(self, DestPort=_htons(self.DestPort))

    def String(self):                        # policymap.go:108-115
        d = "Egress" if self.TrafficDirection == Egress else "Ingress"
        if self.DestPort != 0:
            return f"{d}: {self.Identity} {self.GetPort()}/{self.Nexthdr}"
        return f"{d}: {self.Identity}"


@dataclasses.dataclass
class PolicyEntry:
    ProxyPort: int = 0     # network byte order
    Packets: int = 0
    Bytes: int = 0

    def pack(self) -> bytes:
        return struct.pack("<H6xQQ", self.ProxyPort, self.Packets, self.Bytes)

    @classmethod
    def unpack(cls, b: bytes):
        return cls(*struct.unpack("<H6xQQ", b))

    def Add(self, o: "PolicyEntry"):        # policymap.go:82
        self.Packets += o.Packets
        self.Bytes += o.Bytes


@dataclasses.dataclass
class PolicyEntryDump:
    Key: PolicyKey
    PolicyEntry: PolicyEntry


class PolicyEntriesDump(list):
    """A dump sorted for display (policymap.go:88-106): by traffic
    direction, then identity."""

    def Less(self, i: int, j: int) -> bool:
        a, b = self[i].Key, self[j].Key
        if a.TrafficDirection < b.TrafficDirection:
            return True
        return a.TrafficDirection <= b.TrafficDirection and a.Identity < b.Identity

    def Sort(self):
        self.sort(key=lambda e: (e.Key.TrafficDirection, e.Key.Identity))


class PolicyMap:
    def __init__(self, dp: Datapath, path: str, fd: int):
        self.dp, self.path, self.Fd = dp, path, fd

    # policymap.go:164 — dport/proxy are host order here, stored network order
    def AllowKey(self, k: PolicyKey, proxyPort: int = 0):
        return self.Allow(k.Identity, k.DestPort, k.Nexthdr,
                          k.TrafficDirection, proxyPort)

    def Allow(self, id: int, dport: int, proto: int, trafficDirection: int,
              proxyPort: int = 0):
        key = PolicyKey(id, _htons(dport), proto, trafficDirection)
        entry = PolicyEntry(ProxyPort=_htons(proxyPort))
        self.dp.update_element(self.Fd, key.pack(), entry.pack(), 0)

    def Exists(self, id, dport, proto, trafficDirection) -> bool:
        key = PolicyKey(id, _htons(dport), proto, trafficDirection)
        return self.dp.lookup_element(self.Fd, key.pack()) is not None

    def DeleteKey(self, k: PolicyKey):
        self.dp.delete_element(self.Fd, k.ToNetwork().pack())

    def Delete(self, id, dport, proto, trafficDirection):
        key = PolicyKey(id, _htons(dport), proto, trafficDirection)
        self.dp.delete_element(self.Fd, key.pack())

    def DeleteEntry(self, e: PolicyEntryDump):
        self.dp.delete_element(self.Fd, e.Key.pack())

    def Lookup(self, k: PolicyKey):
        v = self.dp.lookup_element(self.Fd, k.pack())
        return None if v is None else PolicyEntry.unpack(v)

    def DumpToSlice(self):                   # policymap.go:224
        out = []
        for k in self.dp.keys(self.Fd):
            v = self.dp.lookup_element(self.Fd, k)
            if v is not None:
                out.append(PolicyEntryDump(PolicyKey.unpack(k),
                                           PolicyEntry.unpack(v)))
        return out

    def Flush(self):                         # policymap.go:258
        for k in self.dp.keys(self.Fd):
            try:
                self.dp.delete_element(self.Fd, k)
            except OSError:
                pass

    def String(self):
        return self.path

    def Close(self):
        self.dp.obj_close(self.Fd)


def OpenMap(dp: Datapath, path: str):
    """policymap.OpenMap (policymap.go:330) -> (PolicyMap, isNew)."""
    fd, is_new = dp.open_or_create_map(path, BPF_MAP_TYPE_HASH, 8, 24,
                                       MaxEntries, 0)
    return PolicyMap(dp, path, fd), is_new


def path_for(endpoint_id: int, root="/sys/fs/bpf/tc/globals"):
    return f"{root}/{MapName}{endpoint_id}"
