"""Mirror of pkg/maps/ipcache (ipcache.go) and the datapath-facing part of
pkg/datapath/ipcache/listener.go.

Key {u32 Prefixlen; u16 Pad1; u8 Pad2; u8 Family; [16]u8 IP} with
Prefixlen = 32 static bits (pads + family) + the CIDR's mask length
(ipcache.go:57-123); value RemoteEndpointInfo {u32 SecurityIdentity;
[4]u8 TunnelEndpoint} (ipcache.go:127-130).
"""
from __future__ import annotations

import dataclasses
import ipaddress
import struct

from .datapath import Datapath

Name = "cilium_ipcache"              # ipcache.go:39
MaxEntries = 512000                  # ipcache.go:36
BPF_MAP_TYPE_LPM_TRIE = 11
BPF_F_NO_PREALLOC = 1
FamilyIPv4, FamilyIPv6 = 1, 2        # bpf/lib/common.h:139-140
_STATIC_PREFIX_BITS = 32             # getStaticPrefixBits, ipcache.go:72-77


@dataclasses.dataclass(frozen=True)
class Key:
    Prefixlen: int
    Family: int
    IP: bytes                        # 16 bytes
    Pad1: int = 0
    Pad2: int = 0

    def pack(self) -> bytes:
        return struct.pack("<IHBB", self.Prefixlen, self.Pad1, self.Pad2,
                           self.Family) + self.IP

    @classmethod
    def unpack(cls, b: bytes):
        p, p1, p2, f = struct.unpack_from("<IHBB", b)
        return cls(p, f, bytes(b[8:24]), p1, p2)

    def String(self):
        plen = self.Prefixlen - _STATIC_PREFIX_BITS
        if self.Family == FamilyIPv4:
            return f"{ipaddress.IPv4Address(self.IP[:4])}/{plen}"
        return f"{ipaddress.IPv6Address(self.IP)}/{plen}"


def NewKey(cidr: str) -> Key:
    """ipcache.NewKey(ip, mask) (ipcache.go:102-123) from 'a.b.c.d/len'."""
    net = ipaddress.ip_network(cidr, strict=False)
    if net.version == 4:
        ip = net.network_address.packed + bytes(12)
        fam = FamilyIPv4
    else:
        ip = net.network_address.packed
        fam = FamilyIPv6
    return Key(_STATIC_PREFIX_BITS + net.prefixlen, fam, ip)


@dataclasses.dataclass
class RemoteEndpointInfo:
    SecurityIdentity: int
    TunnelEndpoint: bytes = bytes(4)

    def pack(self):
        return struct.pack("<I", self.SecurityIdentity) + self.TunnelEndpoint

    @classmethod
    def unpack(cls, b):
        return cls(struct.unpack_from("<I", b)[0], bytes(b[4:8]))


class Map:
    """ipcache.Map (ipcache.go:142-200) on a Datapath."""

    def __init__(self, dp: Datapath, name: str = Name, max_entries=MaxEntries):
        self.dp = dp
        self.fd, _ = dp.open_or_create_map(name, BPF_MAP_TYPE_LPM_TRIE, 24, 8,
                                           max_entries, BPF_F_NO_PREALLOC)

    def Update(self, k: Key, v: RemoteEndpointInfo):
        self.dp.update_element(self.fd, k.pack(), v.pack(), 0)

    def Delete(self, k: Key):
        self.dp.delete_element(self.fd, k.pack())

    def Lookup(self, k: Key):
        v = self.dp.lookup_element(self.fd, k.pack())
        return None if v is None else RemoteEndpointInfo.unpack(v)

    def Dump(self):
        out = {}
        for k in self.dp.keys(self.fd):
            v = self.dp.lookup_element(self.fd, k)
            out[Key.unpack(k)] = RemoteEndpointInfo.unpack(v)
        return out

    def SupportsDelete(self):        # ipcache.go:218: LPM delete is supported
        return True


class BPFListener:
    """pkg/datapath/ipcache/listener.go:78-127 OnIPIdentityCacheChange."""

    Upsert, Delete = 0, 1

    def __init__(self, m: Map):
        self.m = m

    def OnIPIdentityCacheChange(self, modType, cidr: str, identity: int,
                                hostIP: bytes = bytes(4)):
        k = NewKey(cidr)
        if modType == self.Upsert:
            self.m.Update(k, RemoteEndpointInfo(identity, hostIP))
        else:
            self.m.Delete(k)
