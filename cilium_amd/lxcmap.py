"""Mirror of pkg/maps/lxcmap (lxcmap.go) + pkg/bpf/endpoint.go EndpointKey.

EndpointKey {[16]u8 IP; u8 Family; u8 Pad1; u16 Pad2}       (20 bytes)
EndpointInfo {u32 IfIndex; u16 Unused; u16 LxcID; u32 Flags; u32 _;
              u64 MAC; u64 NodeMAC; [4]u32 Pad}               (48 bytes)
"""
from __future__ import annotations

import dataclasses
import ipaddress
import struct

from .datapath import Datapath

MapName = "cilium_lxc"          # lxcmap.go:30
MaxEntries = 65535              # lxcmap.go:33
EndpointFlagHost = 1            # lxcmap.go:98
EndpointKeyIPv4, EndpointKeyIPv6 = 1, 2
BPF_MAP_TYPE_HASH = 1


@dataclasses.dataclass(frozen=True)
class EndpointKey:
    IP: bytes
    Family: int
    Pad1: int = 0
    Pad2: int = 0

    def pack(self):
        return self.IP + struct.pack("<BBH", self.Family, self.Pad1, self.Pad2)

    @classmethod
    def unpack(cls, b):
        f, p1, p2 = struct.unpack_from("<BBH", b, 16)
        return cls(bytes(b[:16]), f, p1, p2)


def NewEndpointKey(ip: str) -> EndpointKey:
    """bpf.NewEndpointKey (pkg/bpf/endpoint.go:49)."""
    a = ipaddress.ip_address(ip)
    if a.version == 4:
        return EndpointKey(a.packed + bytes(12), EndpointKeyIPv4)
    return EndpointKey(a.packed, EndpointKeyIPv6)


@dataclasses.dataclass
class EndpointInfo:
    IfIndex: int = 0
    LxcID: int = 0
    Flags: int = 0
    MAC: int = 0
    NodeMAC: int = 0

    def pack(self):
        return struct.pack("<IHHI4xQQ16x", self.IfIndex, 0, self.LxcID,
                           self.Flags, self.MAC, self.NodeMAC)

    @classmethod
    def unpack(cls, b):
        ifi, _, lxc, fl, mac, nmac = struct.unpack_from("<IHHI4xQQ", b)
        return cls(ifi, lxc, fl, mac, nmac)

    def IsHost(self):
        return bool(self.Flags & EndpointFlagHost)


class LXCMap:
    def __init__(self, dp: Datapath):
        self.dp = dp
        self.fd, _ = dp.open_or_create_map(MapName, BPF_MAP_TYPE_HASH, 20, 48,
                                           MaxEntries, 0)

    def WriteEndpoint(self, keys, info: EndpointInfo):
        """lxcmap.WriteEndpoint (lxcmap.go:160): one value, all its keys."""
        for k in keys:
            self.dp.update_element(self.fd, k.pack(), info.pack(), 0)

    def AddHostEntry(self, ip: str):
        """lxcmap.AddHostEntry (lxcmap.go:177)."""
        self.dp.update_element(self.fd, NewEndpointKey(ip).pack(),
                               EndpointInfo(Flags=EndpointFlagHost).pack(), 0)

    def DeleteEntry(self, ip: str):
        self.dp.delete_element(self.fd, NewEndpointKey(ip).pack())

    def Lookup(self, ip: str):
        v = self.dp.lookup_element(self.fd, NewEndpointKey(ip).pack())
        return None if v is None else EndpointInfo.unpack(v)
