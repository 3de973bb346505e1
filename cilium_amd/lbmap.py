"""pkg/maps/lbmap over the engine's map API: cilium_lb4_services and
cilium_lb4_reverse_nat with the reference's key and value layouts
(lbmap/ipv4.go: Service4Key {Address, Port, Slave}, Service4Value {Address,
Port, Count, RevNat, Weight}, RevNat4Key, RevNat4Value) and byte order
(ToNetwork: ports, rev-NAT ids and weights network order; count host order),
and UpdateService's slot layout (lbmap.go:351-427, bpfservice.go): backends
in slots 1..n kept stable across updates (a removed backend's slots become
holes refilled by another backend), the master slot 0 carrying the count.  IPv6 (lbmap/ipv6.go):
cilium_lb6_services {Service6Key: Service6Value} and cilium_lb6_reverse_nat,
the same layouts with 16-byte addresses (LBMap6)."""
from __future__ import annotations

import socket
import struct

from .datapath import Datapath

MaxEntries = 65536                        # lbmap.go MaxEntries
Service4MapName = "cilium_lb4_services"
RevNat4MapName = "cilium_lb4_reverse_nat"
Service6MapName = "cilium_lb6_services"
RevNat6MapName = "cilium_lb6_reverse_nat"
MAP_TYPE_HASH = 1


def _be16(x):
    return struct.unpack("<H", struct.pack(">H", x & 0xFFFF))[0]


def _ip(ip):
    return ip if isinstance(ip, bytes) else socket.inet_aton(ip)


def _ip6(ip):
    return ip if isinstance(ip, bytes) else socket.inet_pton(socket.AF_INET6, ip)


class Service4Key:
    """struct lb4_key (bpf/lib/common.h:427-431); port in host order here,
    pack() is ToNetwork()."""

    def __init__(self, ip, port, slave=0):
        self.address, self.port, self.slave = _ip(ip), int(port), int(slave)

    def pack(self):
        return self.address + struct.pack("<HH", _be16(self.port), self.slave)

    def String(self):                                   # ipv4.go:95-97
        return f"{socket.inet_ntoa(self.address)}:{self.port}"


class Service4Value:
    """struct lb4_service (common.h:433-439)."""

    def __init__(self, count=0, target="0.0.0.0", port=0, rev_nat=0, weight=0):
        self.count, self.target, self.port = int(count), _ip(target), int(port)
        self.rev_nat, self.weight = int(rev_nat), int(weight)

    def pack(self):
        return self.target + struct.pack("<HHHH", _be16(self.port), self.count,
                                         _be16(self.rev_nat), _be16(self.weight))

    def String(self):                                   # ipv4.go:196-198
        return f"{socket.inet_ntoa(self.target)}:{self.port} ({self.rev_nat})"


class RevNat4Value:
    def __init__(self, ip, port):
        self.address, self.port = _ip(ip), int(port)

    def pack(self):
        return self.address + struct.pack("<H", _be16(self.port))


class BpfBackend:
    """bpfBackend (bpfservice.go): the backend a slot holds; a hole is a
    slot whose backend was removed, filled with a copy of another one."""

    def __init__(self, value, is_hole=False):
        self.bpfValue, self.id, self.isHole = value, value.String(), is_hole


class BpfService:
    """bpfService (pkg/maps/lbmap/bpfservice.go): the slot layout of one
    frontend.  A removed backend's slots become holes filled with the
    remaining backend that fills the fewest slots, so every other backend
    keeps its slot (CT entries hold slot numbers, lb4_local); a new backend
    takes the oldest hole, else the next slot.  The reference breaks ties
    (and orders the removed slots) in Go map order; here the backend first
    seen in slot order wins and slots go in ascending order."""

    def __init__(self, key):
        self.frontendKey = key
        self.holes = []
        self.backendsByMapIndex = {}
        self.uniqueBackends = {}

    def addBackend(self, backend):
        if self.holes:
            index = self.holes.pop(0)
            self.backendsByMapIndex[index] = BpfBackend(backend)
        else:
            self.backendsByMapIndex[len(self.uniqueBackends) + 1] = BpfBackend(backend)
        self.uniqueBackends[backend.String()] = backend

    def deleteBackend(self, backend):
        rid = backend.String()
        remove, count = [], {}
        for index in sorted(self.backendsByMapIndex):
            b = self.backendsByMapIndex[index]
            if b.id == rid:
                remove.append(index)
            else:
                count[b.id] = count.get(b.id, 0) + 1
        fill = min(count, key=lambda k: count[k]) if count else ""
        if not fill:
            self.holes = []
            self.backendsByMapIndex = {}
        else:
            for index in remove:
                if not self.backendsByMapIndex[index].isHole:
                    self.holes.append(index)
                self.backendsByMapIndex[index] = BpfBackend(self.uniqueBackends[fill], True)
        self.uniqueBackends.pop(rid, None)

    def getBackends(self):
        return [self.backendsByMapIndex[i].bpfValue
                for i in range(1, len(self.backendsByMapIndex) + 1)]


class LBMapCache:
    """lbmapCache (bpfservice.go): one BpfService per frontend."""

    def __init__(self):
        self.entries = {}

    def prepareUpdate(self, fe, backends) -> BpfService:
        svc = self.entries.setdefault(fe.String(), BpfService(fe))
        new = {b.String(): b for b in backends}
        for key, b in list(svc.uniqueBackends.items()):
            if key not in new:
                svc.deleteBackend(b)
        for b in backends:
            if b.String() not in svc.uniqueBackends:
                svc.addBackend(b)
        return svc

    def delete(self, fe):
        self.entries.pop(fe.String(), None)


class LBMap:
    def __init__(self, dp: Datapath):
        self.dp = dp
        self.cache = LBMapCache()
        self.svc, _ = dp.open_or_create_map(Service4MapName, MAP_TYPE_HASH, 8, 12,
                                            MaxEntries)
        self.rnat, _ = dp.open_or_create_map(RevNat4MapName, MAP_TYPE_HASH, 2, 6,
                                             MaxEntries)

    def UpdateService(self, fe: Service4Key, backends, add_revnat=True, revnat_id=0):
        """lbmap.go:351-427 UpdateService: the frontend's slot layout from
        the cache (prepareUpdate: holes keep the other backends' slots), slot
        i + 1 for each, the reverse NAT entry revnat_id -> frontend, then
        the master slot (count, non-zero weights), then stale slots past the
        new count removed."""
        backends = self.cache.prepareUpdate(fe, backends).getBackends()
        old = self.dp.lookup_element(self.svc, Service4Key(fe.address, fe.port, 0).pack())
        existing = struct.unpack_from("<H", old, 6)[0] if old else 0
        for i, be in enumerate(backends):
            self.dp.update_element(self.svc, Service4Key(fe.address, fe.port, i + 1).pack(),
                                   be.pack())
        if add_revnat:
            self.dp.update_element(self.rnat, struct.pack("<H", _be16(revnat_id)),
                                   RevNat4Value(fe.address, fe.port).pack())
        nz = sum(1 for be in backends if be.weight)
        self.dp.update_element(self.svc, Service4Key(fe.address, fe.port, 0).pack(),
                               Service4Value(len(backends), weight=nz).pack())
        for i in range(len(backends) + 1, existing + 1):
            self.dp.delete_element(self.svc, Service4Key(fe.address, fe.port, i).pack())

    def DeleteService(self, fe: Service4Key):
        """The frontend's master and backend slots (the daemon's loop over
        lbmap.go:150-167 DeleteService), and its cache entry."""
        self.cache.delete(fe)
        old = self.dp.lookup_element(self.svc, Service4Key(fe.address, fe.port, 0).pack())
        n = struct.unpack_from("<H", old, 6)[0] if old else 0
        for i in range(n, -1, -1):
            k = Service4Key(fe.address, fe.port, i).pack()
            if self.dp.lookup_element(self.svc, k) is not None:
                self.dp.delete_element(self.svc, k)

    def load_rows(self, lb4, revnat4):
        """Raw synth.LB4_DT / REVNAT4_DT rows (already in map byte order)."""
        import numpy as np
        if lb4 is not None and len(lb4):
            b = np.ascontiguousarray(lb4).view(np.uint8).reshape(len(lb4), 20)
            self.dp.update_batch(self.svc, b[:, :8], b[:, 8:20])
        if revnat4 is not None and len(revnat4):
            b = np.ascontiguousarray(revnat4).view(np.uint8).reshape(len(revnat4), 8)
            self.dp.update_batch(self.rnat, b[:, :2], b[:, 2:8])


class Service6Key(Service4Key):
    """struct lb6_key (common.h:408-412)."""

    def __init__(self, ip, port, slave=0):
        self.address, self.port, self.slave = _ip6(ip), int(port), int(slave)

    def String(self):                                   # ipv6.go:123-125
        return f"[{socket.inet_ntop(socket.AF_INET6, self.address)}]:{self.port}"


class Service6Value(Service4Value):
    """struct lb6_service (common.h:414-420)."""

    def __init__(self, count=0, target="::", port=0, rev_nat=0, weight=0):
        self.count, self.target, self.port = int(count), _ip6(target), int(port)
        self.rev_nat, self.weight = int(rev_nat), int(weight)

    def String(self):                                   # ipv6.go:192-194
        return f"[{socket.inet_ntop(socket.AF_INET6, self.target)}]:{self.port} ({self.rev_nat})"


class RevNat6Value(RevNat4Value):
    """struct lb6_reverse_nat (common.h:422-425)."""

    def __init__(self, ip, port):
        self.address, self.port = _ip6(ip), int(port)


class LBMap6(LBMap):
    """The IPv6 maps (lbmap/ipv6.go) with LBMap's UpdateService / DeleteService
    slot discipline."""

    def __init__(self, dp: Datapath):
        self.dp = dp
        self.cache = LBMapCache()
        self.svc, _ = dp.open_or_create_map(Service6MapName, MAP_TYPE_HASH, 20, 24,
                                            MaxEntries)
        self.rnat, _ = dp.open_or_create_map(RevNat6MapName, MAP_TYPE_HASH, 2, 18,
                                             MaxEntries)

    def UpdateService(self, fe: Service6Key, backends, add_revnat=True, revnat_id=0):
        backends = self.cache.prepareUpdate(fe, backends).getBackends()
        old = self.dp.lookup_element(self.svc, Service6Key(fe.address, fe.port, 0).pack())
        existing = struct.unpack_from("<H", old, 18)[0] if old else 0
        for i, be in enumerate(backends):
            self.dp.update_element(self.svc, Service6Key(fe.address, fe.port, i + 1).pack(),
                                   be.pack())
        if add_revnat:
            self.dp.update_element(self.rnat, struct.pack("<H", _be16(revnat_id)),
                                   RevNat6Value(fe.address, fe.port).pack())
        nz = sum(1 for be in backends if be.weight)
        self.dp.update_element(self.svc, Service6Key(fe.address, fe.port, 0).pack(),
                               Service6Value(len(backends), weight=nz).pack())
        for i in range(len(backends) + 1, existing + 1):
            self.dp.delete_element(self.svc, Service6Key(fe.address, fe.port, i).pack())

    def DeleteService(self, fe: Service6Key):
        self.cache.delete(fe)
        old = self.dp.lookup_element(self.svc, Service6Key(fe.address, fe.port, 0).pack())
        n = struct.unpack_from("<H", old, 18)[0] if old else 0
        for i in range(n, -1, -1):
            k = Service6Key(fe.address, fe.port, i).pack()
            if self.dp.lookup_element(self.svc, k) is not None:
                self.dp.delete_element(self.svc, k)

    def load_rows(self, lb6, revnat6):
        """Raw synth.LB6_DT / REVNAT6_DT rows (already in map byte order)."""
        import numpy as np
        if lb6 is not None and len(lb6):
            b = np.ascontiguousarray(lb6).view(np.uint8).reshape(len(lb6), 44)
            self.dp.update_batch(self.svc, b[:, :20], b[:, 20:44])
        if revnat6 is not None and len(revnat6):
            b = np.ascontiguousarray(revnat6).view(np.uint8).reshape(len(revnat6), 20)
            self.dp.update_batch(self.rnat, b[:, :2], b[:, 2:20])
