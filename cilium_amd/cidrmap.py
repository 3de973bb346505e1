"""Mirror of pkg/maps/cidrmap (cidrmap.go) and pkg/policy/prefilter.go.

cidrKey {u32 Prefixlen; [AddrSize]u8 Net}; the map key size is
4 + AddrSize (cidrmap.go:52-55, 177-183); value is 1 byte.  Fixed maps are
HASH with Prefixlen == full length, dynamic maps are LPM tries.
"""
from __future__ import annotations

import ipaddress
import struct
import threading

from .datapath import Datapath

MapName = "cilium_cidr_"         # cidrmap.go:32
MaxEntries = 16384
LPM_MAP_VALUE_SIZE = 1
BPF_MAP_TYPE_HASH, BPF_MAP_TYPE_LPM_TRIE = 1, 11
BPF_F_NO_PREALLOC = 1
maxLKeys, maxHKeys = 1024 * 64, 1024 * 1024 * 20   # prefilter.go:43-44


class CIDRMap:
    def __init__(self, dp, path, fd, addr_size, prefixlen, dyn):
        self.dp, self.path, self.Fd = dp, path, fd
        self.AddrSize, self.Prefixlen, self.PrefixIsDynamic = addr_size, prefixlen, dyn

    def _key(self, cidr: str):
        net = ipaddress.ip_network(cidr, strict=False)
        addr = net.network_address.packed[-self.AddrSize:]
        return net.prefixlen, struct.pack("<I", net.prefixlen) + addr

    def _check(self, plen, op):        # checkPrefixlen, cidrmap.go:75-85
        if self.Prefixlen != 0 and (
                (self.PrefixIsDynamic and self.Prefixlen < plen) or
                (not self.PrefixIsDynamic and self.Prefixlen != plen)):
            raise ValueError(f"Unable to {op} element with dynamic prefix length "
                             f"cm.Prefixlen={self.Prefixlen} key.Prefixlen={plen}")

    def InsertCIDR(self, cidr: str):
        plen, k = self._key(cidr)
        self._check(plen, "update")
        self.dp.update_element(self.Fd, k, b"\x00", 0)

    def DeleteCIDR(self, cidr: str):
        plen, k = self._key(cidr)
        self._check(plen, "delete")
        self.dp.delete_element(self.Fd, k)

    def CIDRExists(self, cidr: str) -> bool:
        plen, k = self._key(cidr)
        if self._check_ok(plen):
            return self.dp.lookup_element(self.Fd, k) is not None
        return False

    def _check_ok(self, plen):
        try:
            self._check(plen, "lookup")
            return True
        except ValueError:
            return False

    def CIDRDump(self):
        out = []
        for k in self.dp.keys(self.Fd):
            plen = struct.unpack_from("<I", k)[0]
            a = bytes(k[4:])
            ip = ipaddress.ip_address(a) if len(a) in (4, 16) else a
            out.append(f"{ip}/{plen}")
        return out

    def Close(self):
        self.dp.obj_close(self.Fd)


def OpenMapElems(dp: Datapath, path: str, prefixlen: int, prefixdyn: bool,
                 maxelem: int = MaxEntries) -> CIDRMap:
    """cidrmap.OpenMapElems (cidrmap.go:166-220)."""
    if prefixlen <= 0:
        raise ValueError("prefixlen must be > 0")
    nbytes = (prefixlen - 1) // 8 + 1
    mtype = BPF_MAP_TYPE_LPM_TRIE if prefixdyn else BPF_MAP_TYPE_HASH
    fd, _ = dp.open_or_create_map(path, mtype, 4 + nbytes, LPM_MAP_VALUE_SIZE,
                                  maxelem, BPF_F_NO_PREALLOC)
    return CIDRMap(dp, path, fd, nbytes, 0 if prefixdyn else prefixlen,
                   prefixdyn)


class PreFilter:
    """pkg/policy/prefilter.go: four maps v4/v6 x dyn(LPM)/fix(hash) with
    revisioned, all-or-nothing Insert/Delete."""

    V4Dyn, V4Fix, V6Dyn, V6Fix = range(4)

    def __init__(self, dp: Datapath, dyn4=False, dyn6=False, fix4=True,
                 fix6=True):
        # NewPreFilter (prefilter.go:276-298): dyn maps disabled by default
        self.revision = 1
        self.mutex = threading.Lock()
        self.maps = [None] * 4
        cfg = [(self.V4Dyn, 32, True, maxLKeys, "v4_dyn", dyn4),
               (self.V4Fix, 32, False, maxHKeys, "v4_fix", fix4),
               (self.V6Dyn, 128, True, maxLKeys, "v6_dyn", dyn6),
               (self.V6Fix, 128, False, maxHKeys, "v6_fix", fix6)]
        for which, plen, dyn, maxe, suffix, on in cfg:
            if on:
                self.maps[which] = OpenMapElems(dp, MapName + suffix, plen,
                                                dyn, maxe)

    def selectMap(self, cidr: str):              # prefilter.go:108-121
        net = ipaddress.ip_network(cidr, strict=False)
        bits = 32 if net.version == 4 else 128
        if bits == 32:
            return self.V4Fix if net.prefixlen == bits else self.V4Dyn
        return self.V6Fix if net.prefixlen == bits else self.V6Dyn

    def Insert(self, revision: int, cidrs):      # prefilter.go:125-159
        with self.mutex:
            if revision != 0 and self.revision != revision:
                raise ValueError(f"Latest revision is {self.revision} not {revision}")
            undo, err = [], None
            for c in cidrs:
                m = self.maps[self.selectMap(c)]
                if m is None:
                    err = ValueError(f"No map enabled for CIDR string {c}")
                    break
                try:
                    m.InsertCIDR(c)
                    undo.append(c)
                except (OSError, ValueError) as e:
                    err = ValueError(f"Error inserting CIDR string {c}: {e}")
                    break
            if err is None:
                self.revision += 1
                return
            for c in undo:
                self.maps[self.selectMap(c)].DeleteCIDR(c)
            raise err

    def Delete(self, revision: int, cidrs):      # prefilter.go:162-203
        with self.mutex:
            if revision != 0 and self.revision != revision:
                raise ValueError(f"Latest revision is {self.revision} not {revision}")
            for c in cidrs:
                m = self.maps[self.selectMap(c)]
                if m is None:
                    raise ValueError(f"No map enabled for CIDR string {c}")
                if not m.CIDRExists(c):
                    raise ValueError(f"No map entry for CIDR string {c}")
            undo, err = [], None
            for c in cidrs:
                try:
                    self.maps[self.selectMap(c)].DeleteCIDR(c)
                    undo.append(c)
                except (OSError, ValueError) as e:
                    err = ValueError(f"Error deleting CIDR string {c}: {e}")
                    break
            if err is None:
                self.revision += 1
                return
            for c in undo:
                self.maps[self.selectMap(c)].InsertCIDR(c)
            raise err

    def Dump(self):
        with self.mutex:
            out = []
            for m in self.maps:
                if m is not None:
                    out += m.CIDRDump()
            return out, self.revision
