"""Datapath: one libcfc context (one GPU) seen from Python.

Two halves, as in include/cfc.h:
  * the pkg/bpf-shaped map API (`open_or_create_map`, `update_element`, ...)
    that pkg/maps/* mirrors in this package build on;
  * `classify_v4` / `classify_v6`, the batched replacement of the
    reference's per-packet programs, over torch tensors resident on the GPU.
"""
from __future__ import annotations

import ctypes
import dataclasses

from . import _lib as L


@dataclasses.dataclass
class HeaderBatchV4:
    """Device SoA batch (all torch int32 tensors on the same GPU)."""
    saddr: "torch.Tensor"
    daddr: "torch.Tensor"
    ports: "torch.Tensor"     # sport | dport << 16 (be16 raw each)
    meta: "torch.Tensor"      # proto | flags << 8 | len << 16
    mark: "torch.Tensor | None" = None
    tcp_flags: "torch.Tensor | None" = None   # uint8 TCP header byte 13
    hash: "torch.Tensor | None" = None        # skb->hash (lb4_select_slave)

    def __len__(self):
        return int(self.saddr.numel())

    def slice(self, a, b):
        """headers [a, b) (views of the same device memory)"""
        sl = lambda x: None if x is None else x[a:b]   # noqa: E731
        return type(self)(*(sl(getattr(self, f.name))
                            for f in dataclasses.fields(self)))


@dataclasses.dataclass
class HeaderBatchV6:
    """Device SoA batch of IPv6 headers: saddr/daddr int32 tensors of shape
    (n, 4) (16 network-order bytes per address), the rest as in V4."""
    saddr: "torch.Tensor"
    daddr: "torch.Tensor"
    ports: "torch.Tensor"
    meta: "torch.Tensor"      # proto | flags << 8 | len << 16 (HF_EXTHDR)
    mark: "torch.Tensor | None" = None
    tcp_flags: "torch.Tensor | None" = None   # uint8 TCP header byte 13
    hash: "torch.Tensor | None" = None        # skb->hash (lb6_select_slave)

    def __len__(self):
        return int(self.ports.numel())

    def slice(self, a, b):
        """headers [a, b) (views of the same device memory)"""
        sl = lambda x: None if x is None else x[a:b]   # noqa: E731
        return type(self)(*(sl(getattr(self, f.name))
                            for f in dataclasses.fields(self)))


@dataclasses.dataclass
class Verdicts:
    verdict: "torch.Tensor"   # int32
    identity: "torch.Tensor"  # int32 (u32 bits)
    action: "torch.Tensor | None"  # uint8
    ct: "torch.Tensor | None" = None  # uint8 CT byte (cfc.h CFC_CT_*)
    notify: "torch.Tensor | None" = None  # int32 drop-notify site (CFC_NT_*)
    # the packet as the programs left it (cfc_out.pkt_*): int32 (n, 3) saddr,
    # daddr, first L4 word (IPv4); (n, 9) saddr[4], daddr[4], L4 word (IPv6)
    pkt: "torch.Tensor | None" = None
    # IPv6: the three arrays the library writes (saddr rows, daddr rows, L4
    # words, 9n int32); pkt is assembled from them (cfc_ct_apply_v6 may
    # rewrite them: ct_apply assembles pkt again)
    pkt_raw: "torch.Tensor | None" = None


def pack_v4(h, device="cuda"):
    """synth.Headers (numpy) -> HeaderBatchV4 on `device`."""
    import numpy as np
    import torch
    ports = (h.sport.astype(np.uint32) | (h.dport.astype(np.uint32) << 16))
    meta = (h.proto.astype(np.uint32) | (h.flags.astype(np.uint32) << 8)
            | (h.length.astype(np.uint32) << 16))

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32)
                                .view(np.int32)).to(device)
    from .synth import tcp_flags_of
    hs = getattr(h, "hash", None)
    return HeaderBatchV4(t(h.saddr), t(h.daddr), t(ports), t(meta),
                         t(h.mark) if h.mark is not None else None,
                         torch.from_numpy(tcp_flags_of(h).copy()).to(device),
                         t(hs) if hs is not None else None)


def pack_v6(h, device="cuda"):
    """synth.Headers (family 6, numpy) -> HeaderBatchV6 on `device`.  The
    synth flag HF_EXTHDR (4) becomes the ABI's CFC_HF_EXTHDR bit."""
    import numpy as np
    import torch
    ports = (h.sport.astype(np.uint32) | (h.dport.astype(np.uint32) << 16))
    meta = (h.proto.astype(np.uint32) | (h.flags.astype(np.uint32) << 8)
            | (h.length.astype(np.uint32) << 16))

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(device)
    from .synth import tcp_flags_of
    hs = getattr(h, "hash", None)
    return HeaderBatchV6(t(np.ascontiguousarray(h.saddr, np.uint8)).view(-1, 4),
                         t(np.ascontiguousarray(h.daddr, np.uint8)).view(-1, 4),
                         t(ports), t(meta),
                         t(h.mark.astype(np.uint32)) if h.mark is not None else None,
                         torch.from_numpy(tcp_flags_of(h).copy()).to(device),
                         t(np.asarray(hs, np.uint32)) if hs is not None else None)


def pack(h, device="cuda"):
    return pack_v4(h, device) if h.family == 4 else pack_v6(h, device)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def hdr_struct(batch, n=None):
    """cfc_hdr_v4 / cfc_hdr_v6 of a device batch (optionally its first n)."""
    v6 = isinstance(batch, HeaderBatchV6)
    args = (_ptr(batch.saddr), _ptr(batch.daddr), _ptr(batch.ports),
            _ptr(batch.meta), _ptr(batch.mark), _ptr(batch.tcp_flags),
            len(batch) if n is None else n)
    return L.HdrV6(*args, _ptr(batch.hash)) if v6 else L.HdrV4(*args, _ptr(batch.hash))


def _pkt6(raw):
    n = raw.numel() // 9
    return torch_cat([raw[:4 * n].view(n, 4), raw[4 * n:8 * n].view(n, 4),
                      raw[8 * n:].view(n, 1)])


def torch_cat(parts):
    import torch
    return torch.cat(parts, 1)


def out_struct(out):
    pk = getattr(out, "pkt", None)
    raw = getattr(out, "pkt_raw", None)
    if raw is not None:   # IPv6: the library's own three arrays
        n = raw.numel() // 9
        return L.Out(_ptr(out.verdict), _ptr(out.identity), _ptr(out.action),
                     _ptr(out.ct), _ptr(out.notify), _ptr(raw[:4 * n]),
                     _ptr(raw[4 * n:8 * n]), _ptr(raw[8 * n:]))
    cols = (None, None, None) if pk is None else (pk[:, 0], pk[:, 1], pk[:, 2])
    return L.Out(_ptr(out.verdict), _ptr(out.identity), _ptr(out.action),
                 _ptr(out.ct), _ptr(out.notify), *[_col_ptr(c) for c in cols])


def _col_ptr(c):
    # a column of the (n, 3) packet output: every third int32 — the ABI wants
    # three separate arrays, so the tensor is laid out column-major (3, n).T
    return ctypes.c_void_p(c.data_ptr()) if c is not None else None


def _stream_handle(stream):
    if stream is None:
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


class Datapath:
    def __init__(self, device: int = 0):
        self.L = L.lib()
        self.device = device
        self.h = ctypes.c_void_p()
        L.check(self.L.cfc_open(device, ctypes.byref(self.h)), "cfc_open")
        self._vsz = {}
        self._ksz = {}

    def close(self):
        if self.h:
            self.L.cfc_close(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------ pkg/bpf mirror
    def open_or_create_map(self, path, map_type, key_size, value_size,
                           max_entries, flags=0):
        """bpf.OpenOrCreateMap (pkg/bpf/bpf.go:371) -> (fd, is_new)."""
        fd, created = ctypes.c_int(), ctypes.c_int()
        L.check(self.L.cfc_map_open(self.h, path.encode(), map_type, key_size,
                                    value_size, max_entries, flags,
                                    ctypes.byref(fd), ctypes.byref(created)),
                f"open map {path}")
        self._ksz[fd.value] = key_size
        self._vsz[fd.value] = value_size if map_type != 5 else ((value_size + 7) & ~7)
        return fd.value, bool(created.value)

    def update_element(self, fd, key: bytes, value: bytes, flags=0):
        """bpf.UpdateElement (pkg/bpf/bpf.go:153)."""
        L.check(self.L.cfc_map_update(self.h, fd, key, value, flags),
                "update element")

    def update_batch(self, fd, keys, values, flags=0):
        """cfc_map_update_batch (BPF_MAP_UPDATE_BATCH): numpy (n, ksz) keys
        and (n, vsz) values."""
        import numpy as np
        keys = np.ascontiguousarray(keys, np.uint8)
        values = np.ascontiguousarray(values, np.uint8)
        assert len(keys) == len(values)
        L.check(self.L.cfc_map_update_batch(self.h, fd, keys.ctypes.data,
                                            values.ctypes.data, len(keys),
                                            flags), "update batch")

    def lookup_element(self, fd, key: bytes):
        """bpf.LookupElement (pkg/bpf/bpf.go:177) -> value bytes or None."""
        buf = ctypes.create_string_buffer(self._vsz[fd])
        rc = self.L.cfc_map_lookup(self.h, fd, key, buf)
        if rc == -2:  # ENOENT
            return None
        L.check(rc, "lookup element")
        return buf.raw

    def delete_element(self, fd, key: bytes):
        """bpf.DeleteElement (pkg/bpf/bpf.go:214)."""
        L.check(self.L.cfc_map_delete(self.h, fd, key), "delete element")

    def get_next_key(self, fd, key: bytes | None):
        """bpf.GetNextKey (pkg/bpf/bpf.go:225) -> next key or None at end."""
        buf = ctypes.create_string_buffer(self._ksz[fd])
        rc = self.L.cfc_map_get_next_key(self.h, fd, key, buf)
        if rc == -2:
            return None
        L.check(rc, "get next key")
        return buf.raw

    def dump(self, fd):
        """cfc_map_dump -> (keys (n, key_size) u8, values (n, value_size)
        u8) numpy arrays, in iteration order."""
        import numpy as np
        n = ctypes.c_uint64()
        L.check(self.L.cfc_map_dump(self.h, fd, None, None, 0, ctypes.byref(n)), "dump")
        k = np.zeros((n.value, self._ksz[fd]), np.uint8)
        v = np.zeros((n.value, self._vsz[fd]), np.uint8)
        if n.value:
            L.check(self.L.cfc_map_dump(self.h, fd, k.ctypes.data, v.ctypes.data,
                                        n.value, ctypes.byref(n)), "dump")
        return k, v

    def keys(self, fd):
        out, k = [], None
        while True:
            k = self.get_next_key(fd, k)
            if k is None:
                return out
            out.append(k)

    def obj_close(self, fd):
        L.check(self.L.cfc_map_close(self.h, fd), "close map")

    def endpoint_config(self, lxc_id, seclabel):
        L.check(self.L.cfc_endpoint_config(self.h, lxc_id, seclabel),
                "endpoint config")

    def set_node_config(self, ipv4_cluster_range, ipv4_cluster_mask,
                        router_ip6, host_ifindex=1):
        """cfc_set_node_config: what the agent writes into node_config.h
        (daemon/daemon.go:916-934).  The IPv4 values are raw be32 (the
        header's %#x), router_ip6 is 16 bytes."""
        c = L.NodeConfig()
        c.ipv4_cluster_range = int(ipv4_cluster_range) & 0xFFFFFFFF
        c.ipv4_cluster_mask = int(ipv4_cluster_mask) & 0xFFFFFFFF
        c.router_ip6[:] = list(bytes(bytearray(router_ip6)))
        c.host_ifindex = int(host_ifindex)
        L.check(self.L.cfc_set_node_config(self.h, ctypes.byref(c)),
                "node config")

    def node_config(self):
        c = L.NodeConfig()
        L.check(self.L.cfc_get_node_config(self.h, ctypes.byref(c)), "node config")
        return (c.ipv4_cluster_range, c.ipv4_cluster_mask, bytes(c.router_ip6),
                c.host_ifindex)

    # ------------------------------------------------ datapath
    def _stream(self, stream):
        if self.device == L.CFC_DEVICE_NONE:
            return ctypes.c_void_p()
        return _stream_handle(stream)

    def set_option(self, option, value):
        """cfc_set_option: L.OPT_LPM4 (ipcache layout, next commit) or
        L.OPT_TIMING (per-call kernel events)."""
        L.check(self.L.cfc_set_option(self.h, option, value), "set option")

    def timing_collect(self):
        """Kernel device time of the calls since the last collect (needs
        OPT_TIMING): {launches, classify_ms, count_ms} (sums over every
        call) and the same three for the IPv6 calls among them (*_v6)."""
        t = L.Timing()
        L.check(self.L.cfc_timing_collect(self.h, ctypes.byref(t)), "timing")
        return {f: getattr(t, f) for f, _ in L.Timing._fields_}

    def commit(self, stream=None):
        L.check(self.L.cfc_commit(self.h, self._stream(stream)),"commit")

    def classify_v4(self, batch: HeaderBatchV4, mode=L.MODE_INGRESS, ep_lxc=0,
                    out: Verdicts | None = None, want_action=True,
                    want_ct=False, want_notify=False, want_pkt=False,
                    stream=None) -> Verdicts:
        import torch
        n = len(batch)
        dev = batch.saddr.device
        if out is None:
            out = Verdicts(torch.empty(n, dtype=torch.int32, device=dev),
                           torch.empty(n, dtype=torch.int32, device=dev),
                           torch.empty(n, dtype=torch.uint8, device=dev)
                           if want_action else None,
                           torch.empty(n, dtype=torch.uint8, device=dev)
                           if want_ct else None,
                           torch.empty(n, dtype=torch.int32, device=dev)
                           if want_notify else None,
                           # column-major: each column one contiguous array
                           torch.empty((3, n), dtype=torch.int32, device=dev).t()
                           if want_pkt else None)
        if out.pkt is not None:
            assert out.pkt.shape == (n, 3) and out.pkt.stride() == (1, n)
        if batch.hash is not None:
            assert batch.hash.numel() == n and batch.hash.dtype == torch.int32
        for t in (batch.saddr, batch.daddr, batch.ports, batch.meta):
            assert t.is_cuda and t.is_contiguous() and t.numel() == n
            assert t.dtype == torch.int32
        if batch.mark is not None:
            assert batch.mark.numel() == n and batch.mark.dtype == torch.int32
        if batch.tcp_flags is not None:
            assert batch.tcp_flags.numel() == n and batch.tcp_flags.dtype == torch.uint8
        hdr = hdr_struct(batch)
        o = out_struct(out)
        L.check(self.L.cfc_classify_v4(self.h, ctypes.byref(hdr),
                                       ctypes.byref(o), mode, ep_lxc,
                                       self._stream(stream)),"classify")
        return out

    def classify_v6(self, batch: HeaderBatchV6, mode=L.MODE_INGRESS, ep_lxc=0,
                    out: Verdicts | None = None, want_action=True,
                    want_ct=False, want_notify=False, want_pkt=False,
                    stream=None) -> Verdicts:
        import torch
        n = len(batch)
        dev = batch.ports.device
        if out is None:
            out = Verdicts(torch.empty(n, dtype=torch.int32, device=dev),
                           torch.empty(n, dtype=torch.int32, device=dev),
                           torch.empty(n, dtype=torch.uint8, device=dev)
                           if want_action else None,
                           torch.empty(n, dtype=torch.uint8, device=dev)
                           if want_ct else None,
                           torch.empty(n, dtype=torch.int32, device=dev)
                           if want_notify else None)
        for t in (batch.saddr, batch.daddr):
            assert t.is_cuda and t.is_contiguous() and t.dtype == torch.int32
            assert t.shape == (n, 4) and t.data_ptr() % 16 == 0
        for t in (batch.ports, batch.meta):
            assert t.is_cuda and t.is_contiguous() and t.numel() == n
            assert t.dtype == torch.int32
        if batch.mark is not None:
            assert batch.mark.numel() == n and batch.mark.dtype == torch.int32
        if batch.tcp_flags is not None:
            assert batch.tcp_flags.numel() == n and batch.tcp_flags.dtype == torch.uint8
        if batch.hash is not None:
            assert batch.hash.numel() == n and batch.hash.dtype == torch.int32
        hdr = hdr_struct(batch)
        pk = None
        if want_pkt:   # saddr rows, daddr rows, L4 words: three arrays
            pk = torch.empty(9 * n, dtype=torch.int32, device=dev)
        o = L.Out(_ptr(out.verdict), _ptr(out.identity), _ptr(out.action),
                  _ptr(out.ct), _ptr(out.notify),
                  *((_ptr(pk[:4 * n]), _ptr(pk[4 * n:8 * n]), _ptr(pk[8 * n:]))
                    if pk is not None else (None, None, None)))
        L.check(self.L.cfc_classify_v6(self.h, ctypes.byref(hdr),
                                       ctypes.byref(o), mode, ep_lxc,
                                       self._stream(stream)), "classify v6")
        if pk is not None:
            out.pkt_raw = pk
            out.pkt = _pkt6(pk)
        return out

    def classify(self, batch, mode=L.MODE_INGRESS, ep_lxc=0, **kw) -> Verdicts:
        """classify_v4 or classify_v6 by the batch's family."""
        if isinstance(batch, HeaderBatchV6):
            return self.classify_v6(batch, mode, ep_lxc, **kw)
        return self.classify_v4(batch, mode, ep_lxc, **kw)

    def ct_apply(self, batch, out: Verdicts, mode=L.MODE_INGRESS, ep_lxc=0,
                 stream=None):
        """cfc_ct_apply_v4/v6: fold a classified batch (out.ct set) into the
        CT maps — creates, deletes of denied established flows, closing
        flags — in header order.  Synchronises the stream."""
        assert out.ct is not None, "classify with want_ct=True"
        v6 = isinstance(batch, HeaderBatchV6)
        hdr = hdr_struct(batch)
        o = out_struct(out)
        fn = self.L.cfc_ct_apply_v6 if v6 else self.L.cfc_ct_apply_v4
        L.check(fn(self.h, ctypes.byref(hdr), ctypes.byref(o), mode, ep_lxc,
                   self._stream(stream)), "ct apply")
        if v6 and out.pkt_raw is not None:   # (the packet outputs in packet order)
            out.pkt = _pkt6(out.pkt_raw)

    def drop_notify(self, batch, out: Verdicts, mode=L.MODE_INGRESS,
                    ep_lxc=0, cap=None, stream=None, sync=True):
        """cfc_drop_notify_v4/v6: the batch's struct drop_notify records in
        header order -> (records as an (m, 8) int32 tensor in the
        cfc_drop_notify layout, header indices int64, total drops).
        sync=True synchronises the device to read the total and trims the
        tensors to it; sync=False returns (records, indices, total as a
        1-element int64 device tensor) with nothing waited for."""
        return self._events(batch, out, mode, ep_lxc, cap, stream, sync, False)

    def monitor_events(self, batch, out: Verdicts, mode=L.MODE_INGRESS,
                       ep_lxc=0, cap=None, stream=None, sync=True):
        """cfc_monitor_events_v4/v6: every drop_notify and trace_notify
        record of the batch in header order (32 bytes each, the `type` byte
        tells them apart); returns as drop_notify does."""
        return self._events(batch, out, mode, ep_lxc, cap, stream, sync, True)

    def _events(self, batch, out, mode, ep_lxc, cap, stream, sync, traces):
        import torch
        assert out.notify is not None, "classify with want_notify=True"
        n = len(batch)
        cap = n if cap is None else cap
        dev = out.verdict.device
        rec = torch.zeros((max(cap, 1), 8), dtype=torch.int32, device=dev)
        idx = torch.zeros(max(cap, 1), dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        v6 = isinstance(batch, HeaderBatchV6)
        if traces:
            fn = self.L.cfc_monitor_events_v6 if v6 else self.L.cfc_monitor_events_v4
        else:
            fn = self.L.cfc_drop_notify_v6 if v6 else self.L.cfc_drop_notify_v4
        L.check(fn(self.h, ctypes.byref(hdr_struct(batch)), ctypes.byref(out_struct(out)),
                   mode, ep_lxc, _ptr(rec), _ptr(idx), cap, _ptr(cnt),
                   self._stream(stream)), "monitor events")
        if not sync:
            return rec, idx, cnt
        torch.cuda.synchronize(dev)
        total = int(cnt.item())
        m = min(total, cap)
        return rec[:m], idx[:m], total

    def set_clock(self, now):
        """cfc_set_clock: bpf_ktime_get_sec() for the next calls."""
        L.check(self.L.cfc_set_clock(self.h, int(now) & 0xFFFFFFFF), "clock")
        self.clock = int(now) & 0xFFFFFFFF

    clock = 0   # the datapath clock as last set (cfc_set_clock; the library starts at 0)

    def ct_gc(self, fd=-1, time=0, remove_expired=True, valid_ips=None,
              match_ips=None, stream=None):
        """cfc_ct_gc: ctmap.GC with doFiltering (pkg/maps/ctmap/ctmap.go:
        303-350) on CT map `fd` (-1: every CT map).  valid_ips / match_ips:
        iterables of IP address bytes (4 or 16), None = no such set.
        -> gcStats as a dict {deleted, alive, ...}."""
        def ips(lst):
            if lst is None:
                return None, 0
            lst = [bytes(a) for a in lst]
            arr = (L.Ip * max(len(lst), 1))()
            for i, a in enumerate(lst):
                arr[i].family = 4 if len(a) == 4 else 6
                arr[i].addr[:len(a)] = list(a)
            return arr, len(lst)
        va, nv = ips(valid_ips)
        ma, nm = ips(match_ips)
        f = L.GcFilter()
        f.flags = ((L.GC_REMOVE_EXPIRED if remove_expired else 0) |
                   (L.GC_VALID_IPS if va is not None else 0) |
                   (L.GC_MATCH_IPS if ma is not None else 0))
        f.time = int(time) & 0xFFFFFFFF
        f.valid_ips = ctypes.cast(va, ctypes.c_void_p) if va is not None else None
        f.n_valid = nv
        f.match_ips = ctypes.cast(ma, ctypes.c_void_p) if ma is not None else None
        f.n_match = nm
        st = L.GcStats()
        L.check(self.L.cfc_ct_gc(self.h, int(fd), ctypes.byref(f), ctypes.byref(st),
                                 self._stream(stream)), "ct gc")
        return {k: getattr(st, k) for k, _ in L.GcStats._fields_}

    def counters_sync(self, stream=None):
        L.check(self.L.cfc_counters_sync(self.h, self._stream(stream)),
                "counters sync")

    def counters_clear(self, stream=None):
        L.check(self.L.cfc_counters_clear(self.h, self._stream(stream)),
                "counters clear")

    def counters_export(self, t, stream=None):
        """Move the device counter block into int64 tensor `t` (zeroing it)."""
        L.check(self.L.cfc_counters_export(self.h, _ptr(t), t.numel(),
                                           self._stream(stream)), "export")

    def counters_import(self, t, stream=None):
        """Add int64 tensor `t` (e.g. an all-reduced block) into the counters."""
        L.check(self.L.cfc_counters_import(self.h, _ptr(t), t.numel(),
                                           self._stream(stream)), "import")

    def counters_device(self):
        """(device pointer, number of u64) of the live counter block."""
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        L.check(self.L.cfc_counters_device(self.h, ctypes.byref(p),
                                           ctypes.byref(n)), "counters device")
        return p.value, n.value

    def identity_counters(self):
        """cfc_identity_counters: the per-identity forward/drop totals folded
        by counters_sync -> numpy (n, 6) u64 rows {identity, dir (1 ingress,
        2 egress), fwd packets, fwd bytes, drop packets, drop bytes}."""
        import numpy as np
        n = ctypes.c_uint64()
        L.check(self.L.cfc_identity_counters(self.h, None, 0, ctypes.byref(n)),
                "identity counters")
        rows = (L.IdentityCount * max(n.value, 1))()
        L.check(self.L.cfc_identity_counters(self.h, rows, n.value, ctypes.byref(n)),
                "identity counters")
        return np.array([(r.identity, r.dir, r.fwd_packets, r.fwd_bytes,
                          r.drop_packets, r.drop_bytes) for r in rows[:n.value]],
                        np.uint64).reshape(-1, 6)

    def stats(self):
        st = L.Stats()
        L.check(self.L.cfc_get_stats(self.h, ctypes.byref(st)), "stats")
        return {f: getattr(st, f) for f, _ in L.Stats._fields_ if f != "pad0"}


def host_only():
    """A context with the map API only (no GPU): control-plane tooling."""
    return Datapath(L.CFC_DEVICE_NONE)


def errno_name(e: OSError):
    import errno
    return errno.errorcode.get(e.errno, str(e.errno))


__all__ = ["Datapath", "HeaderBatchV4", "HeaderBatchV6", "Verdicts", "pack_v4",
           "pack_v6", "pack", "host_only", "errno_name"]
