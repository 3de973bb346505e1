"""ctypes front-end of the C restatement (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker — never by cilium_amd/.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

MODE_INGRESS, MODE_EGRESS, MODE_XDP, MODE_FULL = 0, 1, 2, 3
CT_ROW = 104     # cfc_oracle.h CFO_CT_ROW

_lib = None

# cfc_drop_notify (include/cfc.h) = struct drop_notify (bpf/lib/drop.h:40-48)
DROP_NOTIFY_DT = np.dtype([("type", "u1"), ("subtype", "u1"), ("source", "<u2"),
                           ("hash", "<u4"), ("len_orig", "<u4"),
                           ("len_cap", "<u4"), ("src_label", "<u4"),
                           ("dst_label", "<u4"), ("dst_id", "<u4"),
                           ("ifindex", "<u4")])
assert DROP_NOTIFY_DT.itemsize == 32


def _fmix32(h):
    h = h.astype(np.uint32)
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x85EBCA6B)
    h ^= h >> np.uint32(13)
    h *= np.uint32(0xC2B2AE35)
    h ^= h >> np.uint32(16)
    return h


def flow_hash(hdr, idx):
    """The engine's drop_notify.hash (cfc.h CFC_FLOW_HASH): a symmetric
    5-tuple hash.  The reference's get_hash_recalc() value is the kernel's
    flow-dissector hash under a boot-random key, which nothing can reproduce."""
    with np.errstate(over="ignore"):
        if hdr.family == 4:
            a = np.asarray(hdr.saddr, np.uint32)[idx]
            b = np.asarray(hdr.daddr, np.uint32)[idx]
        else:
            def fold(x):
                w = np.ascontiguousarray(np.asarray(x, np.uint8)[idx]).view("<u4")
                h = _fmix32(w[:, 3])
                for k in (2, 1, 0):
                    h = _fmix32(w[:, k] ^ h)
                return h
            a, b = fold(hdr.saddr), fold(hdr.daddr)
        lo, hi = np.minimum(a, b), np.maximum(a, b)
        sp = np.asarray(hdr.sport, np.uint32)[idx]
        dp = np.asarray(hdr.dport, np.uint32)[idx]
        pw = np.minimum(sp, dp) | (np.maximum(sp, dp) << np.uint32(16))
        pr = np.asarray(hdr.proto, np.uint32)[idx]
        return _fmix32(lo * np.uint32(0x9E3779B1) + hi * np.uint32(0x85EBCA77)
                       + pw * np.uint32(0xC2B2AE3D) + pr)


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, u8p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8)
        L.cfo_new.restype = vp
        L.cfo_free.argtypes = [vp]
        L.cfo_ipcache_add.argtypes = [vp, ctypes.c_int, ctypes.c_int, u8p,
                                      ctypes.c_uint32]
        L.cfo_endpoint_add.argtypes = [vp, ctypes.c_int, u8p, ctypes.c_uint32,
                                       ctypes.c_uint16, ctypes.c_uint32]
        L.cfo_seclabel_set.argtypes = [vp, ctypes.c_uint16, ctypes.c_uint32]
        L.cfo_policy_add.argtypes = [vp, ctypes.c_uint16, ctypes.c_uint32,
                                     ctypes.c_uint16, ctypes.c_uint8,
                                     ctypes.c_uint8, ctypes.c_uint16]
        L.cfo_prefilter_add.argtypes = [vp, ctypes.c_int, ctypes.c_int, u8p,
                                        ctypes.c_int]
        L.cfo_classify_v4.argtypes = [vp, ctypes.c_int, ctypes.c_uint16,
                                      ctypes.c_size_t] + [vp] * 13 + [ctypes.c_int]
        L.cfo_classify_v6.argtypes = [vp, ctypes.c_int, ctypes.c_uint16,
                                      ctypes.c_size_t] + [vp] * 13 + [ctypes.c_int]
        L.cfo_ct_add.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 vp, vp]
        for f in (L.cfo_ct_apply_v4, L.cfo_ct_apply_v6):
            f.argtypes = [vp, ctypes.c_int, ctypes.c_uint16,
                          ctypes.c_size_t] + [vp] * 11
        L.cfo_ct_add_n.argtypes = [vp, ctypes.c_size_t, vp]
        L.cfo_ct_dump.restype = ctypes.c_size_t
        L.cfo_ct_dump.argtypes = [vp, vp, ctypes.c_size_t]
        L.cfo_policy_create.argtypes = [vp, ctypes.c_uint16]
        L.cfo_policy_dump.restype = ctypes.c_size_t
        L.cfo_policy_dump.argtypes = [vp, ctypes.c_uint16, vp, ctypes.c_size_t]
        L.cfo_metrics_dump.restype = ctypes.c_size_t
        L.cfo_metrics_dump.argtypes = [vp, vp, ctypes.c_size_t]
        L.cfo_counters_reset.argtypes = [vp]
        L.cfo_identity_dump.restype = ctypes.c_size_t
        L.cfo_identity_dump.argtypes = [vp, vp, ctypes.c_size_t]
        L.cfo_set_notify_out.argtypes = [vp, vp]
        L.cfo_node_config.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u8p]
        L.cfo_node_config.restype = None
        _lib = L
    return _lib


def _u8p(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), a


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Oracle:
    def __init__(self, tables=None):
        self.L = lib()
        self.h = self.L.cfo_new()
        self.lxc_ids = []
        self.tables = tables
        if tables is not None:
            self.load(tables)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.cfo_free(self.h)
            self.h = None

    def load(self, t):
        L, h = self.L, self.h
        for e in t.ipcache:
            p, keep = _u8p(e["addr"])
            L.cfo_ipcache_add(h, int(e["family"]), int(e["plen"]), p,
                              int(e["label"]))
        for e in t.endpoints:
            p, keep = _u8p(e["addr"])
            L.cfo_endpoint_add(h, int(e["family"]), p, int(e["ifindex"]),
                               int(e["lxc_id"]), int(e["flags"]))
        for lxc, lab in t.seclabel.items():
            L.cfo_seclabel_set(h, int(lxc), int(lab))
        for lxc, pol in t.policy.items():
            self.lxc_ids.append(int(lxc))
            L.cfo_policy_create(h, int(lxc))
            for r in pol:
                L.cfo_policy_add(h, int(lxc), int(r["identity"]), int(r["dport"]),
                                 int(r["proto"]), int(r["egress"]),
                                 int(r["proxy_port"]))
        for p in t.prefilter:
            a, keep = _u8p(p["addr"])
            L.cfo_prefilter_add(h, int(p["family"]), int(p["plen"]), a,
                                int(p["dyn"]))
        if getattr(t, "ct", None) is not None:
            self.ct_add(t.ct)
        if getattr(t, "node", None) is not None:
            self.node_config(*t.node)

    def node_config(self, v4_cluster_range, v4_cluster_mask, router_ip6):
        """node_config.h IPV4_CLUSTER_RANGE / _MASK (raw be32 as loaded) and
        ROUTER_IP (16 bytes)."""
        p, keep = _u8p(np.asarray(router_ip6, np.uint8).reshape(16))
        self.L.cfo_node_config(self.h, int(v4_cluster_range) & 0xFFFFFFFF,
                               int(v4_cluster_mask) & 0xFFFFFFFF, p)

    def ct_add(self, ct):
        rec = np.ascontiguousarray(ct)
        assert rec.dtype.itemsize == 100, rec.dtype
        self.L.cfo_ct_add_n(self.h, len(rec), _p(rec))

    def _arrays(self, hdr):
        c = np.ascontiguousarray
        at = np.uint32 if hdr.family == 4 else np.uint8
        return [c(hdr.saddr, at), c(hdr.daddr, at),
                c(hdr.sport, np.uint16), c(hdr.dport, np.uint16),
                c(hdr.proto, np.uint8), c(hdr.flags, np.uint8),
                c(hdr.length, np.uint16), c(hdr.mark, np.uint32)]

    def classify(self, hdr, mode, ep_lxc=0, nthreads=1, want_lookups=False,
                 want_ct=False, apply_ct=False, want_notify=False):
        """-> (action, verdict, identity[, lookups][, ct][, notify]).
        apply_ct folds the batch's CT creates/deletes into the oracle's CT
        maps afterwards (what the engine's cfc_ct_apply does); notify is the
        drop-notify site word per header (res_t.nt in cfc_oracle.c)."""
        n = len(hdr)
        act = np.zeros(n, np.int32)
        ver = np.zeros(n, np.int32)
        ide = np.zeros(n, np.uint32)
        lk = np.zeros(n, np.uint8) if want_lookups else None
        ct = np.zeros(n, np.uint8) if (want_ct or apply_ct) else None
        c = np.ascontiguousarray
        at = np.uint32 if hdr.family == 4 else np.uint8
        arrs = [c(hdr.saddr, at), c(hdr.daddr, at),
                c(hdr.sport, np.uint16), c(hdr.dport, np.uint16),
                c(hdr.proto, np.uint8), c(hdr.flags, np.uint8),
                c(hdr.length, np.uint16), c(hdr.mark, np.uint32)]
        if hdr.family == 6:
            assert arrs[0].shape == (n, 16) and arrs[1].shape == (n, 16)
        fn = self.L.cfo_classify_v4 if hdr.family == 4 else self.L.cfo_classify_v6
        nt = np.zeros(n, np.uint32) if want_notify else None
        self.L.cfo_set_notify_out(self.h, _p(nt))
        fn(self.h, mode, ep_lxc, n, *[_p(a) for a in arrs], _p(act), _p(ver),
           _p(ide), _p(lk), _p(ct), nthreads)
        self.L.cfo_set_notify_out(self.h, None)
        if apply_ct:
            self.ct_apply(hdr, mode, ep_lxc, ide, ver, ct)
        out = (act, ver, ide)
        if want_lookups:
            out += (lk,)
        if want_ct:
            out += (ct,)
        if want_notify:
            out += (nt,)
        return out

    def drop_notify(self, hdr, mode, ep_lxc, verdict, identity, sites):
        """The struct drop_notify records (bpf/lib/drop.h:40-78) the
        reference's perf ring would carry for this batch, in header order
        -> (records DROP_NOTIFY_DT, header indices u64).  Uses the tables
        this oracle was loaded with for SECLABEL and ifindex."""
        t = self.tables
        sec = np.zeros(65536, np.uint32)
        for lxc, lab in t.seclabel.items():
            sec[int(lxc)] = int(lab)
        ifx = np.zeros(65536, np.uint32)
        ifx[t.endpoints["lxc_id"].astype(np.int64)] = t.endpoints["ifindex"]
        idx = np.flatnonzero(sites).astype(np.uint64)
        w = sites[idx].astype(np.uint32)
        site, src_lxc = w >> 16, (w & 0xFFFF).astype(np.int64)
        ver = verdict[idx].astype(np.int64)
        ident = identity[idx].astype(np.uint32)
        ln = np.asarray(hdr.length, np.uint32)[idx]
        r = np.zeros(len(idx), DROP_NOTIFY_DT)
        r["type"] = 1                                   # CILIUM_NOTIFY_DROP
        r["subtype"] = (-ver) & 0xFF                    # error = -reason
        r["source"] = np.where(site == 1, 0, src_lxc)   # EVENT_SOURCE
        r["hash"] = flow_hash(hdr, idx)
        r["len_orig"] = ln
        r["len_cap"] = np.minimum(ln, 128)              # TRACE_PAYLOAD_LEN
        # cb[1] = src << 16 | dst & 0xFFFF: both labels keep 16 bits
        own = sec[ep_lxc] if mode == MODE_EGRESS else 0
        src = np.where(site == 2, own,
                       np.where(site == 3, own if mode == MODE_EGRESS else ident, 0))
        dst = np.where(site == 2, ident,
                       np.where(site == 3, sec[src_lxc], 0))
        r["src_label"] = np.asarray(src, np.uint32) & 0xFFFF
        r["dst_label"] = np.asarray(dst, np.uint32) & 0xFFFF
        r["dst_id"] = np.where(site == 3, src_lxc, 0)
        r["ifindex"] = np.where(site == 3, ifx[src_lxc], 0)
        return r, idx

    def ct_apply(self, hdr, mode, ep_lxc, identity, verdict, ct, hazard=False):
        arrs = self._arrays(hdr)
        hz = np.zeros(len(hdr), np.uint8) if hazard else None
        fn = self.L.cfo_ct_apply_v4 if hdr.family == 4 else self.L.cfo_ct_apply_v6
        c = np.ascontiguousarray
        fn(self.h, mode, ep_lxc, len(hdr), *[_p(a) for a in arrs[:7]],
           _p(c(identity, np.uint32)), _p(c(verdict, np.int32)),
           _p(c(ct, np.uint8)), _p(hz))
        return hz

    def ct_dump(self):
        """(n, CT_ROW) u8 rows: owner u16, map u8, family u8, tuple[40],
        ct_entry[56], pad[4]; sorted."""
        n = self.L.cfo_ct_dump(self.h, None, 0)
        rows = np.zeros((n, CT_ROW), np.uint8)
        self.L.cfo_ct_dump(self.h, _p(rows), n)
        return rows

    def policy_counters(self, lxc):
        n = self.L.cfo_policy_dump(self.h, lxc, None, 0)
        rows = np.zeros((n, 7), np.uint64)
        self.L.cfo_policy_dump(self.h, lxc, _p(rows), n)
        return rows

    def metrics(self):
        n = self.L.cfo_metrics_dump(self.h, None, 0)
        rows = np.zeros((n, 4), np.uint64)
        self.L.cfo_metrics_dump(self.h, _p(rows), n)
        return rows

    def identity_counters(self):
        """(n, 6) u64 rows {identity, dir, fwd packets, fwd bytes, drop
        packets, drop bytes} (cfc.h cfc_identity_counters), sorted."""
        n = self.L.cfo_identity_dump(self.h, None, 0)
        rows = np.zeros((n, 6), np.uint64)
        self.L.cfo_identity_dump(self.h, _p(rows), n)
        return rows

    def reset_counters(self):
        self.L.cfo_counters_reset(self.h)
