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
# one perf-ring record of either kind (32 bytes): w6 is drop_notify.dst_id,
# or trace_notify's {u16 dst_id, u8 reason, u8 pad}
EVENT_DT = np.dtype([("type", "u1"), ("subtype", "u1"), ("source", "<u2"),
                     ("hash", "<u4"), ("len_orig", "<u4"), ("len_cap", "<u4"),
                     ("src_label", "<u4"), ("dst_label", "<u4"), ("w6", "<u4"),
                     ("ifindex", "<u4")])
TRACE_TO_LXC, TRACE_TO_PROXY, TRACE_TO_HOST, TRACE_TO_STACK = 0, 1, 2, 3


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


def _tcp_flags(hdr):
    """TCP header byte 13 per header (synth.tcp_flags_of, restated so the
    oracle does not import the product package)"""
    if getattr(hdr, "tcpflags", None) is not None:
        return np.asarray(hdr.tcpflags, np.uint8)
    tcp = np.asarray(hdr.proto) == 6
    close = (np.asarray(hdr.flags) & 2) != 0
    return np.where(tcp, np.where(close, 0x11, 0x02), 0).astype(np.uint8)


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
                                      ctypes.c_size_t] + [vp] * 14 + [ctypes.c_int]
        L.cfo_classify_v6.argtypes = [vp, ctypes.c_int, ctypes.c_uint16,
                                      ctypes.c_size_t] + [vp] * 14 + [ctypes.c_int]
        L.cfo_ct_add.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 vp, vp]
        for f in (L.cfo_ct_apply_v4, L.cfo_ct_apply_v6):
            f.argtypes = [vp, ctypes.c_int, ctypes.c_uint16,
                          ctypes.c_size_t] + [vp] * 13
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
        L.cfo_set_notify_out.argtypes = [vp, vp, vp]
        L.cfo_node_config.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u8p,
                                      ctypes.c_uint32]
        L.cfo_node_config.restype = None
        L.cfo_set_clock.argtypes = [vp, ctypes.c_uint32]
        L.cfo_set_clock.restype = None
        L.cfo_lb4_service_add.argtypes = [vp, vp, vp]
        L.cfo_lb4_revnat_add.argtypes = [vp, ctypes.c_uint16, vp]
        L.cfo_lb6_service_add.argtypes = [vp, vp, vp]
        L.cfo_lb6_revnat_add.argtypes = [vp, ctypes.c_uint16, vp]
        L.cfo_set_lb_io.argtypes = [vp, vp, vp]
        L.cfo_set_lb_io.restype = None
        L.cfo_ipcache_lookup.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, vp, vp, vp]
        L.cfo_ipcache_lookup.restype = None
        L.cfo_ct_gc.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_uint32, vp, ctypes.c_size_t, vp, ctypes.c_size_t]
        L.cfo_ct_gc.restype = ctypes.c_size_t
        L.cfo_run_seq.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint16,
                                  ctypes.c_size_t] + [vp] * 15
        L.cfo_run_seq.restype = None
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
        self.host_ifindex = 1
        self.mon = None       # the last classify's per-header monitor lengths
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
        if getattr(t, "lb4", None) is not None:
            for r in np.asarray(t.lb4):
                b = r.tobytes()
                k, v = _u8p(np.frombuffer(b[:8], np.uint8)), _u8p(np.frombuffer(b[8:20], np.uint8))
                L.cfo_lb4_service_add(h, ctypes.cast(k[0], ctypes.c_void_p),
                                      ctypes.cast(v[0], ctypes.c_void_p))
        if getattr(t, "revnat4", None) is not None:
            for r in np.asarray(t.revnat4):
                v, keep = _u8p(np.frombuffer(r.tobytes()[2:8], np.uint8))
                L.cfo_lb4_revnat_add(h, int(r["index"]), ctypes.cast(v, ctypes.c_void_p))
        if getattr(t, "lb6", None) is not None:   # (LB6_DT: key 20 B, value 24 B)
            for r in np.asarray(t.lb6):
                b = r.tobytes()
                k, kk = _u8p(np.frombuffer(b[:20], np.uint8))
                v, vk = _u8p(np.frombuffer(b[20:44], np.uint8))
                L.cfo_lb6_service_add(h, ctypes.cast(k, ctypes.c_void_p),
                                      ctypes.cast(v, ctypes.c_void_p))
        if getattr(t, "revnat6", None) is not None:   # (REVNAT6_DT: index, 18 B)
            for r in np.asarray(t.revnat6):
                v, keep = _u8p(np.frombuffer(r.tobytes()[2:20], np.uint8))
                L.cfo_lb6_revnat_add(h, int(r["index"]), ctypes.cast(v, ctypes.c_void_p))

    def node_config(self, v4_cluster_range, v4_cluster_mask, router_ip6,
                    host_ifindex=1):
        """node_config.h IPV4_CLUSTER_RANGE / _MASK (raw be32 as loaded),
        ROUTER_IP (16 bytes) and HOST_IFINDEX."""
        p, keep = _u8p(np.asarray(router_ip6, np.uint8).reshape(16))
        self.host_ifindex = int(host_ifindex)
        self.L.cfo_node_config(self.h, int(v4_cluster_range) & 0xFFFFFFFF,
                               int(v4_cluster_mask) & 0xFFFFFFFF, p,
                               self.host_ifindex)

    def set_clock(self, now):
        """bpf_ktime_get_sec() of the next classify / ct_apply calls."""
        self.L.cfo_set_clock(self.h, int(now) & 0xFFFFFFFF)

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
                c(hdr.length, np.uint16), c(hdr.mark, np.uint32),
                c(_tcp_flags(hdr), np.uint8)]

    def _lb_io(self, hdr, pkt=None):
        hs = getattr(hdr, "hash", None)
        hs = None if hs is None else np.ascontiguousarray(hs, np.uint32)
        self._lb_keep = hs
        self.L.cfo_set_lb_io(self.h, _p(hs), _p(pkt))

    def classify(self, hdr, mode, ep_lxc=0, nthreads=1, want_lookups=False,
                 want_ct=False, apply_ct=False, want_notify=False, want_pkt=False,
                 seq=True):
        """-> (action, verdict, identity[, lookups][, ct][, notify][, pkt]).
        apply_ct folds the batch's CT creates/deletes into the oracle's CT
        maps — by default (seq) the reference's way, one header at a time
        (run_sequential: what the engine's classify + cfc_ct_apply give);
        seq=False: every header looked up against the maps as the batch found
        them, the writes folded afterwards (the batch model whose differences
        ct_apply(hazard=True) reports).  notify is the drop-notify site word
        per header (res_t.nt in cfc_oracle.c); pkt the packet's (saddr,
        daddr, sport | dport << 16) after the service translation and
        reverse NAT: (n, 3) u32 for IPv4, (n, 9) u32 for IPv6 (saddr and
        daddr as four raw words each)."""
        if apply_ct and seq:
            assert not want_lookups
            r = self.run_sequential(hdr, mode, ep_lxc, want_ct=True, want_pkt=want_pkt)
            act, ver, ide, words, ct = r[:5]
            out = (act, ver, ide)
            if want_ct:
                out += (ct,)
            if want_notify:
                out += (words,)
            if want_pkt:
                out += (r[5],)
            return out
        n = len(hdr)
        act = np.zeros(n, np.int32)
        ver = np.zeros(n, np.int32)
        ide = np.zeros(n, np.uint32)
        lk = np.zeros(n, np.uint8) if want_lookups else None
        ct = np.zeros(n, np.uint8) if (want_ct or apply_ct) else None
        c = np.ascontiguousarray
        at = np.uint32 if hdr.family == 4 else np.uint8
        arrs = self._arrays(hdr)
        if hdr.family == 6:
            assert arrs[0].shape == (n, 16) and arrs[1].shape == (n, 16)
        fn = self.L.cfo_classify_v4 if hdr.family == 4 else self.L.cfo_classify_v6
        nt = np.zeros(n, np.uint32) if want_notify else None
        self.mon = np.zeros(n, np.uint32)
        pkt = np.zeros((n, 3 if hdr.family == 4 else 9), np.uint32) if want_pkt else None
        self.L.cfo_set_notify_out(self.h, _p(nt), _p(self.mon))
        self._lb_io(hdr, pkt)
        fn(self.h, mode, ep_lxc, n, *[_p(a) for a in arrs], _p(act), _p(ver),
           _p(ide), _p(lk), _p(ct), nthreads)
        self.L.cfo_set_notify_out(self.h, None, None)
        self.L.cfo_set_lb_io(self.h, None, None)
        if apply_ct:
            self.ct_apply(hdr, mode, ep_lxc, ide, ver, ct)
        out = (act, ver, ide)
        if want_lookups:
            out += (lk,)
        if want_ct:
            out += (ct,)
        if want_notify:
            out += (nt,)
        if want_pkt:
            out += (pkt,)
        return out

    def events(self, hdr, mode, ep_lxc, verdict, identity, words, drops=True,
               traces=True):
        """The monitor events the reference's perf ring cilium_events would
        carry for this batch, in header order -> (EVENT_DT records, header
        indices u64): struct drop_notify (bpf/lib/drop.h:40-78) for drops,
        struct trace_notify (trace.h:71-81, send_trace_notify :97-155) for
        forwarded packets.  words = the classify's per-header event words
        (want_notify).  SECLABEL / ifindex come from the loaded tables."""
        t = self.tables
        sec = np.zeros(65536, np.uint32)
        for lxc, lab in t.seclabel.items():
            sec[int(lxc)] = int(lab)
        ifx = np.zeros(65536, np.uint32)
        ifx[t.endpoints["lxc_id"].astype(np.int64)] = t.endpoints["ifindex"]
        words = np.asarray(words, np.uint32)
        kind = (words >> 16) & 0xF
        # (a trace of monitor length 0 — class 0 — is not sent)
        sel = ((kind >= 1) & (kind <= 3) & drops) | \
            ((kind >= 4) & (((words >> 22) & 3) != 0) & traces)
        idx = np.flatnonzero(sel).astype(np.uint64)
        w = words[idx]
        k, lxc = (w >> 16) & 0xF, (w & 0xFFFF).astype(np.int64)
        ver = np.asarray(verdict)[idx].astype(np.int64)
        ident = np.asarray(identity)[idx].astype(np.uint32)
        ln = np.asarray(hdr.length, np.uint32)[idx]
        # an event after a NAT hop (cfc.h CFC_NT_NATLEN): the translated
        # packet's skb->len, the IPv4 header being 20 bytes shorter
        nat = (w >> 24) & 1 != 0
        ln = np.where(nat, ln.astype(np.int64) + (20 if hdr.family == 4 else -20),
                      ln).astype(np.uint32)
        own = sec[ep_lxc] if mode == MODE_EGRESS else 0
        r = np.zeros(len(idx), EVENT_DT)
        hs = getattr(hdr, "hash", None)
        r["hash"] = flow_hash(hdr, idx) if hs is None else np.asarray(hs, np.uint32)[idx]
        r["len_orig"] = ln
        # drops: cb[1] = src << 16 | dst & 0xFFFF, both labels 16 bits
        d = k <= 3
        r["type"] = np.where(d, 1, 4)                     # CILIUM_NOTIFY_DROP / TRACE
        r["subtype"] = np.where(d, (-ver) & 0xFF, k - 4)  # -reason / obs point
        r["source"] = np.where(k == 1, 0, lxc)            # EVENT_SOURCE
        mc = (w >> 22) & 3                                # TRACE_PAYLOAD_LEN / MTU / 1
        mon = np.where(mc == 2, 1500, np.where(mc == 3, 1, 128))
        r["len_cap"] = np.minimum(ln, np.where(d, 128, mon))
        i64 = lambda x: np.broadcast_to(np.asarray(x, np.int64), k.shape)  # noqa: E731
        ownv = i64(own)
        peer = ownv if mode == MODE_EGRESS else i64(ident)
        src = np.select([k == 2, k == 3, k == 4, k >= 5],
                        [ownv, peer, peer, i64(sec[lxc])], 0)
        dst = np.select([k == 2, k == 3, k == 4, k == 6, k == 7],
                        [i64(ident), i64(sec[lxc]), i64(sec[lxc]), i64(1), i64(ident)], 0)
        r["src_label"] = np.where(d, np.asarray(src, np.uint32) & 0xFFFF, src)
        r["dst_label"] = np.where(d, np.asarray(dst, np.uint32) & 0xFFFF, dst)
        # drop_notify.dst_id (u32) / trace_notify {dst_id u16, reason u8, pad}
        reason = (w >> 20) & 3
        reason = reason.astype(np.int64)
        r["w6"] = np.select([k == 3, k == 4, k >= 5],
                            [lxc, lxc | reason << 16, reason << 16], 0)
        r["ifindex"] = np.select([k == 3, k == 4, (k == 5) | (k == 6)],
                                 [i64(ifx[lxc]), i64(ifx[lxc]), i64(self.host_ifindex)], 0)
        return r, idx

    def run_sequential(self, hdr, mode, ep_lxc, clock=None, want_ct=False, want_pkt=False):
        """The reference's own semantics: one header at a time, each folded
        into the CT maps before the next (cfo_run_seq), at the
        bpf_ktime_get_sec() value clock[i] (None: the clock as set; a scalar:
        that clock for every header) -> (action, verdict, identity, event
        words[, ct][, pkt])."""
        n = len(hdr)
        act = np.zeros(n, np.int32)
        ver = np.zeros(n, np.int32)
        ide = np.zeros(n, np.uint32)
        words = np.zeros(n, np.uint32)
        ct = np.zeros(n, np.uint8)
        pkt = np.zeros((n, 3 if hdr.family == 4 else 9), np.uint32) if want_pkt else None
        clk = None
        if clock is not None:
            clk = np.ascontiguousarray(np.broadcast_to(np.asarray(clock, np.int64), (n,))
                                       .astype(np.uint32))
        arrs = self._arrays(hdr)
        self._lb_io(hdr, pkt)
        self.L.cfo_run_seq(self.h, hdr.family, mode, ep_lxc, n,
                           *[_p(a) for a in arrs], _p(clk), _p(act), _p(ver), _p(ide),
                           _p(ct), _p(words))
        self.L.cfo_set_lb_io(self.h, None, None)
        out = (act, ver, ide, words)
        if want_ct:
            out += (ct,)
        if want_pkt:
            out += (pkt,)
        return out

    def drop_notify(self, hdr, mode, ep_lxc, verdict, identity, sites):
        """The struct drop_notify records (bpf/lib/drop.h:40-78) of this
        batch in header order -> (records DROP_NOTIFY_DT, header indices)."""
        r, idx = self.events(hdr, mode, ep_lxc, verdict, identity, sites,
                             traces=False)
        return r.view(DROP_NOTIFY_DT), idx

    def ct_apply(self, hdr, mode, ep_lxc, identity, verdict, ct, hazard=False,
                 trace_hazards=False):
        """Fold a classified batch into the CT maps (cfo_ct_apply_*).  With
        hazard, returns per header 1 where a packet-at-a-time run would see a
        different CT result — and, with trace_hazards, a different monitor
        length (from the last classify) — because of an earlier header."""
        arrs = self._arrays(hdr)
        hz = np.zeros(len(hdr), np.uint8) if hazard else None
        fn = self.L.cfo_ct_apply_v4 if hdr.family == 4 else self.L.cfo_ct_apply_v6
        c = np.ascontiguousarray
        mon = c(self.mon, np.uint32) if trace_hazards else None
        self._lb_io(hdr)
        fn(self.h, mode, ep_lxc, len(hdr), *[_p(a) for a in arrs[:7]],
           _p(arrs[8]), _p(c(identity, np.uint32)), _p(c(verdict, np.int32)),
           _p(c(ct, np.uint8)), _p(mon), _p(hz))
        self.L.cfo_set_lb_io(self.h, None, None)
        return hz

    def ipcache_lookup(self, family, addrs):
        """ipcache_lookup4/6 (eps.h:56-80) of each address -> (label u32,
        hit u8); family 4: u32 addresses as loaded, 6: (n, 16) bytes."""
        a = np.ascontiguousarray(addrs, np.uint32 if family == 4 else np.uint8)
        n = len(a)
        lab = np.zeros(n, np.uint32)
        hit = np.zeros(n, np.uint8)
        self.L.cfo_ipcache_lookup(self.h, 1 if family == 4 else 2, n, _p(a), _p(lab), _p(hit))
        return lab, hit

    def ct_gc(self, time=None, remove_expired=True, valid=None, match=None,
              family=0, owner=-1, kind=-1):
        """ctmap.GC + doFiltering (pkg/maps/ctmap/ctmap.go:303-350) -> entries
        deleted.  valid / match: lists of (family 4|6, address bytes), None:
        no such set (an empty list is an empty set)."""
        def ips(lst):
            if lst is None:
                return None, ctypes.c_size_t(-1).value
            a = np.zeros((max(len(lst), 1), 17), np.uint8)
            for i, (f, b) in enumerate(lst):
                a[i, 0] = 1 if f == 4 else 2
                a[i, 1:1 + len(b)] = np.frombuffer(bytes(b), np.uint8)
            return a, len(lst)
        va, nv = ips(valid)
        ma, nm = ips(match)
        self._gc_keep = (va, ma)
        return int(self.L.cfo_ct_gc(self.h, family, owner, kind, int(bool(remove_expired)),
                                    int(time or 0) & 0xFFFFFFFF, _p(va), nv, _p(ma), nm))

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
