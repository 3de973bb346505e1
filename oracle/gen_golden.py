"""Generate golden vectors by running the reference BPF datapath.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (root, kernel with
BPF_PROG_TEST_RUN); writes small fixtures to tests/golden/*.npz which the
CPU oracle and the GPU parity tests are checked against.

Reference programs driven (compiled by oracle/Makefile from the reference):
  ingress : bpf_netdev.o "from-netdev" (FROM_HOST, netdev_config.h)
            -> tail 2/7 handle_ipv4 (bpf_netdev.c:357-453: ipcache src
            identity, cilium_lxc lookup) -> ipv4_local_delivery (l3.h:103)
            -> cilium_policy[lxc_id] = bpf_lxc.o "1/0x1010" handle_policy
            (bpf_lxc.c:1039) -> tail 2/11 ipv4_policy (bpf_lxc.c:898-1015)
            -> __policy_can_access (policy.h:46-110)
  egress  : bpf_lxc.o "from-container" (bpf_lxc.c:718) -> tail 2/7
            handle_ipv4_from_lxc (bpf_lxc.c:440-692)
  xdp     : bpf_xdp.o "from-netdev" (bpf_xdp.c:158-184)
  full    : xdp, then ingress for XDP_PASS packets.

Per header we record the program's return code, skb->cb[] and the rewritten
L4 destination port; after the stream, every policymap's packets/bytes and
the cilium_metrics map (summed over CPUs).  From those the expected
(action, verdict, identity) triple is derived (see `_derive_*`).

Usage: python3 oracle/gen_golden.py [scenario ...]
"""
import os
import struct
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from cilium_amd import synth as S  # noqa: E402
import bpf_harness as H            # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")

LXC_MAC = bytes([0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff])    # lxc_config.h
NODE_MAC = bytes([0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde])   # lxc/node_config.h
HOST_IFINDEX = 1                                         # node_config.h
TC_ACT_OK, TC_ACT_SHOT, TC_ACT_REDIRECT = 0, 2, 7
XDP_DROP, XDP_PASS = 1, 2

MODE_INGRESS, MODE_EGRESS, MODE_XDP, MODE_FULL = 0, 1, 2, 3
MODES = {"ingress": MODE_INGRESS, "egress": MODE_EGRESS, "xdp": MODE_XDP,
         "full": MODE_FULL}


# ------------------------------------------------------------ packets
def build_packet_v4(h, i, eth_src=b"\x02" * 6, eth_dst=b"\x04" * 6):
    proto = int(h.proto[i])
    L = int(h.length[i])
    frag = 0x2000 if (h.flags[i] & S.HF_FRAG) else 0      # MF, offset 0
    ip = struct.pack(">BBHHHBBH", 0x45, 0, L - 14, i & 0xFFFF, frag, 64,
                     proto, 0)
    ip += struct.pack("<II", int(h.saddr[i]), int(h.daddr[i]))
    sp, dp = int(h.sport[i]), int(h.dport[i])
    if proto == S.IPPROTO_TCP:
        # HF_TCP_CLOSE: what ct_lookup reads as "rst || fin".  union
        # tcp_flags (conntrack.h:86-99) declares its bitfields as separate
        # union members, so each of them is bit 0 of TCP header byte 12;
        # FIN|ACK in byte 13 is set too, as a real close would carry.
        close = bool(h.flags[i] & S.HF_TCP_CLOSE)
        fl = int(S.tcp_flags_of(h.slice(i, i + 1))[0])
        l4 = struct.pack("<HH", sp, dp) + struct.pack(
            ">IIBBHHH", 1, 0, 0x51 if close else 0x50, fl, 1024, 0, 0)
    elif proto == S.IPPROTO_UDP:
        l4 = struct.pack("<HH", sp, dp) + struct.pack(">HH", L - 34, 0)
    else:   # ICMP (type/code in sport word, csum in dport word) and others
        l4 = struct.pack("<HH", sp, dp) + b"\x00" * 4
    pkt = eth_dst + eth_src + b"\x08\x00" + ip + l4
    assert len(pkt) <= L, (len(pkt), L)
    return pkt + bytes(L - len(pkt))


def build_packet_v6(h, i, eth_src=b"\x02" * 6, eth_dst=b"\x04" * 6):
    """Ethernet + IPv6 (+ one 8-byte destination-options header when
    HF_EXTHDR) + L4; `proto` is the next header after the extension headers
    (44 / 59 produce the fragment / no-next-header drops)."""
    proto = int(h.proto[i])
    L = int(h.length[i])
    ext = bool(h.flags[i] & S.HF_EXTHDR)
    sp, dp = int(h.sport[i]), int(h.dport[i])
    if proto == S.IPPROTO_TCP:
        # HF_TCP_CLOSE: what ct_lookup reads as "rst || fin".  union
        # tcp_flags (conntrack.h:86-99) declares its bitfields as separate
        # union members, so each of them is bit 0 of TCP header byte 12;
        # FIN|ACK in byte 13 is set too, as a real close would carry.
        close = bool(h.flags[i] & S.HF_TCP_CLOSE)
        fl = int(S.tcp_flags_of(h.slice(i, i + 1))[0])
        l4 = struct.pack("<HH", sp, dp) + struct.pack(
            ">IIBBHHH", 1, 0, 0x51 if close else 0x50, fl, 1024, 0, 0)
    elif proto == S.IPPROTO_UDP:
        l4 = struct.pack("<HH", sp, dp) + struct.pack(">HH", 8, 0)
    elif proto == 59:
        l4 = b""
    else:   # ICMPv6 (type/code in the sport word, csum in dport), others
        l4 = struct.pack("<HH", sp, dp) + b"\x00" * 4
    eh = bytes([proto, 0, 1, 4, 0, 0, 0, 0]) if ext else b""   # PadN option
    payload = eh + l4
    first = 60 if ext else proto
    ip = struct.pack(">IHBB", 0x60000000, L - 54, first, 64)
    ip += bytes(h.saddr[i]) + bytes(h.daddr[i])
    pkt = eth_dst + eth_src + b"\x86\xdd" + ip + payload
    assert len(pkt) <= L, (len(pkt), L)
    return pkt + bytes(L - len(pkt))


def l4_offset(h, i):
    if h.family == 4:
        return 14 + 20
    return 14 + 40 + (8 if h.flags[i] & S.HF_EXTHDR else 0)


# ------------------------------------------------------------ datapath
CT_MAPS = ("cilium_ct_tcp4_111", "cilium_ct_any4_111", "cilium_ct_tcp6_111",
           "cilium_ct_any6_111")


def u32(x):
    return struct.pack("<I", x)


def ipcache_key(e):
    # struct ipcache_key: lpm prefixlen = 32 static bits + plen (eps.h:49-52)
    return struct.pack("<IHBB", 32 + int(e["plen"]), 0, 0,
                       int(e["family"])) + bytes(e["addr"])


def endpoint_key(e):
    return bytes(e["addr"]) + struct.pack("<BBH", int(e["family"]), 0, 0)


def endpoint_value(e):
    # struct endpoint_info (common.h:165-173), 48 bytes
    return struct.pack("<IHHI4xQQ16x", int(e["ifindex"]), 0, int(e["lxc_id"]),
                       int(e["flags"]), 0, 0)


def policy_key(r):
    return struct.pack("<IHBB", int(r["identity"]), int(r["dport"]),
                       int(r["proto"]), int(r["egress"]))


class RefDatapath:
    def __init__(self, t: S.Tables):
        n_ipc = max(512000, len(t.ipcache) + 16)
        n_pf = max(1024, len(t.prefilter) + 16)
        ct_max = {m: 65536 for m in CT_MAPS}      # LRU: never near full
        self.L = L = H.Loader({"cilium_ipcache": n_ipc, "v4_fix": n_pf,
                               "v4_dyn": n_pf, "v6_fix": n_pf, "v6_dyn": n_pf,
                               "cilium_policy_foo": 16384 * 2, **ct_max})
        self.t = t
        SC = H.PROG_SCHED_CLS
        nd = {"cilium_calls_111": "calls_nd"}
        self.netdev = L.load("bpf_netdev.o", "from-netdev", SC, nd)
        nd_v4 = L.load("bpf_netdev.o", "2/7", SC, nd)
        L.maps["calls_nd"].update(u32(7), u32(nd_v4))
        # __send_drop_notify (drop.h:50, tail call CILIUM_CALL_DROP_NOTIFY 1)
        L.maps["calls_nd"].update(u32(1), u32(L.load("bpf_netdev.o", "2/1", SC, nd)))
        self.ep_prog = {}
        self.policy_map = {}
        self.ct_maps = {}     # lxc -> {ct map name in the object: renamed}
        for k, e in enumerate(t.endpoints):
            lxc = int(e["lxc_id"])
            if int(e["flags"]) & 1 or lxc not in t.policy or lxc in self.ep_prog:
                continue   # host entry, an endpoint without a program, or
                           # the second address of a dual-stack endpoint
            rn = {"cilium_calls_111": f"calls_lxc{k}",
                  "cilium_policy_foo": f"policy{k}"}
            for ct in CT_MAPS:
                rn[ct] = f"{ct}_{k}"
            self.ct_maps[lxc] = {ct: f"{ct}_{k}" for ct in CT_MAPS}
            pol = L.load("bpf_lxc.o", "1/0x1010", SC, rn)
            calls = {}
            # (2/8 tail_ipv6_to_ipv4 and 2/9 tail_ipv4_to_ipv6: LXC_NAT46 is on
            # in the reference's config, lxc_config.h:28 + nat46.h:30-32)
            for sec, idx in (("2/11", 11), ("2/7", 7), ("2/12", 12), ("2/10", 10),
                             ("2/8", 8), ("2/9", 9)):
                calls[idx] = L.load("bpf_lxc.o", sec, SC, rn)
            egress = L.load("bpf_lxc.o", "from-container", SC, rn)
            calls[1] = L.load("bpf_lxc.o", "2/1", SC, rn)   # __send_drop_notify
            for idx, fd in calls.items():
                L.maps[f"calls_lxc{k}"].update(u32(idx), u32(fd))
            L.maps["cilium_policy"].update(u32(lxc), u32(pol))
            self.ep_prog[lxc] = egress
            pm = L.maps[f"policy{k}"]
            self.policy_map[lxc] = pm
            for r in t.policy.get(lxc, []):
                pm.update(policy_key(r), struct.pack("<H6xQQ",
                                                     int(r["proxy_port"]), 0, 0))
        self.xdp = L.load("bpf_xdp.o", "from-netdev", H.PROG_XDP)
        # the perf ring cilium_events on the CPU this process is pinned to:
        # every trace_notify / drop_notify sample of a test run lands there
        self.cpu = H.pin_cpu()
        self.ring = H.PerfRing(self.cpu)
        L.maps["cilium_events"].update(u32(self.cpu), u32(self.ring.fd))
        for e in t.ipcache:
            L.maps["cilium_ipcache"].update(
                ipcache_key(e), struct.pack("<II", int(e["label"]),
                                            int(e["tunnel"])))
        for e in t.endpoints:
            L.maps["cilium_lxc"].update(endpoint_key(e), endpoint_value(e))
        # service load balancing (bpf/lib/lb.h:62-76): cilium_lb4_services
        # {struct lb4_key: struct lb4_service}, cilium_lb4_reverse_nat
        if getattr(t, "lb4", None) is not None:
            for r in t.lb4:
                b = r.tobytes()
                L.maps["cilium_lb4_services"].update(b[:8], b[8:20])
        if getattr(t, "revnat4", None) is not None:
            for r in t.revnat4:
                L.maps["cilium_lb4_reverse_nat"].update(
                    struct.pack("<H", int(r["index"])), r.tobytes()[2:8])
        # IPv6 (lb.h:38-53): cilium_lb6_services {struct lb6_key (20 B):
        # struct lb6_service (24 B)}, cilium_lb6_reverse_nat (18 B)
        if getattr(t, "lb6", None) is not None:
            for r in t.lb6:
                b = r.tobytes()
                L.maps["cilium_lb6_services"].update(b[:20], b[20:44])
        if getattr(t, "revnat6", None) is not None:
            for r in t.revnat6:
                L.maps["cilium_lb6_reverse_nat"].update(
                    struct.pack("<H", int(r["index"])), r.tobytes()[2:20])
        for p in t.prefilter:
            fam = int(p["family"])
            an = 4 if fam == 1 else 16
            name = ("v4_" if fam == 1 else "v6_") + ("dyn" if p["dyn"] else "fix")
            key = struct.pack("<I", int(p["plen"])) + bytes(p["addr"][:an])
            L.maps[name].update(key, b"\x01")

    def close(self):
        self.ring.close()
        self.L.close()

    def take_proxy_identity(self, family):
        """The identity ipv{4,6}_redirect_to_host_port stored in the proxy
        map (lxc.h:101-131: proxy4_tbl_value.identity) for the last packet;
        the map is emptied after each read."""
        m = self.L.maps.get("cilium_proxy4" if family == 4 else "cilium_proxy6")
        if m is None:
            return None
        keys = m.keys()
        ids = set()
        for k in keys:
            v = m.lookup(k)
            off = 8 if family == 4 else 20   # orig_daddr + orig_dport + pad
            ids.add(struct.unpack_from("<I", v, off)[0])
            m.delete(k)
        assert len(ids) <= 1, ids
        return ids.pop() if ids else None

    # ------------------------------------------------------- conntrack
    def ct_dump(self):
        """Every live entry of every endpoint's CT maps as oracle-format
        rows (cfc_oracle.h CFO_CT_ROW), sorted."""
        rows = []
        for lxc, names in self.ct_maps.items():
            for ct, nm in names.items():
                m = self.L.maps.get(nm)
                if m is None:
                    continue
                fam = 1 if ct.endswith("4_111") else 2
                kind = 0 if "_tcp" in ct else 1
                for k in m.keys():
                    v = m.lookup(k)
                    if v is None:
                        continue
                    r = bytearray(S.CT_ROW)
                    struct.pack_into("<HBB", r, 0, lxc + 1, kind, fam)
                    r[4:4 + len(k)] = k
                    r[44:100] = v[:56]
                    rows.append(bytes(r))
        rows.sort(key=lambda r: r[:44])
        return np.frombuffer(b"".join(rows), np.uint8).reshape(-1, S.CT_ROW).copy()

    def reset_counters(self):
        """Zero policy-entry counters and cilium_metrics (after a history
        run that only exists to populate CT)."""
        for lxc, pm in self.policy_map.items():
            for k in pm.keys():
                v = pm.lookup(k)
                pm.update(k, v[:2] + bytes(22))
        m = self.L.maps.get("cilium_metrics")
        if m is not None:
            for k in m.keys():
                m.delete(k)

    # ------------------------------------------------------- counters
    def policy_counters(self):
        out = {}
        for lxc, pm in self.policy_map.items():
            rows = []
            for k in pm.keys():
                v = pm.lookup(k)
                ident, dport, proto, eg = struct.unpack("<IHBB", k)
                pp, pk, by = struct.unpack("<H6xQQ", v)
                rows.append((ident, dport, proto, eg, pp, pk, by))
            rows.sort()
            out[lxc] = np.array(rows, dtype=np.uint64).reshape(-1, 7)
        return out

    def metrics(self):
        m = self.L.maps.get("cilium_metrics")
        rows = []
        if m is None:
            return np.zeros((0, 4), np.uint64)
        ncpu = H.ncpus_possible()
        for k in m.keys():
            v = m.lookup(k)
            cnt = sum(struct.unpack_from("<Q", v, 16 * c)[0] for c in range(ncpu))
            byt = sum(struct.unpack_from("<Q", v, 16 * c + 8)[0]
                      for c in range(ncpu))
            reason, dirb = k[0], k[1] & 3
            rows.append((reason, dirb, cnt, byt))
        rows.sort()
        return np.array(rows, dtype=np.uint64).reshape(-1, 4)


# ------------------------------------------------------------ run + derive
def _dport_out(pkt_out, off=14 + 20):
    return struct.unpack_from("<H", pkt_out, off + 2)[0]


NOTIFY_DROP, NOTIFY_TRACE = 1, 4                 # common.h:210-215
TRACE_TO_LXC, TRACE_TO_PROXY, TRACE_TO_HOST, TRACE_TO_STACK = 0, 1, 2, 3
EV_DT = np.dtype([("type", "u1"), ("subtype", "u1"), ("source", "<u2"),
                  ("hash", "<u4"), ("len_orig", "<u4"), ("len_cap", "<u4"),
                  ("src_label", "<u4"), ("dst_label", "<u4"), ("w6", "<u4"),
                  ("ifindex", "<u4")])
assert EV_DT.itemsize == 32


def _trace(evs, obs):
    """the trace_notify record (trace.h:71-81) at observation point obs"""
    for e in evs:
        if e["type"] == NOTIFY_TRACE and e["subtype"] == obs:
            return e
    return None


def _derive_ingress(h, i, ret, cb, pkt_out, evs, proxy_id):
    """-> action, verdict, identity, id_mask"""
    if ret == TC_ACT_SHOT:
        # send_drop_notify(skb, src_label, SECLABEL, LXC_ID, ...):
        # cb[1] = src << 16 | dst & 0xFFFF, cb[2] = reason (drop.h:94-102).
        # A missed tail call is reported by the netdev program with src 0.
        if cb[2] in (-140, -156, -157):
            # errors of the netdev program itself (send_drop_notify_error:
            # no identities recorded)
            return ret, cb[2], 0, 0
        return ret, cb[2], (cb[1] >> 16) & 0xFFFF, 0xFFFF
    if ret == TC_ACT_REDIRECT and cb[1] == HOST_IFINDEX:
        # proxy redirect rewrote the dport (lxc.h:118) and set
        # cb[CB_IFINDEX] = HOST_IFINDEX (bpf_lxc.c:1004); the source
        # identity is what the proxy map entry records
        v = _dport_out(pkt_out, l4_offset(h, i))
        assert proxy_id is not None
        assert proxy_id == cb[0] & 0xFFFFFFFF   # cb[CB_SRC_LABEL], l3.h:119
        return ret, v, proxy_id, 0xFFFFFFFF
    # delivered to a local endpoint: TRACE_TO_LXC carries the full source
    # identity (bpf_lxc.c:1006, :873); to the stack: not observable
    e = _trace(evs, TRACE_TO_LXC)
    if e is not None:
        return ret, 0, int(e["src_label"]), 0xFFFFFFFF
    return ret, 0, 0, 0


def _derive_egress(h, i, ret, cb, pkt_out, evs, proxy_id):
    if ret == TC_ACT_SHOT:
        if cb[3] == 0:
            # egress-stage drop: send_drop_notify(SECLABEL, dstID, 0, ...)
            return ret, cb[2], cb[1] & 0xFFFF, 0xFFFF
        # dropped by the destination endpoint's ingress policy
        return ret, cb[2], 0, 0
    if ret == TC_ACT_REDIRECT:
        # a proxy redirect (bpf_lxc.c:582-604) rewrote the dport to the proxy
        # port and left a proxy map entry; local delivery and to_host did
        # neither (a service may have rewritten the dport itself)
        if proxy_id is None:
            return ret, 0, 0, 0
        return ret, _dport_out(pkt_out, l4_offset(h, i)), 0, 0
    # to the stack: TRACE_TO_STACK carries dstID (bpf_lxc.c:687, :390)
    e = _trace(evs, TRACE_TO_STACK)
    if e is not None:
        return ret, 0, int(e["dst_label"]), 0xFFFFFFFF
    return ret, 0, 0, 0


def _events(dp, pkt):
    """the perf-ring samples of one packet -> EV_DT records (the len_cap
    payload bytes after each — the packet as the program had rewritten it
    so far — are not kept).  The
    reference objects are built with the config headers' DEBUG on, so the
    ring also carries cilium_dbg messages (CILIUM_NOTIFY_DBG_MSG, dbg.h) —
    a debugging aid outside the verdict path, skipped here."""
    out = []
    for raw in dp.ring.read():
        if raw[0] not in (NOTIFY_DROP, NOTIFY_TRACE):
            continue
        rec = np.frombuffer(raw[:32], EV_DT)[0]
        assert len(raw) >= 32 + int(rec["len_cap"])
        out.append(rec)
    return out


def run(dp: RefDatapath, h: S.Headers, mode, ep_lxc=None):
    n = len(h)
    action = np.zeros(n, np.int32)
    verdict = np.zeros(n, np.int32)
    ident = np.zeros(n, np.uint32)
    idmask = np.zeros(n, np.uint32)
    # skb->cb[0..4] after the run: for TC_ACT_SHOT these are the arguments
    # send_drop_notify left for the drop-notify tail call (drop.h:98-102:
    # exitcode, src << 16 | dst & 0xFFFF, reason, dst_id, ifindex)
    cbs = np.zeros((n, 5), np.int32)
    # IPv4: the packet's (saddr, daddr, first L4 word) as the program left
    # it (service translation, reverse NAT, a proxy's port); skb->hash as
    # the first perf-ring record of the header reports it (get_hash_recalc,
    # what lb4_select_slave reduced), hash_ok = 0 where none was sent
    pktv = np.zeros((n, 3 if h.family == 4 else 9), np.uint32)
    # IPv6 headers whose packet left as IPv4 (a NAT64 hop, bpf_lxc.c:1070-1083):
    # (saddr, daddr, first L4 word) of that IPv4 packet — its daddr is what
    # the IPv4 egress program's dstID derives from after a service step
    pkt4 = np.zeros((n, 3), np.uint32)
    pkt4_ok = np.zeros(n, np.uint8)
    hsh = np.zeros(n, np.uint32)
    hsh_ok = np.zeros(n, np.uint8)
    ev_hdr, ev_rec = [], []
    # bpf_ktime_get_sec() of each header's run (CLOCK_MONOTONIC seconds,
    # read before and after; 0xFFFFFFFF when a second boundary fell inside)
    clock = np.zeros(n, np.uint32)
    build = build_packet_v4 if h.family == 4 else build_packet_v6
    dp.ring.read()
    for i in range(n):
        # keep each run inside one second of bpf_ktime_get_sec() so its
        # clock is known exactly
        t = time.clock_gettime(time.CLOCK_MONOTONIC)
        if t - int(t) > 0.995:
            time.sleep(int(t) + 1.0005 - t)
        t0 = int(time.clock_gettime(time.CLOCK_MONOTONIC))
        if h.family == 4:
            pktv[i] = (h.saddr[i], h.daddr[i], int(h.sport[i]) | int(h.dport[i]) << 16)
        else:
            pktv[i, :4] = np.frombuffer(bytes(h.saddr[i]), "<u4")
            pktv[i, 4:8] = np.frombuffer(bytes(h.daddr[i]), "<u4")
            pktv[i, 8] = int(h.sport[i]) | int(h.dport[i]) << 16
        if mode in (MODE_XDP, MODE_FULL):
            ret = H.test_run_xdp(dp.xdp, build(h, i))
            if mode == MODE_XDP or ret == XDP_DROP:
                action[i] = ret
                verdict[i] = 0 if ret == XDP_PASS else -1
                assert not dp.ring.read()   # bpf_xdp.c notifies nothing
                continue
        if mode in (MODE_INGRESS, MODE_FULL):
            pkt = build(h, i)
            ret, cb, po = H.test_run_skb(dp.netdev, pkt, mark=int(h.mark[i]))
            evs = _events(dp, pkt)
            r = _derive_ingress(h, i, ret, cb, po, evs, dp.take_proxy_identity(h.family))
        else:
            pkt = build(h, i, LXC_MAC, NODE_MAC)
            ret, cb, po = H.test_run_skb(dp.ep_prog[ep_lxc], pkt)
            evs = _events(dp, pkt)
            r = _derive_egress(h, i, ret, cb, po, evs, dp.take_proxy_identity(h.family))
        action[i], verdict[i], ident[i], idmask[i] = r
        cbs[i] = cb
        if h.family == 4 and len(po) >= 14 + 20:
            l4 = l4_offset(h, i)
            pktv[i, 0], pktv[i, 1] = struct.unpack_from("<II", po, 14 + 12)
            if len(po) >= l4 + 4 and h.proto[i] in (6, 17):
                pktv[i, 2] = struct.unpack_from("<I", po, l4)[0]
        elif h.family == 6 and len(po) >= 14 + 20 and po[12:14] == b"\x08\x00":
            pkt4[i, 0], pkt4[i, 1] = struct.unpack_from("<II", po, 14 + 12)
            if len(po) >= 14 + 24 and h.proto[i] in (6, 17):
                pkt4[i, 2] = struct.unpack_from("<I", po, 14 + 20)[0]
            pkt4_ok[i] = 1
        elif h.family == 6 and len(po) >= 14 + 40:
            l4 = l4_offset(h, i)
            pktv[i, :8] = struct.unpack_from("<8I", po, 14 + 8)
            if len(po) >= l4 + 4 and h.proto[i] in (6, 17):
                pktv[i, 8] = struct.unpack_from("<I", po, l4)[0]
        if evs:
            hsh[i], hsh_ok[i] = int(evs[0]["hash"]), 1
        t1 = int(time.clock_gettime(time.CLOCK_MONOTONIC))
        clock[i] = t0 if t0 == t1 else 0xFFFFFFFF
        for e in evs:
            ev_hdr.append(i)
            ev_rec.append(e)
    assert dp.ring.lost == 0, f"perf ring lost {dp.ring.lost} samples"
    ev = np.array(ev_rec, EV_DT) if ev_rec else np.zeros(0, EV_DT)
    return (action, verdict, ident, idmask, cbs, np.array(ev_hdr, np.uint32), ev,
            clock, pktv, hsh, hsh_ok, pkt4, pkt4_ok)


def lpm_pin(ipc_map, h: S.Headers, pkt=None):
    """The kernel's own longest-prefix match (BPF_MAP_LOOKUP_ELEM on the LPM
    trie cilium_ipcache, kernel/bpf/lpm_trie.c) of every header's addresses,
    with the key ipcache_lookup4/6 builds (eps.h:49-80: prefixlen 32 static
    bits + the full address, family byte) -> (labels (n, 4) u32, hits (n, 4)
    u8) for the columns saddr, daddr, and the packet's saddr / daddr as the
    program left them (pkt = (saddrs, daddrs) after service translation;
    else saddr / daddr again).  The identity derivations of headers the reference reports
    nothing for rest on these lookups (bpf_netdev.c:374-398, bpf_lxc.c:516-532)."""
    n = len(h)
    fam = 1 if h.family == 4 else 2
    cols = [h.saddr, h.daddr,
            h.saddr if pkt is None else pkt[0], h.daddr if pkt is None else pkt[1]]
    lab = np.zeros((n, 4), np.uint32)
    hit = np.zeros((n, 4), np.uint8)
    for c, a in enumerate(cols):
        for i in range(n):
            ab = struct.pack("<I", int(a[i])) + bytes(12) if fam == 1 else bytes(a[i])
            key = struct.pack("<IHBB", 32 + (32 if fam == 1 else 128), 0, 0, fam) + ab
            v = ipc_map.lookup(key)
            if v is not None:
                lab[i, c] = struct.unpack_from("<I", v, 0)[0]
                hit[i, c] = 1
    return lab, hit


def save(name, t: S.Tables, h: S.Headers, mode, ep_lxc, res, dp):
    action, verdict, ident, idmask, cbs, ev_hdr, ev, clock, pkt, hsh, hsh_ok, pkt4, pkt4_ok = res
    extra = {}
    lb = getattr(t, "lb4", None) is not None or getattr(t, "lb6", None) is not None
    pk = None
    if lb:   # the packet's addresses as the programs left them
        pk = (pkt[:, 0], pkt[:, 1]) if h.family == 4 else \
            (np.ascontiguousarray(pkt[:, 0:4]).view(np.uint8).reshape(-1, 16),
             np.ascontiguousarray(pkt[:, 4:8]).view(np.uint8).reshape(-1, 16))
    lab, hit = lpm_pin(dp.L.maps["cilium_ipcache"], h, pk)
    extra.update(x_lpm=lab, x_lpm_hit=hit)
    if h.family == 6:
        # NAT64's IPv4 egress looks the v4-mapped destination's low 32 bits
        # up in the IPv4 ipcache (bpf_lxc.c:516-532 after :1070-1083)
        d4 = np.ascontiguousarray(np.asarray(h.daddr, np.uint8)[:, 12:16]).view("<u4").ravel()
        if getattr(t, "lb4", None) is not None and pkt4_ok.any():
            # (an IPv4 service step after the hop: the destination it left,
            # the backend, bpf_lxc.c:476-501)
            d4 = np.where(pkt4_ok != 0, pkt4[:, 1], d4).astype(np.uint32)
            extra.update(x_pkt4=pkt4, x_pkt4_ok=pkt4_ok)
        h4 = S.Headers(4, d4, d4, h.sport, h.dport, h.proto, h.flags, h.length, h.mark)
        l4, k4 = lpm_pin(dp.L.maps["cilium_ipcache"], h4)
        extra.update(x_lpm_nat=l4[:, 1], x_lpm_nat_hit=k4[:, 1])
    if lb:
        if getattr(t, "lb4", None) is not None:
            extra.update(lb4=t.lb4, revnat4=t.revnat4)
        if getattr(t, "lb6", None) is not None:
            extra.update(lb6=t.lb6, revnat6=t.revnat6)
        extra.update(x_pkt=pkt, x_hash=hsh, x_hash_ok=hsh_ok)
        if h.hash is not None:
            extra["h_hash"] = h.hash
    if t.ct is not None:
        # CT before (loaded by the oracle / engine) and after the stream
        extra.update(ct=t.ct, x_ct=dp.ct_dump())
    d = dict(mode=np.int32(mode), ep_lxc=np.int32(ep_lxc or 0),
             ipcache=t.ipcache, endpoints=t.endpoints, prefilter=t.prefilter,
             seclabel=np.array(sorted(t.seclabel.items()), np.uint32).reshape(-1, 2),
             h_family=np.int32(h.family), h_saddr=h.saddr, h_daddr=h.daddr,
             h_sport=h.sport, h_dport=h.dport, h_proto=h.proto,
             h_flags=h.flags, h_length=h.length, h_mark=h.mark,
             x_action=action, x_verdict=verdict, x_identity=ident,
             x_idmask=idmask, x_cb=cbs, x_metrics=dp.metrics(),
             # cilium_events perf-ring samples (trace_notify / drop_notify
             # records, 32 bytes each) and the header each belongs to
             x_ev_hdr=ev_hdr, x_ev=ev.view(np.uint8).reshape(-1, 32),
             x_clock=clock, **extra)
    if h.tcpflags is not None:
        d["h_tcpflags"] = h.tcpflags
    for lxc, pol in t.policy.items():
        d[f"policy_{lxc}"] = pol
    for lxc, c in dp.policy_counters().items():
        d[f"x_counters_{lxc}"] = c
    out_dir = GOLDEN + "_oracle" if name in ORACLE_ONLY else GOLDEN
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"{name}.npz")
    np.savez_compressed(path, **d)
    return path


# ------------------------------------------------------------ scenarios
def sc_c2_ingress(n=20000, seed=2, n_prefixes=100_000, n_policy=16384):
    t = S.config_c2(seed, n_prefixes=n_prefixes, n_policy=n_policy)
    h = S.headers_c2(t, int(n * 1.02), seed=seed)
    h = _keep(h, S.ensure_no_reverse(h))
    h = h.slice(0, n)
    return t, h, MODE_INGRESS, None


def sc_small_ingress(n=20000, seed=1):
    """C1-sized: a few hundred prefixes, ~100 identities, 3 endpoints with
    small policies (examples/policies scale)."""
    rng = np.random.default_rng(seed)
    ipc = S.gen_ipcache_v4(rng, 300, label_base=256, label_mod=100)
    eps = np.concatenate([S.endpoint_v4(S.LXC_IPV4, 100, S.EP_LXC_ID),
                          S.endpoint_v4(S.ip4("10.0.1.2"), 101, 0x2020),
                          S.endpoint_v4(S.ip4("10.0.1.3"), 0, 0x3030),
                          S.endpoint_v4(S.ip4("10.0.1.4"), 104, 0x4040),  # no program
                          S.endpoint_v4(S.ip4("10.0.255.254"), 0, 0xFFF0, 1)])
    idents = np.unique(ipc["label"])
    pol = {S.EP_LXC_ID: S.gen_policy(rng, 50, idents, wildcard=3,
                                     proxy_frac=0.2),
           0x2020: S.gen_policy(rng, 40, idents, wildcard=2, l3_frac=0.2),
           0x3030: np.zeros(0, S.POLICY_DT)}
    t = S.Tables(ipc, eps, pol, np.zeros(0, S.PREFILTER_DT),
                 {int(e["lxc_id"]): S.EP_SECLABEL for e in eps})
    h = S.gen_headers_v4(rng, int(n * 1.02), ipc, S.local_v4_addrs(t),
                         local_frac=0.9, frag=0.05, mark_host=0.05,
                         mark_proxy=0.05, other_proto=0.02,
                         proxy_ident=np.concatenate([idents[:8], [1, 2, 3, 4, 5, 70000]]))
    h = _keep(h, S.ensure_no_reverse(h)).slice(0, n)
    return t, h, MODE_INGRESS, None


def sc_c1_ingress(n=20000, seed=1):
    """C1 (BASELINE.json configs[0]): the MapState the example policies of
    examples/policies/{l3,l4} give 11 local endpoints (cilium_amd.
    policy_resolver), ~100 pod + reserved + CIDR identities; the C1 stream
    into those endpoints.  The harness runs one bpf_lxc.o, so every
    endpoint carries the compiled SECLABEL here."""
    t, _ = S.config_c1(seed)
    t.seclabel = {k: S.EP_SECLABEL for k in t.seclabel}
    h = S.headers_c1(t, int(n * 1.02), seed=seed)
    h = _keep(h, S.ensure_no_reverse(h)).slice(0, n)
    return t, h, MODE_INGRESS, None


def sc_edge_ingress(seed=7):
    """Hand-picked fallback cases: L4 hit, L3 fallback, wildcard port,
    fragments (L3 only), proxy, ICMP echo -> port 2048 quirk, unknown proto,
    identity override rules (label 0/HOST/CLUSTER ignored), marks."""
    ipc = np.concatenate([
        S._v4_entries(np.array([S.ip4("172.16.0.0")], np.uint32), [12], [1000]),
        S._v4_entries(np.array([S.ip4("172.16.5.0")], np.uint32), [24], [1001]),
        S._v4_entries(np.array([S.ip4("172.16.5.128")], np.uint32), [25], [0]),
        S._v4_entries(np.array([S.ip4("172.16.6.0")], np.uint32), [24], [S.HOST_ID]),
        S._v4_entries(np.array([S.ip4("172.16.7.0")], np.uint32), [24], [S.CLUSTER_ID]),
        S._v4_entries(np.array([S.ip4("172.16.8.8")], np.uint32), [32], [4242]),
        S._v4_entries(np.array([S.ip4("0.0.0.0")], np.uint32), [0], [7]),
        S._v4_entries(np.array([S.ip4("192.168.0.0")], np.uint32), [16], [0x80000001]),
    ])
    eps = np.concatenate([S.endpoint_v4(S.LXC_IPV4, 100, S.EP_LXC_ID),
                          S.endpoint_v4(S.ip4("10.0.255.254"), 0, 0xFFF0, 1)])
    ht = lambda p: int(S.htons(p))   # noqa: E731
    rows = [(1000, ht(80), 6, 0, 0), (1000, ht(53), 17, 0, 0),
            (1001, 0, 0, 0, 0), (4242, ht(443), 6, 0, ht(10001)),
            (0, ht(8080), 6, 0, 0), (0, ht(9090), 6, 0, ht(10002)),
            (7, 0, 0, 0, 0), (1000, 8, 1, 0, 0), (1000, 0, 1, 0, 0),
            (S.WORLD_ID, ht(22), 6, 0, 0), (S.HOST_ID, 0, 0, 0, 0),
            (0x80000001, ht(80), 6, 0, 0), (1000, ht(80), 6, 1, 0),
            (70000, 0, 0, 0, 0), (1001, ht(80), 6, 0, ht(10003))]
    pol = np.zeros(len(rows), S.POLICY_DT)
    a = np.array(rows, dtype=np.int64)
    pol["identity"], pol["dport"], pol["proto"] = a[:, 0], a[:, 1], a[:, 2]
    pol["egress"], pol["proxy_port"] = a[:, 3], a[:, 4]
    t = S.Tables(ipc, eps, {S.EP_LXC_ID: pol}, np.zeros(0, S.PREFILTER_DT),
                 {S.EP_LXC_ID: S.EP_SECLABEL, 0xFFF0: S.EP_SECLABEL})
    srcs = ["172.16.1.1", "172.16.5.9", "172.16.5.200", "172.16.6.1",
            "172.16.7.1", "172.16.8.8", "8.8.8.8", "192.168.3.4", "0.0.0.0"]
    dsts = ["64.48.32.16", "10.0.255.254", "9.9.9.9"]
    cases = []
    for s in srcs:
        for d in dsts:
            for proto, sp, dp in ((6, 40000, 80), (6, 40001, 443), (6, 40002, 8080),
                                  (6, 40003, 9090), (6, 40004, 22), (17, 40005, 53),
                                  (17, 40006, 80), (1, 8, 0x1234), (1, 0, 7),
                                  (1, 3, 0), (1, 11, 0), (47, 0, 0), (132, 1, 2)):
                for fl in (0, S.HF_FRAG, S.HF_TCP_CLOSE):
                    for mark in (0, 0xC00, 0xA00 | (4242 & 0xFFFF) << 16,
                                 0xB00 | (70000 & 0xFFFF) << 16 | (70000 >> 16),
                                 0xB00 | (3 << 16)):
                        cases.append((s, d, proto, sp, dp, fl, mark))
    n = len(cases)
    rng = np.random.default_rng(seed)
    h = S.Headers(4, np.array([S.ip4(c[0]) for c in cases], np.uint32),
                  np.array([S.ip4(c[1]) for c in cases], np.uint32),
                  np.array([c[3] if c[2] == 1 else ht(c[3]) for c in cases], np.uint16),
                  np.array([c[4] if c[2] == 1 else ht(c[4]) for c in cases], np.uint16),
                  np.array([c[2] for c in cases], np.uint8),
                  np.array([c[5] for c in cases], np.uint8),
                  rng.integers(60, 200, size=n).astype(np.uint16),
                  np.array([c[6] for c in cases], np.uint32))
    # make source ports distinct per case so no two headers form a reverse pair
    tcpudp = (h.proto == 6) | (h.proto == 17)
    h.sport[tcpudp] = S.htons(20000 + np.arange(n)[tcpudp] % 40000)
    return t, h, MODE_INGRESS, None


def sc_c2_egress(n=20000, seed=3):
    t = S.config_c2(seed, n_prefixes=100_000, n_policy=16384, n_endpoints=2)
    rng = np.random.default_rng(seed + 7)
    h = S.gen_headers_v4(rng, n, t.ipcache, S.local_v4_addrs(t),
                         local_frac=0.05, mark_host=0, mark_proxy=0,
                         src_fixed=S.LXC_IPV4)
    # swap roles: destination addresses come from the ipcache (in_prefix),
    # sources are the endpoint; 2% spoofed sources (DROP_INVALID_SIP)
    dst = S._addr_in_prefix_v4(rng, t.ipcache,
                               rng.integers(0, len(t.ipcache), size=n))
    loc = S.local_v4_addrs(t)
    r = rng.random(n)
    h.daddr = np.where(r < 0.85, dst, np.where(
        r < 0.95, loc[rng.integers(0, len(loc), size=n)],
        rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32))
    ).astype(np.uint32)
    # cluster range 0x100000 mask 0xff0000: some 16.x destinations -> CLUSTER_ID
    cl = rng.random(n) < 0.02
    h.daddr[cl] = (h.daddr[cl] & np.uint32(0xFF00FFFF)) | np.uint32(0x100000)
    spoof = rng.random(n) < 0.02
    h.saddr[spoof] = S.ip4("64.48.32.17")
    h = _keep(h, S.ensure_no_reverse(h))
    return t, h, MODE_EGRESS, S.EP_LXC_ID


def _prefilter_v4(rng, ipc, n_fix, n_dyn):
    pf = np.zeros(n_fix + n_dyn, S.PREFILTER_DT)
    pf["family"] = 1
    fix = rng.integers(1 << 24, 224 << 24, size=n_fix, dtype=np.uint64).astype(np.uint32)
    pf["plen"][:n_fix] = 32
    pf["addr"][:n_fix, :4] = S.be32_to_bytes(S.byteswap32(fix))
    dl = rng.choice(np.array([8, 12, 16, 20, 24, 28, 31, 32]), size=n_dyn)
    dh = rng.integers(1 << 24, 224 << 24, size=n_dyn, dtype=np.uint64).astype(np.uint32)
    dh &= (np.uint64(0xFFFFFFFF) << (32 - dl.astype(np.uint64))).astype(np.uint32)
    pf["plen"][n_fix:] = dl
    pf["addr"][n_fix:, :4] = S.be32_to_bytes(S.byteswap32(dh))
    pf["dyn"][n_fix:] = 1
    # unique keys
    _, u = np.unique(np.stack([pf["dyn"], pf["plen"],
                               pf["addr"][:, :4].copy().view("<u4").ravel()], 1),
                     axis=0, return_index=True)
    return pf[np.sort(u)]


def sc_xdp(n=20000, seed=4, mode=MODE_XDP):
    t = S.config_c2(seed, n_prefixes=20_000, n_policy=4096)
    rng = np.random.default_rng(seed + 11)
    t.prefilter = _prefilter_v4(rng, t.ipcache, 5000, 300)
    h = S.headers_c2(t, n, seed=seed, local_frac=0.85)
    r = rng.random(n)
    fix = t.prefilter[t.prefilter["dyn"] == 0]
    dyn = t.prefilter[t.prefilter["dyn"] == 1]
    fa = fix["addr"][:, :4].copy().view("<u4").ravel()
    sel = r < 0.25
    h.saddr[sel] = fa[rng.integers(0, len(fa), size=int(sel.sum()))]
    sel2 = (r >= 0.25) & (r < 0.4)
    di = rng.integers(0, len(dyn), size=int(sel2.sum()))
    base = S.byteswap32(dyn["addr"][di, :4].copy().view("<u4").ravel()).astype(np.uint64)
    pl = dyn["plen"][di].astype(np.uint64)
    hb = rng.integers(0, 1 << 32, size=len(di), dtype=np.uint64) & ((np.uint64(1) << (np.uint64(32) - pl)) - np.uint64(1))
    h.saddr[sel2] = S.byteswap32((base | hb).astype(np.uint32))
    h = _keep(h, S.ensure_no_reverse(h))
    return t, h, mode, None


def sc_empty(n=2000, seed=5):
    """Empty ipcache / policymap / prefilter: everything WORLD, DROP_POLICY."""
    t = S.Tables(np.zeros(0, S.IPCACHE_DT),
                 S.endpoint_v4(S.LXC_IPV4, 100, S.EP_LXC_ID),
                 {S.EP_LXC_ID: np.zeros(0, S.POLICY_DT)},
                 np.zeros(0, S.PREFILTER_DT), {S.EP_LXC_ID: S.EP_SECLABEL})
    rng = np.random.default_rng(seed)
    ipc = S.gen_ipcache_v4(rng, 100)
    h = S.gen_headers_v4(rng, n, ipc, S.local_v4_addrs(t))
    h = _keep(h, S.ensure_no_reverse(h))
    return t, h, MODE_INGRESS, None


# ------------------------------------------------------------ IPv6 scenarios
def _v6(*specs):
    """[(addr string, plen, label), ...] -> ipcache entries"""
    return np.concatenate([S._v6_entries(S.ip6(a)[None, :], [l], [lab])
                           for a, l, lab in specs])


def sc_edge_ingress_v6(seed=8):
    """The IPv6 fallback cases: L4 / L3 / wildcard-port hits, ICMPv6 (echo
    request -> port 128, other types -> 0), extension headers, the
    FRAGMENT / NONE next-header drops, unknown protocols, the identity
    override rule (label 0/CLUSTER ignored) and the marks."""
    ipc = _v6(("2001:db8::", 32, 1000), ("2001:db8:5::", 48, 1001),
              ("2001:db8:5:8000::", 49, 0), ("2001:db8:6::", 48, S.HOST_ID),
              ("2001:db8:7::", 48, S.CLUSTER_ID), ("2001:db8:8::8", 128, 4242),
              ("::", 0, 7), ("fd00::", 16, 0x80000001),
              ("2001:db8:9::", 64, 70000))
    host = S.LXC_IPV6.copy()
    host[12:] = [0xff, 0xff, 0xff, 0xfe]
    eps = np.concatenate([S.endpoint_v6(S.LXC_IPV6, 100, S.EP_LXC_ID),
                          S.endpoint_v6(host, 0, 0xFFF0, 1)])
    ht = lambda p: int(S.htons(p))   # noqa: E731
    rows = [(1000, ht(80), 6, 0, 0), (1000, ht(53), 17, 0, 0),
            (1001, 0, 0, 0, 0), (4242, ht(443), 6, 0, ht(10001)),
            (0, ht(8080), 6, 0, 0), (0, ht(9090), 6, 0, ht(10002)),
            (7, 0, 0, 0, 0), (1000, 128, 58, 0, 0), (1001, 0x8000, 58, 0, 0),
            (4242, 0, 58, 0, 0), (S.WORLD_ID, ht(22), 6, 0, 0),
            (S.HOST_ID, 0, 0, 0, 0), (0x80000001, ht(80), 6, 0, 0),
            (1000, ht(80), 6, 1, 0), (70000, ht(22), 6, 0, ht(10003)),
            (1001, ht(80), 6, 0, ht(10003)), (1000, 0, 132, 0, 0)]
    pol = np.zeros(len(rows), S.POLICY_DT)
    a = np.array(rows, dtype=np.int64)
    pol["identity"], pol["dport"], pol["proto"] = a[:, 0], a[:, 1], a[:, 2]
    pol["egress"], pol["proxy_port"] = a[:, 3], a[:, 4]
    t = S.Tables(ipc, eps, {S.EP_LXC_ID: pol}, np.zeros(0, S.PREFILTER_DT),
                 {S.EP_LXC_ID: S.EP_SECLABEL, 0xFFF0: S.EP_SECLABEL})
    srcs = ["2001:db8:1::1", "2001:db8:5::9", "2001:db8:5:8000::1",
            "2001:db8:6::1", "2001:db8:7::1", "2001:db8:8::8", "3fff::1",
            "fd00:1::4", "2001:db8:9::77", "::"]
    dsts = [S.LXC_IPV6, host, S.ip6("2001:db8:ffff::1")]
    cases = []
    for si, sa in enumerate(srcs):
        for d in dsts:
            for proto, sp, dp in ((6, 40000, 80), (6, 40001, 443), (6, 40002, 8080),
                                  (6, 40003, 9090), (6, 40004, 22), (17, 40005, 53),
                                  (17, 40006, 80), (58, 128, 0x1234),
                                  (58, 129, 0x77), (58, 1, 0), (58, 3, 0),
                                  (58, 136, 0), (47, 0, 0), (132, 1, 2),
                                  (44, 0, 0), (59, 0, 0)):
                for fl in (0, S.HF_EXTHDR, S.HF_TCP_CLOSE):
                    for mark in (0, 0xC00, 0xA00 | (4242 & 0xFFFF) << 16,
                                 0xB00 | (70000 & 0xFFFF) << 16 | (70000 >> 16),
                                 0xB00 | (3 << 16)):
                        cases.append((S.ip6(sa), d, proto, sp, dp, fl, mark))
    n = len(cases)
    rng = np.random.default_rng(seed)
    raw = lambda c: c[2] in (58, 44, 59, 47)   # noqa: E731  (no port swap)
    h = S.Headers(6, np.stack([c[0] for c in cases]).astype(np.uint8),
                  np.stack([np.asarray(c[1], np.uint8) for c in cases]),
                  np.array([c[3] if raw(c) else ht(c[3]) for c in cases], np.uint16),
                  np.array([c[4] if raw(c) else ht(c[4]) for c in cases], np.uint16),
                  np.array([c[2] for c in cases], np.uint8),
                  np.array([c[5] for c in cases], np.uint8),
                  rng.integers(100, 300, size=n).astype(np.uint16),
                  np.array([c[6] for c in cases], np.uint32))
    tcpudp = (h.proto == 6) | (h.proto == 17)
    h.sport[tcpudp] = S.htons(20000 + np.arange(n)[tcpudp] % 40000)
    return t, h, MODE_INGRESS, None


def sc_c3_ingress(n=20000, seed=3):
    t = S.config_c3(seed, n_prefixes=100_000, n_v4_prefixes=20_000,
                    n_policy=16384, n_prefilter=0)
    h = S.headers_c3(t, int(n * 1.02), seed=seed, ext=0.05, exthdr_drop=0.01,
                     local_frac=0.9)
    h = _keep(h, S.ensure_no_reverse(h)).slice(0, n)
    return t, h, MODE_INGRESS, None


def sc_c3_egress(n=20000, seed=9):
    t = S.config_c3(seed, n_prefixes=100_000, n_v4_prefixes=20_000,
                    n_policy=16384, n_endpoints=2, n_prefilter=0)
    rng = np.random.default_rng(seed + 7)
    ipc6 = t.ipcache[t.ipcache["family"] == 2]
    loc = S.local_v6_addrs(t)
    h = S.gen_headers_v6(rng, n, ipc6, loc, local_frac=1.0, mark_host=0,
                         mark_proxy=0, src_fixed=S.LXC_IPV6, ext=0.05)
    dst = S._addr_in_prefix_v6(rng, ipc6, rng.integers(0, len(ipc6), size=n))
    r = rng.random(n)
    sel_loc = (r >= 0.85) & (r < 0.93)
    sel_rnd = r >= 0.93
    d = dst.copy()
    d[sel_loc] = loc[rng.integers(0, len(loc), size=int(sel_loc.sum()))]
    d[sel_rnd] = rng.integers(0, 256, size=(int(sel_rnd.sum()), 16),
                              dtype=np.uint16).astype(np.uint8)
    # inside the router's /64 (match_prefix_64 -> CLUSTER_ID), never the
    # router address itself (echo requests to it are answered, not routed)
    cl = rng.random(n) < 0.03
    d[cl, :8] = S.ROUTER_IPV6[:8]
    d[cl, 8] = 0x80 | d[cl, 8]
    h.daddr = d
    spoof = rng.random(n) < 0.02
    h.saddr[spoof] = S.ip6("2001:db8::dead")
    h = _keep(h, S.ensure_no_reverse(h) & _no_related(h))
    return t, h, MODE_EGRESS, S.EP_LXC_ID


def _no_related(h):
    """Drop ICMPv6 error messages (types 1-4) between an address pair that
    already carried ICMPv6: ct_lookup6 looks them up as TUPLE_F_RELATED
    (conntrack.h) and an earlier packet's entry would then skip policy —
    state the per-batch oracle does not model."""
    keep = np.ones(len(h), bool)
    seen = set()
    for i in range(len(h)):
        if int(h.proto[i]) != S.IPPROTO_ICMPV6:
            continue
        pair = frozenset((bytes(h.saddr[i]), bytes(h.daddr[i])))
        if 1 <= (int(h.sport[i]) & 0xFF) <= 4 and pair in seen:
            keep[i] = False
        seen.add(pair)
    return keep


def _prefilter_v6(rng, n_fix, n_dyn):
    pf = np.zeros(n_fix + n_dyn, S.PREFILTER_DT)
    pf["family"] = 2
    a = rng.integers(0, 256, size=(n_fix + n_dyn, 16), dtype=np.uint16).astype(np.uint8)
    a[:, 0] = 0x20 | (a[:, 0] & 0x0F)
    pl = np.full(n_fix + n_dyn, 128)
    pl[n_fix:] = rng.choice(np.array([16, 24, 32, 48, 56, 64, 96, 127, 128]),
                            size=n_dyn)
    pf["plen"] = pl
    pf["addr"] = S.mask_v6(a, pl)
    pf["dyn"][n_fix:] = 1
    _, u = np.unique(np.concatenate([pf["dyn"][:, None], pf["plen"][:, None],
                                     pf["addr"]], 1), axis=0, return_index=True)
    return pf[np.sort(u)]


def sc_xdp_v6(n=20000, seed=10, mode=MODE_XDP):
    t = S.config_c3(seed, n_prefixes=20_000, n_v4_prefixes=5_000,
                    n_policy=4096, n_prefilter=0)
    rng = np.random.default_rng(seed + 11)
    t.prefilter = np.concatenate([_prefilter_v4(rng, t.ipcache[t.ipcache["family"] == 1],
                                                500, 50),
                                  _prefilter_v6(rng, 5000, 300)])
    h = S.headers_c3(t, n, seed=seed, local_frac=0.85, ext=0.05)
    r = rng.random(n)
    pf6 = t.prefilter[t.prefilter["family"] == 2]
    fix, dyn = pf6[pf6["dyn"] == 0], pf6[pf6["dyn"] == 1]
    sel = r < 0.25
    h.saddr[sel] = fix["addr"][rng.integers(0, len(fix), size=int(sel.sum()))]
    sel2 = (r >= 0.25) & (r < 0.4)
    di = rng.integers(0, len(dyn), size=int(sel2.sum()))
    h.saddr[sel2] = S._addr_in_prefix_v6(rng, dyn, di)
    h = _keep(h, S.ensure_no_reverse(h))
    return t, h, mode, None


# ------------------------------------------------------------ conntrack
def _ct_tables(seed, family):
    """small_ingress-sized tables, two endpoints with programs (EP_LXC_ID and
    0x2020), dual-stack when family == 6."""
    rng = np.random.default_rng(seed)
    if family == 4:
        t = S.config_c2(seed, n_prefixes=2000, n_policy=400, n_endpoints=2)
    else:
        t = S.config_c3(seed, n_prefixes=2000, n_v4_prefixes=500, n_policy=400,
                        n_endpoints=2, n_prefilter=0)
    return t, rng


def _ct_history(family, seed):
    """Tables, and the CT state the reference itself made from a history
    stream: flows into both endpoints, flows out of EP_LXC_ID (some to the
    other local endpoint), with extra L3 allow rules that are removed before
    the test stream (a policy change: those flows become denied)."""
    t, rng = _ct_tables(seed, family)
    fam_ipc = t.ipcache[t.ipcache["family"] == (1 if family == 4 else 2)]
    gen = S.gen_headers_v4 if family == 4 else S.gen_headers_v6
    loc = S.local_v4_addrs(t) if family == 4 else S.local_v6_addrs(t)
    ep_addr = S.LXC_IPV4 if family == 4 else S.LXC_IPV6
    kw = dict(frag=0) if family == 4 else dict(ext=0, exthdr_drop=0)
    h_in = gen(rng, 1500, fam_ipc, loc[:2], local_frac=1.0, mark_host=0,
               mark_proxy=0, other_proto=0, **kw)
    h_in.flags[:] &= np.uint8(0xFF ^ S.HF_TCP_CLOSE)
    h_out = gen(rng, 1500, fam_ipc, loc[:2], local_frac=0.4, mark_host=0,
                mark_proxy=0, other_proto=0, src_fixed=ep_addr, **kw)
    h_out.flags[:] &= np.uint8(0xFF ^ S.HF_TCP_CLOSE)
    dst = gen(rng, 1500, fam_ipc, loc[:1], local_frac=1.0, **kw).saddr
    nonloc = rng.random(1500) < 0.6
    h_out.daddr[nonloc] = dst[nonloc]
    idents = np.unique(fam_ipc["label"])
    extra = rng.choice(idents, size=2 * len(idents) // 3, replace=False)
    hist_pol = {}
    for lxc, pol in t.policy.items():
        add = np.zeros(2 * len(extra), S.POLICY_DT)
        add["identity"] = np.concatenate([extra, extra])
        add["egress"][len(extra):] = 1
        have = {(int(r["identity"]), int(r["dport"]), int(r["proto"]),
                 int(r["egress"])) for r in pol}
        add = add[[(int(r["identity"]), 0, 0, int(r["egress"])) not in have
                   for r in add]]
        hist_pol[lxc] = np.concatenate([pol, add])
    th = S.Tables(t.ipcache, t.endpoints, hist_pol, t.prefilter, t.seclabel)
    dp = RefDatapath(th)
    run(dp, h_in, MODE_INGRESS)
    run(dp, h_out, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    for lxc, pol in hist_pol.items():       # the policy change
        pm = dp.policy_map[lxc]
        for r in pol[len(t.policy[lxc]):]:
            pm.delete(policy_key(r))
    dp.reset_counters()
    return t, rng, dp, dict(fam_ipc=fam_ipc, gen=gen, loc=loc, ep_addr=ep_addr,
                            kw=kw, h_in=h_in, h_out=h_out, dst=dst, extra=extra)


def _ct_scenario(family, mode, seed, n=6000):
    """Conntrack: CT state made by the reference
    itself from a history stream, then a test stream of established
    packets, replies, ICMP errors related to known flows, FIN/RST on known
    flows, new flows, and established flows that a policy change now denies
    (ct_delete).  Intra-batch CT hazards are removed with the oracle's
    sequential check so the batch engine and the per-packet reference see
    the same CT state for every header (the ct_seq_* fixtures keep them)."""
    import oracle as O
    t, rng, dp, X = _ct_history(family, seed)
    fam_ipc, gen, loc, ep_addr, kw = X["fam_ipc"], X["gen"], X["loc"], X["ep_addr"], X["kw"]
    h_in, h_out, dst = X["h_in"], X["h_out"], X["dst"]
    # test stream
    icmp = S.IPPROTO_ICMP if family == 4 else S.IPPROTO_ICMPV6
    err = 3 if family == 4 else 1
    if mode == MODE_INGRESS:
        fwd, rep = h_in, h_out
    else:   # replies leave from EP_LXC_ID (the program under test)
        fwd = h_out
        rep = S.take(h_in, (h_in.daddr == loc[0]).all(-1) if family == 6
                     else h_in.daddr == loc[0])
    m = int(n * 1.4)
    parts = []

    def tcp_flags(x, opening):
        """TCP byte 13 of established traffic: ACK, PSH|ACK, (SYN|)ACK, and
        FIN|ACK or RST on the closing packets (HF_TCP_CLOSE, byte 12 bit 0):
        what ct_update_timeout accumulates into the entry's seen flags and
        reports on change (conntrack.h:137-185)"""
        k = len(x)
        close = (x.flags & S.HF_TCP_CLOSE) != 0
        f = rng.choice(np.array([0x10, 0x18, opening], np.uint8), size=k)
        f = np.where(close, rng.choice(np.array([0x11, 0x04], np.uint8), size=k), f)
        x.tcpflags = np.where(x.proto == S.IPPROTO_TCP, f, 0).astype(np.uint8)
        return x
    a = S.take(fwd, rng.integers(0, len(fwd), size=int(m * 0.35)))
    a.flags[(rng.random(len(a)) < 0.08) & (a.proto == S.IPPROTO_TCP)] |= np.uint8(S.HF_TCP_CLOSE)
    parts.append(tcp_flags(a, 0x02))
    b = S.reverse(S.take(rep, rng.integers(0, len(rep), size=int(m * 0.3))))
    b.flags[(rng.random(len(b)) < 0.08) & (b.proto == S.IPPROTO_TCP)] |= np.uint8(S.HF_TCP_CLOSE)
    parts.append(tcp_flags(b, 0x12))
    c = S.reverse(S.take(rep, rng.integers(0, len(rep), size=int(m * 0.05))))
    c.proto[:] = icmp
    c.sport[:] = err
    c.dport[:] = 0
    parts.append(c)
    if mode == MODE_INGRESS:
        d = gen(rng, int(m * 0.3), fam_ipc, loc, local_frac=0.95, **kw)
    else:
        d = gen(rng, int(m * 0.3), fam_ipc, loc, local_frac=0.1,
                src_fixed=ep_addr, **kw)
        sel = rng.random(len(d)) < 0.8
        d.daddr[sel] = dst[rng.integers(0, len(dst), size=int(sel.sum()))]
    parts.append(d)
    h = S.concat(parts)
    h = S.take(h, rng.permutation(len(h)))
    ep = S.EP_LXC_ID if mode == MODE_EGRESS else 0
    for _ in range(6):
        o = O.Oracle(t)
        oa, ov, oi, ct = o.classify(h, mode, ep, want_ct=True)
        hz = o.ct_apply(h, mode, ep, oi, ov, ct, hazard=True)
        if not hz.any():
            break
        h = _keep(h, hz == 0)
    assert not hz.any()
    h = h.slice(0, n)
    return t, h, mode, ep or None, dp


def _ct_seq_scenario(family, mode, seed, n=7000):
    """The tables and CT history of _ct_scenario, and a test stream that
    keeps every intra-batch conntrack dependency (the reference applies each
    packet's CT writes before the next packet's lookup, conntrack.h:221-285,
    615-772; the reply override bpf_lxc.c:963-970, :538-545): new flows with
    several packets (SYN, then ACK / data, FIN or RST, a packet after the
    close), the replies of new flows between the two local endpoints and
    ICMP errors related to them, runs of packets of established flows
    (report aggregation, __ct_update_timeout), and several packets of
    established flows the policy change now denies (ct_delete, then the
    flow's later packets).  Nothing is removed: the reference runs the
    stream packet by packet and the fixture is its result."""
    t, rng, dp, X = _ct_history(family, seed)
    fam_ipc, gen, loc, ep_addr, kw = X["fam_ipc"], X["gen"], X["loc"], X["ep_addr"], X["kw"]
    h_in, h_out, dst = X["h_in"], X["h_out"], X["dst"]
    icmp = S.IPPROTO_ICMP if family == 4 else S.IPPROTO_ICMPV6
    err, echo = (3, 8) if family == 4 else (1, 128)
    TCP = S.IPPROTO_TCP
    parts, pos = [], []

    def tcpf(h, f, close=False):
        h.tcpflags = np.where(h.proto == TCP, np.asarray(f, np.uint8), 0).astype(np.uint8)
        if close:
            h.flags[h.proto == TCP] |= np.uint8(S.HF_TCP_CLOSE)
        else:
            h.flags[:] &= np.uint8(0xFF ^ S.HF_TCP_CLOSE)
        return h

    def steps(base, script):
        """one flow per row of base; script: (probability, make(Headers) ->
        Headers) per step, in order; every step after the one before"""
        k = len(base)
        at = rng.random(k) * 0.85
        for p, make in script:
            keep = rng.random(k) < p
            h = make(S.take(base, np.flatnonzero(keep)))
            h.length = rng.integers(60 if family == 4 else 100, 1500,
                                    size=len(h)).astype(np.uint16)
            parts.append(h)
            pos.append(at[keep])
            at = at + rng.random(k) * 0.03

    def fix_icmp(h):   # a new ICMP flow opens with an echo request
        ic = h.proto == icmp
        h.sport[ic] = echo
        h.dport[ic] = 0
        return h

    def icmp_err(h):   # an ICMP error travelling the other way, related to the flow
        r = S.reverse(h)
        r.proto[:] = icmp
        r.sport[:] = err
        r.dport[:] = 0
        r.tcpflags = np.zeros(len(r), np.uint8)
        return r
    def icmp_same(h):  # an ICMP error the same way (e.g. a router's, about the flow)
        r = S.take(h, np.arange(len(h)))
        r.proto[:] = icmp
        r.sport[:] = err
        r.dport[:] = 0
        r.tcpflags = np.zeros(len(r), np.uint8)
        return r
    copy = lambda x: S.take(x, np.arange(len(x)))   # noqa: E731
    m = n // 7
    if mode == MODE_INGRESS:   # replies: of the endpoint's own flows (history)
        fwd, rep = h_in, h_out
    else:
        fwd = h_out
        rep = S.take(h_in, (h_in.daddr == loc[0]).all(-1) if family == 6
                     else h_in.daddr == loc[0])
    # the identity each flow is checked with (ingress: its source's;
    # egress: its destination's), and what the policy (after the change)
    # admits on L3: most new flows are opened from / to those
    o = __import__("oracle").Oracle(t)
    ep0 = S.EP_LXC_ID if mode == MODE_EGRESS else 0
    _, fv, _, fct = o.classify(fwd, mode, ep0, want_ct=True)
    est_ok = ((fct & 7) == 5) & (fv >= 0)            # established, still allowed
    denied = ((fct & 7) == 5) & (fv == -133)         # established, now denied
    egr = 1 if mode == MODE_EGRESS else 0
    allow = np.unique(np.concatenate([
        pol["identity"][(pol["dport"] == 0) & (pol["proto"] == 0) & (pol["egress"] == egr)]
        for lxc, pol in t.policy.items() if mode == MODE_INGRESS or lxc == S.EP_LXC_ID]))
    okp = np.flatnonzero(np.isin(fam_ipc["label"], allow))
    addr_in = S._addr_in_prefix_v4 if family == 4 else S._addr_in_prefix_v6

    def allowed_peers(k):
        return addr_in(rng, fam_ipc, okp[rng.integers(0, len(okp), size=k)])
    # established flows: runs of packets, some closing, a packet after the close
    live = np.flatnonzero(est_ok)
    est = S.take(fwd, live[rng.integers(0, len(live), size=m)])
    steps(est, [(1.0, lambda h: tcpf(h, rng.choice([0x10, 0x18], size=len(h)))),
                (0.7, lambda h: tcpf(h, 0x18)),
                (0.5, lambda h: tcpf(h, 0x10)),
                (0.2, lambda h: tcpf(h, rng.choice([0x11, 0x04], size=len(h)), close=True)),
                (0.15, lambda h: tcpf(h, 0x10))])
    if len(rep):
        r = S.reverse(S.take(rep, rng.integers(0, len(rep), size=m // 2)))
        steps(r, [(1.0, lambda h: tcpf(h, 0x10)), (0.6, lambda h: tcpf(h, 0x18)),
                  (0.3, lambda h: tcpf(h, 0x10))])
        steps(S.take(rep, rng.integers(0, len(rep), size=m // 6)),
              [(1.0, icmp_err)])
    # new flows into the endpoints (ingress) / out of EP_LXC_ID (egress)
    if mode == MODE_INGRESS:
        d = gen(rng, m, fam_ipc, loc, local_frac=0.95, mark_host=0, mark_proxy=0,
                other_proto=0, **kw)
    else:
        d = gen(rng, m, fam_ipc, loc, local_frac=0.3, mark_host=0, mark_proxy=0,
                other_proto=0, src_fixed=ep_addr, **kw)
        sel = rng.random(len(d)) < 0.7
        d.daddr[sel] = dst[rng.integers(0, len(dst), size=int(sel.sum()))]
    ok = rng.random(len(d)) < 0.8
    if mode == MODE_INGRESS:
        d.saddr[ok] = allowed_peers(int(ok.sum()))
    else:
        d.daddr[ok] = allowed_peers(int(ok.sum()))
    d = fix_icmp(d)
    steps(d, [(1.0, lambda h: tcpf(h, 0x02)), (0.8, lambda h: tcpf(h, 0x10)),
              (0.3, icmp_same),
              (0.5, lambda h: tcpf(h, 0x18)),
              (0.25, lambda h: tcpf(h, rng.choice([0x11, 0x04], size=len(h)), close=True)),
              (0.15, lambda h: tcpf(h, 0x10))])
    # new flows between the two local endpoints: both directions pass a CT
    # lookup (ingress: each end's policy program; egress: the sender's and,
    # on local delivery, the destination's), so replies and related ICMP
    # errors of a flow the stream itself opens are in the batch
    k2 = m // 2
    a = gen(rng, k2, fam_ipc, loc[:2], local_frac=1.0, mark_host=0, mark_proxy=0,
            other_proto=0, **kw)
    if mode == MODE_INGRESS:
        if family == 4:
            a.saddr[:] = np.where(a.daddr == loc[0], loc[1], loc[0])
        else:
            isl0 = (a.daddr == loc[0]).all(1)
            a.saddr[:] = np.where(isl0[:, None], loc[1], loc[0])
        script = [(1.0, lambda h: tcpf(h, 0x02)),
                  (0.7, lambda h: tcpf(S.reverse(h), 0x12)),
                  (0.3, icmp_err),
                  (0.7, lambda h: tcpf(copy(h), 0x10)),
                  (0.5, lambda h: tcpf(S.reverse(h), 0x18)),
                  (0.2, lambda h: tcpf(copy(h), rng.choice([0x11, 0x04], size=len(h)),
                                       close=True)),
                  (0.2, lambda h: tcpf(S.reverse(h), 0x10))]
    else:   # (the replies leave the other endpoint: not this program's)
        a.saddr[:] = ep_addr
        a.daddr[:] = loc[1] if len(loc) > 1 else loc[0]
        script = [(1.0, lambda h: tcpf(h, 0x02)), (0.7, lambda h: tcpf(copy(h), 0x10)),
                  (0.5, lambda h: tcpf(copy(h), 0x18)),
                  (0.2, lambda h: tcpf(copy(h), rng.choice([0x11, 0x04], size=len(h)),
                                       close=True)),
                  (0.2, lambda h: tcpf(copy(h), 0x10))]
    a = fix_icmp(a)
    steps(a, script)
    # established flows the policy change denies: their first packet deletes
    # the entry (ct_delete), the later ones find none
    den = np.flatnonzero(denied)
    if len(den):
        dn = S.take(fwd, den[rng.integers(0, len(den), size=m // 2)])
        steps(dn, [(1.0, lambda h: tcpf(h, 0x10)), (0.8, lambda h: tcpf(h, 0x18)),
                   (0.5, lambda h: tcpf(h, 0x10)), (0.3, lambda h: tcpf(h, 0x02))])
    h = S.concat(parts)
    h = S.take(h, np.argsort(np.concatenate(pos), kind="stable"))
    ep = S.EP_LXC_ID if mode == MODE_EGRESS else 0
    return t, h.slice(0, n), mode, ep or None, dp


# ------------------------------------------------------------ load balancing
def _lb_setup(seed):
    """C2-shaped small tables (two endpoints with programs) plus services
    (synth.lb4_services); the sending endpoint's egress policy allows most
    backend identities, the other endpoint admits the sender."""
    t = S.config_c2(seed, n_prefixes=2000, n_policy=400, n_endpoints=2)
    rng = np.random.default_rng(seed + 1)
    t.lb4, t.revnat4, vips, ports, protos = S.lb4_services(rng, t)
    ipc = t.ipcache[t.ipcache["family"] == 1]
    idents = np.unique(ipc["label"])
    allow = rng.choice(idents, size=int(0.8 * len(idents)), replace=False)
    for lxc, pol in t.policy.items():
        one = np.zeros(len(allow) + 4, S.POLICY_DT)
        one["identity"][:len(allow)] = allow
        one["identity"][len(allow):] = [S.WORLD_ID, S.CLUSTER_ID, S.HOST_ID,
                                       S.EP_SECLABEL]
        add = np.concatenate([one, one])
        add["egress"][len(one):] = 1
        # the sender's own ingress: half the identities (a looped-back flow
        # is checked against it, with src = its own SECLABEL)
        add = add[(add["egress"] == 1) | (np.arange(len(add)) % 2 == 0)]
        have = {(int(r["identity"]), int(r["dport"]), int(r["proto"]),
                 int(r["egress"])) for r in pol}
        add = add[[(int(r["identity"]), 0, 0, int(r["egress"])) not in have
                   for r in add]]
        t.policy[lxc] = np.concatenate([pol, add])
    return t, rng, vips, ports, protos


def _svc_flows(rng, n, vips, ports, protos, sport_base):
    """n new flows from the endpoint to service VIPs (unique source ports):
    80% on the service's port and protocol, 10% another port (the L3
    fall-back key), 10% ICMP echo"""
    k = rng.integers(0, len(vips), size=n)
    h = S.Headers(4, np.full(n, S.LXC_IPV4, np.uint32), vips[k].copy(),
                  S.htons(sport_base + np.arange(n)), ports[k].copy(),
                  protos[k].copy(), np.zeros(n, np.uint8),
                  rng.integers(60, 1500, size=n).astype(np.uint16),
                  np.zeros(n, np.uint32))
    z = h.dport == 0
    h.dport[z] = S.htons(rng.choice(np.array([80, 8443, 22]), size=int(z.sum())))
    r = rng.random(n)
    other = r < 0.1
    h.dport[other] = S.htons(rng.integers(1, 65536, size=int(other.sum())))
    icmp = r > 0.9
    h.proto[icmp] = S.IPPROTO_ICMP
    h.sport[icmp] = 8          # echo request: type 8, code 0
    h.dport[icmp] = 0
    return h


def sc_lb_egress(n=5000, seed=41):
    """Service load balancing in the sending endpoint's egress program
    (bpf_lxc.c:476-576, lb.h): a history stream opens service flows (the
    reference's CT_SERVICE and reverse-NAT entries), then the test stream:
    established service flows, new ones, replies of a flow the service
    looped back into the endpoint itself (lb4_rev_nat with lb_loopback),
    and plain traffic.  skb->hash is the reference's (from its records)."""
    import oracle as O
    t, rng, vips, ports, protos = _lb_setup(seed)
    hist = _svc_flows(rng, 1200, vips, ports, protos, 20000)
    plain = S.gen_headers_v4(rng, 300, t.ipcache[t.ipcache["family"] == 1],
                             S.local_v4_addrs(t), local_frac=0.3, mark_host=0,
                             mark_proxy=0, src_fixed=S.LXC_IPV4, frag=0)
    hist = S.concat([hist, plain])
    dp = RefDatapath(t)
    hres = run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    # test stream
    parts = []
    est = S.take(hist, rng.integers(0, 1200, size=int(n * 0.45)))
    est.flags[(rng.random(len(est)) < 0.05) & (est.proto == S.IPPROTO_TCP)] |= \
        np.uint8(S.HF_TCP_CLOSE)
    parts.append(est)
    # new service flows, several packets each (the first creates the
    # CT_SERVICE entry and the flow's entry, the later ones find them)
    new = _svc_flows(rng, int(n * 0.12), vips, ports, protos, 40000)
    parts.append(S.take(new, rng.integers(0, len(new), size=int(n * 0.35))))
    # the looped-back flows: the endpoint, as the backend, answers the
    # client address it saw (IPV4_LOOPBACK) from its translated port
    pk = hres[8]
    lb = (pk[:, 0] == S.IPV4_LOOPBACK) & (hres[0] != 2)
    if lb.any():
        src = S.take(hist, np.flatnonzero(lb))
        pr = pk[lb]
        m = max(1, int(n * 0.05))
        pick = rng.integers(0, len(src), size=m)
        rep = S.Headers(4, np.full(m, S.LXC_IPV4, np.uint32),
                        np.full(m, S.IPV4_LOOPBACK, np.uint32),
                        (pr[pick, 2] >> 16).astype(np.uint16),
                        (pr[pick, 2] & 0xFFFF).astype(np.uint16),
                        src.proto[pick].copy(), np.zeros(m, np.uint8),
                        src.length[pick].copy(), np.zeros(m, np.uint32))
        parts.append(rep)
    parts.append(S.gen_headers_v4(rng, int(n * 0.15), t.ipcache[t.ipcache["family"] == 1],
                                  S.local_v4_addrs(t), local_frac=0.3, mark_host=0,
                                  mark_proxy=0, src_fixed=S.LXC_IPV4, frag=0))
    h = S.concat(parts)
    h = S.take(h, rng.permutation(len(h)))
    h.hash = None
    # (every intra-batch CT dependency kept: the reference runs the stream
    # packet by packet and the fixture is its result)
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


def sc_lb_reply(n=4000, seed=43):
    """Replies of load-balanced flows arriving from the backends (from-netdev,
    then the client endpoint's ipv4_policy): CT_REPLY on the entries the
    egress path created, source translated back to the service address
    (lb4_rev_nat, bpf_lxc.c:946-955); plus new inbound traffic."""
    t, rng, vips, ports, protos = _lb_setup(seed)
    hist = _svc_flows(rng, 1500, vips, ports, protos, 20000)
    dp = RefDatapath(t)
    hres = run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    pk = hres[8]
    fw = (hres[0] != 2) & (pk[:, 0] == S.LXC_IPV4) & (hist.proto != S.IPPROTO_ICMP)
    idx = np.flatnonzero(fw)
    m = int(n * 0.7)
    pick = idx[rng.integers(0, len(idx), size=m)]
    rep = S.Headers(4, pk[pick, 1].copy(), pk[pick, 0].copy(),
                    (pk[pick, 2] >> 16).astype(np.uint16),
                    (pk[pick, 2] & 0xFFFF).astype(np.uint16),
                    hist.proto[pick].copy(), np.zeros(m, np.uint8),
                    rng.integers(60, 1500, size=m).astype(np.uint16),
                    np.zeros(m, np.uint32))
    rep.flags[(rng.random(m) < 0.05) & (rep.proto == S.IPPROTO_TCP)] |= np.uint8(S.HF_TCP_CLOSE)
    new = S.gen_headers_v4(rng, (n - m) // 3, t.ipcache[t.ipcache["family"] == 1],
                           S.local_v4_addrs(t)[:1], local_frac=1.0, mark_host=0,
                           mark_proxy=0, frag=0)
    new = S.take(new, rng.integers(0, len(new), size=n - m))   # several packets a flow
    h = S.concat([rep, new])
    h = S.take(h, rng.permutation(len(h)))
    return t, h, MODE_INGRESS, None, dp


def _keep(h, m):
    return S.take(h, m)


# ------------------------------------------------------------ IPv6 services
def _lb_setup6(seed):
    """C3-shaped small tables (two dual-stack endpoints with programs) plus
    IPv6 services (synth.lb6_services); the sending endpoint's egress policy
    allows most backend identities, both endpoints' ingress half of them and
    the sender."""
    t = S.config_c3(seed, n_prefixes=2000, n_v4_prefixes=100, n_policy=400,
                    n_endpoints=2, n_prefilter=0)
    rng = np.random.default_rng(seed + 1)
    t.lb6, t.revnat6, vips, ports, protos = S.lb6_services(rng, t)
    ipc = t.ipcache[t.ipcache["family"] == 2]
    idents = np.unique(ipc["label"])
    allow = rng.choice(idents, size=int(0.8 * len(idents)), replace=False)
    for lxc, pol in t.policy.items():
        one = np.zeros(len(allow) + 4, S.POLICY_DT)
        one["identity"][:len(allow)] = allow
        one["identity"][len(allow):] = [S.WORLD_ID, S.CLUSTER_ID, S.HOST_ID,
                                       S.EP_SECLABEL]
        add = np.concatenate([one, one])
        add["egress"][len(one):] = 1
        add = add[(add["egress"] == 1) | (np.arange(len(add)) % 2 == 0)]
        have = {(int(r["identity"]), int(r["dport"]), int(r["proto"]),
                 int(r["egress"])) for r in pol}
        add = add[[(int(r["identity"]), 0, 0, int(r["egress"])) not in have
                   for r in add]]
        t.policy[lxc] = np.concatenate([pol, add])
    return t, rng, vips, ports, protos


def _svc_flows6(rng, n, vips, ports, protos, sport_base):
    """n new IPv6 flows from the endpoint to service VIPs: 80% on the
    service's port and protocol, 10% another port (the L3 fall-back key),
    10% ICMPv6 echo"""
    k = rng.integers(0, len(vips), size=n)
    h = S.Headers(6, np.tile(S.LXC_IPV6, (n, 1)), vips[k].copy(),
                  S.htons(sport_base + np.arange(n)), ports[k].copy(),
                  protos[k].copy(), np.zeros(n, np.uint8),
                  rng.integers(100, 1500, size=n).astype(np.uint16),
                  np.zeros(n, np.uint32))
    z = h.dport == 0
    h.dport[z] = S.htons(rng.choice(np.array([80, 8443, 22]), size=int(z.sum())))
    r = rng.random(n)
    other = r < 0.1
    h.dport[other] = S.htons(rng.integers(1, 65536, size=int(other.sum())))
    icmp = r > 0.9
    h.proto[icmp] = S.IPPROTO_ICMPV6
    h.sport[icmp] = 128        # echo request: type 128, code 0
    h.dport[icmp] = 0
    return h


def _no_hazard(t, h, mode, ep):
    import oracle as O
    for _ in range(6):
        o = O.Oracle(t)
        oa, ov, oi, ct = o.classify(h, mode, ep or 0, want_ct=True)
        hz = o.ct_apply(h, mode, ep or 0, oi, ov, ct, hazard=True)
        if not hz.any():
            break
        h = _keep(h, hz == 0)
    assert not hz.any()
    return h


def sc_lb_egress_v6(n=4000, seed=51):
    """IPv6 service load balancing in the sending endpoint's egress program
    (ipv6_l3_from_lxc, bpf_lxc.c:149-167, 255-266; lb.h:336-481): a history
    stream opens service flows (CT_SERVICE entries, the flows' entries with
    rev_nat_index and slave), then the test stream: established service
    flows, new ones, a service whose backend is the sender itself, and plain
    traffic.  skb->hash is the reference's (from its records)."""
    t, rng, vips, ports, protos = _lb_setup6(seed)
    hist = _svc_flows6(rng, 1000, vips, ports, protos, 20000)
    plain = S.gen_headers_v6(rng, 300, t.ipcache[t.ipcache["family"] == 2],
                             S.local_v6_addrs(t), local_frac=0.3, mark_host=0,
                             mark_proxy=0, src_fixed=S.LXC_IPV6, ext=0,
                             exthdr_drop=0)
    hist = S.concat([hist, plain])
    dp = RefDatapath(t)
    run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    # inbound flows to the endpoint (ipv6_policy's entries carry the
    # endpoint address's rev_nat_index): the test stream's egress replies
    # to them are reverse-NATed (bpf_lxc.c:255-266)
    inb = S.gen_headers_v6(rng, 400, t.ipcache[t.ipcache["family"] == 2],
                           S.local_v6_addrs(t)[:1], local_frac=1.0, mark_host=0,
                           mark_proxy=0, ext=0, exthdr_drop=0)
    inb.proto[:] = np.where(rng.random(len(inb)) < 0.6, S.IPPROTO_TCP, S.IPPROTO_UDP)
    ires = run(dp, inb, MODE_INGRESS)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    fw_in = np.flatnonzero(ires[0] != 2)
    replies = S.reverse(S.take(inb, fw_in[rng.integers(0, len(fw_in), size=int(n * 0.1))]))
    est = S.take(hist, rng.integers(0, 1000, size=int(n * 0.4)))
    est.flags[(rng.random(len(est)) < 0.05) & (est.proto == S.IPPROTO_TCP)] |= \
        np.uint8(S.HF_TCP_CLOSE)
    new = _svc_flows6(rng, int(n * 0.12), vips, ports, protos, 40000)
    parts = [est, replies, S.take(new, rng.integers(0, len(new), size=int(n * 0.35))),
             S.gen_headers_v6(rng, int(n * 0.15), t.ipcache[t.ipcache["family"] == 2],
                              S.local_v6_addrs(t), local_frac=0.3, mark_host=0,
                              mark_proxy=0, src_fixed=S.LXC_IPV6, ext=0,
                              exthdr_drop=0)]
    h = S.concat(parts)
    h = S.take(h, rng.permutation(len(h)))
    h.hash = None
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


def sc_lb_reply_v6(n=3000, seed=53):
    """Replies of load-balanced IPv6 flows from the backends (from-netdev,
    then the client endpoint's ipv6_policy): CT_REPLY on the entries the
    egress path created and lb6_rev_nat of every hit carrying a
    rev_nat_index (bpf_lxc.c:808-815); plus new inbound traffic."""
    t, rng, vips, ports, protos = _lb_setup6(seed)
    hist = _svc_flows6(rng, 1200, vips, ports, protos, 20000)
    dp = RefDatapath(t)
    hres = run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    pk = hres[8]
    src = np.ascontiguousarray(pk[:, 0:4]).view(np.uint8).reshape(-1, 16)
    dst = np.ascontiguousarray(pk[:, 4:8]).view(np.uint8).reshape(-1, 16)
    fw = (hres[0] != 2) & (src == S.LXC_IPV6).all(1) & (hist.proto != S.IPPROTO_ICMPV6)
    idx = np.flatnonzero(fw)
    m = int(n * 0.7)
    pick = idx[rng.integers(0, len(idx), size=m)]
    rep = S.Headers(6, dst[pick].copy(), src[pick].copy(),
                    (pk[pick, 8] >> 16).astype(np.uint16),
                    (pk[pick, 8] & 0xFFFF).astype(np.uint16),
                    hist.proto[pick].copy(), np.zeros(m, np.uint8),
                    rng.integers(100, 1500, size=m).astype(np.uint16),
                    np.zeros(m, np.uint32))
    rep.flags[(rng.random(m) < 0.05) & (rep.proto == S.IPPROTO_TCP)] |= np.uint8(S.HF_TCP_CLOSE)
    # new inbound flows to the endpoint, several packets each: the later
    # packets hit the entry the first one created, whose rev_nat_index
    # ipv6_policy took from the daddr (bpf_lxc.c:787-788), and are
    # reverse-NATed by it (:808-815)
    new = S.gen_headers_v6(rng, (n - m) // 3, t.ipcache[t.ipcache["family"] == 2],
                           S.local_v6_addrs(t)[:1], local_frac=1.0, mark_host=0,
                           mark_proxy=0, ext=0, exthdr_drop=0)
    new = S.take(new, rng.integers(0, len(new), size=n - m))
    h = S.concat([rep, new])
    h = S.take(h, rng.permutation(len(h)))
    return t, h, MODE_INGRESS, None, dp


# ------------------------------------------------------------ NAT46 / NAT64
def _nat_setup(seed):
    """Dual-stack small tables for LXC_NAT46 (lxc_config.h:28): IPv4 peers
    reached from the endpoint's IPv6 side through ::ffff:0:0/96.  EP_LXC_ID's
    egress policy admits WORLD (the IPv6 stage: a v4-mapped peer has no
    IPv6 ipcache entry) and most IPv4 identities (the IPv4 stage after the
    translation); its ingress policy admits some IPv4 identities (the
    replies, translated back, are checked by ipv6_policy with the IPv4
    source's identity).  ::ffff:10.0.0.0/104 is in the ipcache as
    CLUSTER_ID: those destinations are not translated (bpf_lxc.c:353-354)."""
    t = S.config_c3(seed, n_prefixes=2000, n_v4_prefixes=500, n_policy=300,
                    n_endpoints=2, n_prefilter=0)
    rng = np.random.default_rng(seed + 1)
    cl = np.zeros(1, S.IPCACHE_DT)
    cl["family"] = 2
    cl["plen"] = 104
    cl["addr"][0, 10:13] = [0xff, 0xff, 10]
    cl["label"] = S.CLUSTER_ID
    t.ipcache = np.concatenate([t.ipcache, cl])
    ipc4 = t.ipcache[t.ipcache["family"] == 1]
    ids4 = np.unique(ipc4["label"])
    out_ok = rng.choice(ids4, size=int(0.7 * len(ids4)), replace=False)
    in_ok = rng.choice(ids4, size=int(0.5 * len(ids4)), replace=False)
    pol = t.policy[S.EP_LXC_ID]
    add = np.zeros(1 + len(out_ok) + len(in_ok), S.POLICY_DT)
    add["identity"][0] = S.WORLD_ID
    add["egress"][0] = 1
    add["identity"][1:1 + len(out_ok)] = out_ok
    add["egress"][1:1 + len(out_ok)] = 1
    add["identity"][1 + len(out_ok):] = in_ok
    have = {(int(r["identity"]), int(r["dport"]), int(r["proto"]), int(r["egress"]))
            for r in pol}
    add = add[[(int(r["identity"]), 0, 0, int(r["egress"])) not in have for r in add]]
    t.policy[S.EP_LXC_ID] = np.concatenate([pol, add])
    return t, rng, ipc4


def _mapped(v4):
    """::ffff:a.b.c.d of raw be32 IPv4 addresses"""
    a = np.zeros((len(v4), 16), np.uint8)
    a[:, 10:12] = 0xff
    a[:, 12:16] = np.asarray(v4, np.uint32).view(np.uint8).reshape(-1, 4)
    return a


def _nat64_flows(rng, ipc4, n, sport_base):
    """n new IPv6 flows from the endpoint to v4-mapped peers inside IPv4
    ipcache prefixes: TCP 60%, UDP 25%, ICMPv6 echo 15%"""
    peers = S._addr_in_prefix_v4(rng, ipc4, rng.integers(0, len(ipc4), size=n))
    r = rng.random(n)
    proto = np.where(r < 0.6, S.IPPROTO_TCP,
                     np.where(r < 0.85, S.IPPROTO_UDP, S.IPPROTO_ICMPV6)).astype(np.uint8)
    h = S.Headers(6, np.tile(S.LXC_IPV6, (n, 1)), _mapped(peers),
                  S.htons(sport_base + np.arange(n)),
                  S.htons(rng.choice(np.array([80, 443, 53, 8080]), size=n)),
                  proto, np.zeros(n, np.uint8),
                  rng.integers(100, 1500, size=n).astype(np.uint16), np.zeros(n, np.uint32))
    ic = proto == S.IPPROTO_ICMPV6
    h.sport[ic] = 128      # echo request
    h.dport[ic] = S.htons(np.arange(int(ic.sum())) + 1).astype(np.uint16)
    h.tcpflags = np.where(proto == S.IPPROTO_TCP, 0x02, 0).astype(np.uint8)
    return h


def sc_nat46_egress_v6(n=3000, seed=61):
    """NAT64 in the endpoint's IPv6 egress (bpf_lxc.c:353-360,
    tail_ipv6_to_ipv4 :1070-1083, nat46.h:336-420): packets to v4-mapped
    peers outside the cluster leave through the IPv4 egress program,
    translated (saddr LXC_IPV4, daddr the low 32 bits, ICMPv6 as ICMP) — its
    CT entries carry nat46 (conntrack.h:714-716).  A history stream opens
    flows; the test stream: their later packets (ESTABLISHED in both maps),
    new flows with several packets, ICMPv6 errors of every translation
    outcome (FRAG_NEEDED fall-through, unknown codes and types),
    extension-header packets (DROP_INVALID_EXTHDR), CLUSTER-mapped peers
    (not translated) and plain IPv6 traffic."""
    t, rng, ipc4 = _nat_setup(seed)
    hist = _nat64_flows(rng, ipc4, 800, 20000)
    dp = RefDatapath(t)
    run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    parts, pos = [], []

    def add(h, p):
        parts.append(h)
        pos.append(p)
    est = S.take(hist, rng.integers(0, len(hist), size=int(n * 0.35)))
    est.tcpflags = np.where(est.proto == S.IPPROTO_TCP,
                            rng.choice(np.array([0x10, 0x18], np.uint8), size=len(est)), 0
                            ).astype(np.uint8)
    est.length = rng.integers(100, 1500, size=len(est)).astype(np.uint16)
    add(est, rng.random(len(est)))
    new = _nat64_flows(rng, ipc4, int(n * 0.12), 40000)
    at = rng.random(len(new)) * 0.9
    add(new, at)
    for f, p_ in ((0x10, 0.8), (0x18, 0.5)):
        sel = np.flatnonzero(rng.random(len(new)) < p_)
        h = S.take(new, sel)
        h.tcpflags = np.where(h.proto == S.IPPROTO_TCP, f, 0).astype(np.uint8)
        at = at + rng.random(len(new)) * 0.03
        add(h, at[sel])
    # ICMPv6 errors to mapped peers: each type/code outcome of icmp6_to_icmp4
    k = int(n * 0.08)
    e = _nat64_flows(rng, ipc4, k, 50000)
    tc = np.array([[1, 0], [1, 3], [1, 4], [1, 1], [1, 7], [2, 0], [3, 0], [3, 1],
                   [4, 0], [4, 1], [4, 2], [137, 0]], np.uint16)
    pick = tc[rng.integers(0, len(tc), size=k)]
    e.proto[:] = S.IPPROTO_ICMPV6
    e.sport[:] = (pick[:, 0] | pick[:, 1] << 8).astype(np.uint16)
    e.dport[:] = 0
    e.tcpflags = np.zeros(k, np.uint8)
    add(e, rng.random(k))
    # extension headers before the L4 header: ipv6_to_ipv4 drops them
    x = _nat64_flows(rng, ipc4, int(n * 0.03), 60000)
    x.flags[:] |= np.uint8(S.HF_EXTHDR)
    add(x, rng.random(len(x)))
    # CLUSTER-mapped peers (::ffff:10.x.y.z): to the stack untranslated
    c = _nat64_flows(rng, ipc4, int(n * 0.04), 61000)
    c.daddr[:, 12] = 10
    add(c, rng.random(len(c)))
    plain = S.gen_headers_v6(rng, int(n * 0.1), t.ipcache[t.ipcache["family"] == 2],
                             S.local_v6_addrs(t), local_frac=0.3, mark_host=0,
                             mark_proxy=0, src_fixed=S.LXC_IPV6, ext=0, exthdr_drop=0)
    add(plain, rng.random(len(plain)))
    h = S.concat(parts)
    h = S.take(h, np.argsort(np.concatenate(pos), kind="stable"))
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


def sc_nat64_lb_v6(n=2400, seed=67, loopback=False):
    """Load-balanced NAT64 hops (an oracle-only fixture, tests/golden_oracle:
    the engine was not run against it): IPv6 packets to v4-mapped IPv4
    service VIPs leave through the IPv4 egress program (bpf_lxc.c:353-360 ->
    tail_ipv6_to_ipv4 :1070-1083), whose service step (lb4_local,
    :476-492) selects a backend, creates the CT_SERVICE entry and translates
    the destination before ct_create4 writes the flow's entry (with nat46).
    A history opens service flows; the test stream: their later packets, new
    service flows of several packets, and plain NAT64 flows beside them."""
    t, rng, ipc4 = _nat_setup(seed)
    t.lb4, t.revnat4, vips, ports, protos = S.lb4_services(rng, t, loopback=loopback)
    if loopback:
        # (loopback: a service whose backend is the endpoint itself — lb4_local
        # SNATs to IPV4_LOOPBACK and the endpoint's ingress admits its own
        # identity on the services' ports)
        pol = t.policy[S.EP_LXC_ID]
        add = np.zeros(len(ports), S.POLICY_DT)
        add["identity"] = int(t.seclabel[S.EP_LXC_ID])
        add["dport"] = ports
        add["proto"] = protos
        t.policy[S.EP_LXC_ID] = np.concatenate([pol, add])

    # (not the service whose backend slot lives only under the L3 key: every
    # packet of its flows re-selects from its own skb->hash, which the
    # reference's records do not carry for an untraced packet)
    pick = np.flatnonzero(np.arange(len(vips)) != 5)

    def svc64(k, base):
        kk = pick[rng.integers(0, len(pick), size=k)]
        h = _nat64_flows(rng, ipc4, k, base)
        h.daddr = _mapped(vips[kk])
        l4 = h.proto != S.IPPROTO_ICMPV6
        h.proto[l4] = protos[kk][l4]
        m = l4 & (ports[kk] != 0)
        h.dport[m] = ports[kk][m]
        h.tcpflags = np.where(h.proto == S.IPPROTO_TCP, 0x02, 0).astype(np.uint8)
        return h
    hist = S.concat([svc64(600, 20000), _nat64_flows(rng, ipc4, 200, 30000)])
    dp = RefDatapath(t)
    run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    parts, pos = [], []

    def add(h, p):
        parts.append(h)
        pos.append(p)
    est = S.take(hist, rng.integers(0, len(hist), size=int(n * 0.4)))
    est.tcpflags = np.where(est.proto == S.IPPROTO_TCP,
                            rng.choice(np.array([0x10, 0x18], np.uint8), size=len(est)), 0
                            ).astype(np.uint8)
    add(est, rng.random(len(est)))
    new = svc64(int(n * 0.15), 40000)
    at = rng.random(len(new)) * 0.9
    add(new, at)
    for f, p_ in ((0x10, 0.8), (0x18, 0.5)):
        sel = np.flatnonzero(rng.random(len(new)) < p_)
        h = S.take(new, sel)
        h.tcpflags = np.where(h.proto == S.IPPROTO_TCP, f, 0).astype(np.uint8)
        at = at + rng.random(len(new)) * 0.03
        add(h, at[sel])
    far = _nat64_flows(rng, ipc4, int(n * 0.1), 50000)
    add(far, rng.random(len(far)))
    h = S.concat(parts)
    h = S.take(h, np.argsort(np.concatenate(pos), kind="stable"))
    h.hash = None
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


def sc_nat46_reply_v4(n=3000, seed=63):
    """NAT46 in ipv4_policy (bpf_lxc.c:939-944, tail_ipv4_to_ipv6
    :1098-1110, nat46.h:236-328): IPv4 replies from the peers of NAT64'd
    flows find their nat46 CT entry (conntrack.h:241-244) and are checked
    by ipv6_policy translated (saddr NAT46_PREFIX + the IPv4 source, daddr
    LXC_IP, ICMP as ICMPv6), with the IPv4 source's identity; ICMP errors
    related to those flows, new IPv4 traffic, and replies of ordinary
    flows."""
    t, rng, ipc4 = _nat_setup(seed)
    hist = _nat64_flows(rng, ipc4, 1000, 20000)
    dp = RefDatapath(t)
    hres = run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    ok = np.flatnonzero(hres[0] != 2)
    m = int(n * 0.6)
    pick = ok[rng.integers(0, len(ok), size=m)]
    src = S.take(hist, pick)
    peer = np.ascontiguousarray(src.daddr[:, 12:16]).view("<u4").ravel()
    icmp = src.proto == S.IPPROTO_ICMPV6
    rep = S.Headers(4, peer.copy(), np.full(m, S.LXC_IPV4, np.uint32),
                    np.where(icmp, 0, src.dport).astype(np.uint16),
                    np.where(icmp, src.dport, src.sport).astype(np.uint16),
                    np.where(icmp, S.IPPROTO_ICMP, src.proto).astype(np.uint8),
                    np.zeros(m, np.uint8), rng.integers(60, 1500, size=m).astype(np.uint16),
                    np.zeros(m, np.uint32))
    rep.tcpflags = np.where(rep.proto == S.IPPROTO_TCP,
                            rng.choice(np.array([0x12, 0x10, 0x18], np.uint8), size=m), 0
                            ).astype(np.uint8)
    # ICMP errors about those flows from their peers: every translation case
    k = int(n * 0.12)
    ep_ = S.take(rep, rng.integers(0, m, size=k))
    tc = np.array([[3, 0], [3, 1], [3, 2], [3, 3], [3, 4], [3, 5], [3, 9], [3, 13],
                   [3, 14], [11, 0], [12, 0], [5, 0]], np.uint16)
    pick2 = tc[rng.integers(0, len(tc), size=k)]
    ep_.proto[:] = S.IPPROTO_ICMP
    ep_.sport[:] = (pick2[:, 0] | pick2[:, 1] << 8).astype(np.uint16)
    ep_.dport[:] = 0
    ep_.tcpflags = np.zeros(k, np.uint8)
    new = S.gen_headers_v4(rng, n - m - k, ipc4, S.local_v4_addrs(t)[:1], local_frac=1.0,
                           mark_host=0, mark_proxy=0, frag=0)
    h = S.concat([rep, ep_, new])
    h = S.take(h, rng.permutation(len(h)))
    return t, h, MODE_INGRESS, None, dp


def sc_nat64_local_v6(n=2400, seed=65):
    """NAT64 to a local endpoint: the translated packet's IPv4 destination
    is an endpoint of this node, so handle_ipv4_from_lxc delivers it
    locally (ipv4_local_delivery, l3.h:103-131) and the destination's
    ipv4_policy runs its own ct_lookup4 / ct_create4 — a third CT stage
    after the IPv6 and the IPv4 egress lookups (its entries without nat46:
    conntrack.h:714-716 sets it for CT_EGRESS only).  A history stream
    opens flows; the test stream: their later packets, new flows of several
    packets (SYN, ACK, data), and NAT64 flows to remote peers beside them."""
    t, rng, ipc4 = _nat_setup(seed)
    loc = S.local_v4_addrs(t)
    # the sender may reach any identity on the flows' ports (identity 0:
    # the wildcard entry, policy.h:93-101); each endpoint admits the
    # sender's SECLABEL on some of them only
    pol = t.policy[S.EP_LXC_ID]
    add = np.zeros(3, S.POLICY_DT)
    add["dport"] = S.htons(np.array([80, 53, 443]))
    add["proto"] = [S.IPPROTO_TCP, S.IPPROTO_UDP, S.IPPROTO_TCP]
    add["egress"] = 1
    t.policy[S.EP_LXC_ID] = np.concatenate([pol, add])
    sec = int(t.seclabel[S.EP_LXC_ID])
    for lxc in np.unique(t.endpoints["lxc_id"]):
        p_ = t.policy.get(int(lxc))
        if p_ is None:
            continue
        ing = np.zeros(3, S.POLICY_DT)
        ing["identity"] = sec
        ing["dport"] = S.htons(np.array([80, 53, 8080]))
        ing["proto"] = [S.IPPROTO_TCP, S.IPPROTO_UDP, S.IPPROTO_TCP]
        t.policy[int(lxc)] = np.concatenate([p_, ing])

    def flows(k, base, local=True):
        h = _nat64_flows(rng, ipc4, k, base)
        if local:
            h.daddr = _mapped(rng.choice(loc, size=k))
        return h
    hist = flows(300, 20000)
    dp = RefDatapath(t)
    run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    parts, pos = [], []

    def add_(h, p):
        parts.append(h)
        pos.append(p)
    est = S.take(hist, rng.integers(0, len(hist), size=int(n * 0.3)))
    est.tcpflags = np.where(est.proto == S.IPPROTO_TCP,
                            rng.choice(np.array([0x10, 0x18], np.uint8), size=len(est)), 0
                            ).astype(np.uint8)
    est.length = rng.integers(100, 1500, size=len(est)).astype(np.uint16)
    add_(est, rng.random(len(est)))
    new = flows(int(n * 0.2), 40000)
    at = rng.random(len(new)) * 0.9
    add_(new, at)
    for f, p_ in ((0x10, 0.8), (0x18, 0.6)):
        sel = np.flatnonzero(rng.random(len(new)) < p_)
        h = S.take(new, sel)
        h.tcpflags = np.where(h.proto == S.IPPROTO_TCP, f, 0).astype(np.uint8)
        at = at + rng.random(len(new)) * 0.03
        add_(h, at[sel])
    far = flows(int(n * 0.15), 50000, local=False)
    add_(far, rng.random(len(far)))
    h = S.concat(parts)
    h = S.take(h, np.argsort(np.concatenate(pos), kind="stable"))
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


def sc_nat46_self_v4(n=1600, seed=69):
    """NAT46 behind an IPv4 egress batch's local delivery (an oracle-only
    fixture, tests/golden_oracle: the engine was not run against it): the
    endpoint's NAT64 flows to its own IPv4 address (::ffff:LXC_IPV4,
    delivered to itself by the IPv4 egress program) are answered by IPv4
    packets LXC_IPV4 -> LXC_IPV4; the egress program delivers them locally
    (ipv4_local_delivery, l3.h:103-131), the destination's ipv4_policy finds
    the flow's nat46 entry (conntrack.h:241-244) and tail_ipv4_to_ipv6
    (bpf_lxc.c:939-944, :1098-1110) hands the translated packet to
    ipv6_policy, whose ct_lookup6 / ct_create6 is a third CT stage.  The
    test stream: replies of several packets per flow and plain IPv4 egress
    traffic beside them."""
    t, rng, ipc4 = _nat_setup(seed)
    a4 = np.uint32(S.LXC_IPV4)
    sec = int(t.seclabel[S.EP_LXC_ID])
    # the endpoint admits its own identity on the flows' ports (ingress)
    pol = t.policy[S.EP_LXC_ID]
    add = np.zeros(4, S.POLICY_DT)
    add["identity"] = sec
    add["dport"] = S.htons(np.array([80, 53, 443, 0]))
    add["proto"] = [S.IPPROTO_TCP, S.IPPROTO_UDP, S.IPPROTO_TCP, 0]
    t.policy[S.EP_LXC_ID] = np.concatenate([pol, add])
    hist = _nat64_flows(rng, ipc4, 500, 20000)
    hist.daddr = _mapped(np.full(len(hist), a4))
    hist.hash = None
    dp = RefDatapath(t)
    hres = run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    ok = np.flatnonzero(hres[0] != 2)
    parts, pos = [], []
    at = rng.random(len(ok)) * 0.9
    for f, p_ in ((0x12, 1.0), (0x10, 0.7), (0x18, 0.5)):
        sel = np.flatnonzero(rng.random(len(ok)) < p_)
        src = S.take(hist, ok[sel])
        k = len(sel)
        # (an ICMPv6 echo request's reply: ICMP echo reply, type 0, same id)
        icmp = src.proto == S.IPPROTO_ICMPV6
        rep = S.Headers(4, np.full(k, a4, np.uint32), np.full(k, a4, np.uint32),
                        np.where(icmp, 0, src.dport).astype(np.uint16),
                        np.where(icmp, src.dport, src.sport).astype(np.uint16),
                        np.where(icmp, S.IPPROTO_ICMP, src.proto).astype(np.uint8),
                        np.zeros(k, np.uint8), rng.integers(60, 1500, size=k).astype(np.uint16),
                        np.zeros(k, np.uint32),
                        np.where(src.proto == S.IPPROTO_TCP, f, 0).astype(np.uint8))
        parts.append(rep)
        pos.append(at[sel])
        at = at + rng.random(len(ok)) * 0.03
    # ICMP errors the endpoint sends itself about those flows: every
    # translation case of icmp4_to_icmp6 (nat46.h)
    k = int(n * 0.1)
    err = S.take(parts[0], rng.integers(0, len(parts[0]), size=k))
    tc = np.array([[3, 0], [3, 1], [3, 3], [3, 4], [3, 9], [3, 13], [11, 0], [12, 0], [5, 0]],
                  np.uint16)
    pick = tc[rng.integers(0, len(tc), size=k)]
    err.proto[:] = S.IPPROTO_ICMP
    err.sport[:] = (pick[:, 0] | pick[:, 1] << 8).astype(np.uint16)
    err.dport[:] = 0
    err.tcpflags = np.zeros(k, np.uint8)
    parts.append(err)
    pos.append(rng.random(k))
    plain = S.gen_headers_v4(rng, int(n * 0.2), ipc4, S.local_v4_addrs(t)[:1], local_frac=0.0,
                             mark_host=0, mark_proxy=0, frag=0, src_fixed=S.LXC_IPV4)
    parts.append(plain)
    pos.append(rng.random(len(plain)))
    h = S.concat(parts)
    h = S.take(h, np.argsort(np.concatenate(pos), kind="stable"))
    h.hash = None
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


def _hdrs4(sa, da, sp, dp, proto, tcpf, length):
    n = len(sp)
    tcpf = np.asarray(tcpf, np.uint8)
    h = S.Headers(4, np.full(n, sa, np.uint32), np.full(n, da, np.uint32),
                  S.htons(sp), S.htons(dp), np.asarray(proto, np.uint8),
                  np.zeros(n, np.uint8), np.asarray(length, np.uint16),
                  np.zeros(n, np.uint32), tcpf)
    h.flags[(h.proto == S.IPPROTO_TCP) & ((tcpf & 0x05) != 0)] = S.HF_TCP_CLOSE
    return h


def sc_self_egress(n=2600, seed=45):
    """Traffic to itself inside one egress stream (the keys whose two
    addresses are the sender's own, conntrack.h:487-494, and a looped-back
    service flow's TUPLE_F_IN entry, :725-748): the endpoint opens TCP and
    UDP flows to its own address and answers them (the answer's egress
    lookup finds, as k1, the entry the opening packet's ingress stage
    created: CT_REPLY), pings itself and sends ICMP errors about those
    flows, and opens flows to the service whose backend is itself and
    answers them to IPV4_LOOPBACK — all in the stream that creates the
    entries.  Its own ingress admits its SECLABEL on TCP 80 and UDP 53 only,
    so some opening packets are dropped at their second stage."""
    t, rng, vips, ports, protos = _lb_setup(seed)
    sec = int(t.seclabel[S.EP_LXC_ID])
    pol = t.policy[S.EP_LXC_ID]
    pol = pol[~((pol["egress"] == 0) & (pol["identity"] == sec))]
    ing = np.zeros(2, S.POLICY_DT)
    ing["identity"] = sec
    ing["dport"] = S.htons(np.array([80, 53]))
    ing["proto"] = [S.IPPROTO_TCP, S.IPPROTO_UDP]
    t.policy[S.EP_LXC_ID] = np.concatenate([pol, ing])
    A = int(S.LXC_IPV4)
    lb = t.lb4
    k6 = int(np.flatnonzero((lb["target"] == A))[0])
    vip, vport = int(lb["addr"][k6]), int(lb["dport"][k6])

    def svc_flows(x, f):
        m = len(x)
        return S.Headers(4, np.full(m, A, np.uint32), np.full(m, vip, np.uint32),
                         S.htons(x), np.full(m, vport, np.uint16),
                         np.full(m, S.IPPROTO_TCP, np.uint8), np.zeros(m, np.uint8),
                         rng.integers(60, 1500, size=m).astype(np.uint16),
                         np.zeros(m, np.uint32), np.full(m, f, np.uint8))
    # a history: self flows opened and answered, service flows opened
    hx = 29000 + np.arange(20)
    hy = rng.choice(np.array([80, 8080]), size=20)
    hist = S.concat([_hdrs4(A, A, hx, hy, np.full(20, S.IPPROTO_TCP), np.full(20, 0x02),
                            np.full(20, 100)),
                     _hdrs4(A, A, hy, hx, np.full(20, S.IPPROTO_TCP), np.full(20, 0x12),
                            np.full(20, 100)),
                     svc_flows(44000 + np.arange(40), 0x02),
                     # (plain traffic too: the other endpoint's local CT maps
                     # hold entries before the stream)
                     S.gen_headers_v4(rng, 200, t.ipcache[t.ipcache["family"] == 1],
                                      S.local_v4_addrs(t), local_frac=0.3, mark_host=0,
                                      mark_proxy=0, src_fixed=S.LXC_IPV4, frag=0)])
    hist.hash = None
    dp = RefDatapath(t)
    run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    parts, pos = [], []

    def add_(h, p):
        parts.append(h)
        pos.append(np.asarray(p, np.float64))
    # the history's flows: later packets, some closing
    est = S.take(hist, rng.integers(0, len(hist), size=300))
    est.tcpflags = np.where(rng.random(300) < 0.1, 0x11, 0x10).astype(np.uint8)
    est.flags = np.where(est.tcpflags == 0x11, S.HF_TCP_CLOSE, 0).astype(np.uint8)
    add_(est, rng.random(300))
    # TCP to itself: SYN, SYN-ACK back, ACK, data back, some FIN, a re-open
    m = 60
    x = 30000 + np.arange(m)
    y = rng.choice(np.array([80, 8080, 80, 443]), size=m)
    p0 = rng.random(m) * 0.7
    seq = [(x, y, 0x02), (y, x, 0x12), (x, y, 0x10), (y, x, 0x18), (x, y, 0x11),
           (x, y, 0x02)]
    keep = np.ones(m, bool)
    for j, (a, b, f) in enumerate(seq):
        if j == 4:
            keep = rng.random(m) < 0.4
        elif j == 5:
            keep &= rng.random(m) < 0.5
        sel = np.flatnonzero(keep)
        add_(_hdrs4(A, A, a[sel], b[sel], np.full(len(sel), S.IPPROTO_TCP),
                    np.full(len(sel), f), rng.integers(60, 1500, size=len(sel))),
             p0[sel] + 0.04 * j + rng.random(len(sel)) * 0.01)
    # UDP to itself (53 allowed at its own ingress, 5353 not), answers
    m = 40
    x = 33000 + np.arange(m)
    y = rng.choice(np.array([53, 5353]), size=m)
    p0 = rng.random(m) * 0.7
    for j, (a, b) in enumerate([(x, y), (y, x), (x, y), (y, x)]):
        sel = np.flatnonzero(rng.random(m) < (1.0 if j < 2 else 0.6))
        add_(_hdrs4(A, A, a[sel], b[sel], np.full(len(sel), S.IPPROTO_UDP),
                    np.zeros(len(sel)), rng.integers(60, 1500, size=len(sel))),
             p0[sel] + 0.05 * j + rng.random(len(sel)) * 0.01)
    # pings to itself and their replies; ICMP errors about its own flows
    m = 30
    p0 = rng.random(m) * 0.8
    for j, ty in enumerate([8, 0, 8, 0]):
        add_(_hdrs4(A, A, np.full(m, ty), np.zeros(m), np.full(m, S.IPPROTO_ICMP),
                    np.zeros(m), rng.integers(60, 200, size=m)),
             p0 + 0.03 * j + rng.random(m) * 0.01)
    m = 40
    add_(_hdrs4(A, A, rng.choice(np.array([3, 11]), size=m), np.zeros(m),
                np.full(m, S.IPPROTO_ICMP), np.zeros(m), rng.integers(60, 200, size=m)),
         0.2 + rng.random(m) * 0.8)
    # flows to the service whose backend is the endpoint itself
    m = 150
    p0 = rng.random(m) * 0.6
    svc = svc_flows(45000 + np.arange(m), 0x02)
    add_(svc, p0)
    later = S.take(svc, np.arange(m))
    later.tcpflags = np.full(m, 0x10, np.uint8)
    add_(later, p0 + 0.1)
    # plain traffic beside it
    plain = S.gen_headers_v4(rng, int(n * 0.35), t.ipcache[t.ipcache["family"] == 1],
                             S.local_v4_addrs(t), local_frac=0.3, mark_host=0,
                             mark_proxy=0, src_fixed=S.LXC_IPV4, frag=0)
    add_(plain, rng.random(len(plain)))
    h = S.concat(parts)
    order = np.argsort(np.concatenate(pos), kind="stable")
    h = S.take(h, order)
    h.hash = None
    # the looped-back flows' answers (the history's and the stream's): the endpoint, as the backend, replies
    # to the address it saw (IPV4_LOOPBACK) from its translated port, after
    # the flow's first packet (a dry run of the reference tells which flows
    # looped back and their ports)
    dry = RefDatapath(t)
    try:
        res = run(dry, h, MODE_EGRESS, S.EP_LXC_ID)
    finally:
        dry.close()
    pk = res[8]
    lo = np.flatnonzero((pk[:, 0] == S.IPV4_LOOPBACK) & (h.proto == S.IPPROTO_TCP) &
                        (res[0] != 2))
    _, first = np.unique(h.sport[lo], return_index=True)
    lo = lo[first]
    if len(lo):
        rp = _hdrs4(A, S.IPV4_LOOPBACK, np.zeros(len(lo), np.uint16),
                    np.zeros(len(lo), np.uint16), np.full(len(lo), S.IPPROTO_TCP),
                    np.full(len(lo), 0x12), rng.integers(60, 1500, size=len(lo)))
        rp.sport = (pk[lo, 2] >> 16).astype(np.uint16)   # be16 raw, as the packet left
        rp.dport = (pk[lo, 2] & 0xFFFF).astype(np.uint16)
        at = np.concatenate([np.arange(len(h)), lo + 0.5 + rng.random(len(lo)) * 40])
        h = S.concat([h, rp])
        h = S.take(h, np.argsort(at, kind="stable"))
        h.hash = None
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


def _hdrs6(sa, da, sp, dp, proto, tcpf, length):
    n = len(sp)
    tcpf = np.asarray(tcpf, np.uint8)
    h = S.Headers(6, np.tile(sa, (n, 1)), np.tile(da, (n, 1)),
                  S.htons(sp), S.htons(dp), np.asarray(proto, np.uint8),
                  np.zeros(n, np.uint8), np.asarray(length, np.uint16),
                  np.zeros(n, np.uint32), tcpf)
    h.flags[(h.proto == S.IPPROTO_TCP) & ((tcpf & 0x05) != 0)] = S.HF_TCP_CLOSE
    return h


def sc_self_egress_v6(n=2400, seed=47):
    """The IPv6 counterpart of self_egress_v4: an endpoint's TCP / UDP flows
    to its own address and their answers, pings (ICMPv6 echo) and ICMPv6
    errors to itself, and flows to the IPv6 service whose backend is the
    endpoint (lb6_local translates the destination back to the sender; no
    loopback address in IPv6) answered from the backend port — all in the
    stream that creates the entries.  Its own ingress admits its SECLABEL
    on TCP 80 and UDP 53 only."""
    t, rng, vips, ports, protos = _lb_setup6(seed)
    sec = int(t.seclabel[S.EP_LXC_ID])
    pol = t.policy[S.EP_LXC_ID]
    pol = pol[~((pol["egress"] == 0) & (pol["identity"] == sec))]
    ing = np.zeros(2, S.POLICY_DT)
    ing["identity"] = sec
    ing["dport"] = S.htons(np.array([80, 53]))
    ing["proto"] = [S.IPPROTO_TCP, S.IPPROTO_UDP]
    t.policy[S.EP_LXC_ID] = np.concatenate([pol, ing])
    A = np.asarray(S.LXC_IPV6, np.uint8)
    lb = t.lb6
    own = np.flatnonzero((np.asarray(lb["target"]).reshape(len(lb), -1) == A).all(1) &
                         (lb["slave"] != 0))
    k6 = int(own[0])
    vip, vport = np.asarray(lb["addr"][k6], np.uint8), int(lb["dport"][k6])

    def svc_flows(x, f):
        m = len(x)
        return S.Headers(6, np.tile(A, (m, 1)), np.tile(vip, (m, 1)), S.htons(x),
                         np.full(m, vport, np.uint16), np.full(m, S.IPPROTO_TCP, np.uint8),
                         np.zeros(m, np.uint8),
                         rng.integers(100, 1500, size=m).astype(np.uint16),
                         np.zeros(m, np.uint32), np.full(m, f, np.uint8))
    ipc = t.ipcache[t.ipcache["family"] == 2]
    hx = 29000 + np.arange(20)
    hy = rng.choice(np.array([80, 8080]), size=20)
    hist = S.concat([_hdrs6(A, A, hx, hy, np.full(20, S.IPPROTO_TCP), np.full(20, 0x02),
                            np.full(20, 100)),
                     _hdrs6(A, A, hy, hx, np.full(20, S.IPPROTO_TCP), np.full(20, 0x12),
                            np.full(20, 100)),
                     svc_flows(44000 + np.arange(40), 0x02),
                     S.gen_headers_v6(rng, 200, ipc, S.local_v6_addrs(t), local_frac=0.3,
                                      mark_host=0, mark_proxy=0, src_fixed=S.LXC_IPV6,
                                      ext=0, exthdr_drop=0)])
    hist.hash = None
    dp = RefDatapath(t)
    run(dp, hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(dp.ct_dump())
    dp.reset_counters()
    parts, pos = [], []

    def add_(h, p):
        parts.append(h)
        pos.append(np.asarray(p, np.float64))
    est = S.take(hist, rng.integers(0, len(hist), size=300))
    est.tcpflags = np.where(rng.random(300) < 0.1, 0x11, 0x10).astype(np.uint8)
    est.flags = np.where((est.tcpflags == 0x11) & (est.proto == S.IPPROTO_TCP),
                         S.HF_TCP_CLOSE, 0).astype(np.uint8)
    add_(est, rng.random(300))
    m = 60
    x = 30000 + np.arange(m)
    y = rng.choice(np.array([80, 8080, 80, 443]), size=m)
    p0 = rng.random(m) * 0.7
    keep = np.ones(m, bool)
    for j, (a, b, f) in enumerate([(x, y, 0x02), (y, x, 0x12), (x, y, 0x10), (y, x, 0x18),
                                   (x, y, 0x11), (x, y, 0x02)]):
        if j == 4:
            keep = rng.random(m) < 0.4
        elif j == 5:
            keep &= rng.random(m) < 0.5
        sel = np.flatnonzero(keep)
        add_(_hdrs6(A, A, a[sel], b[sel], np.full(len(sel), S.IPPROTO_TCP),
                    np.full(len(sel), f), rng.integers(100, 1500, size=len(sel))),
             p0[sel] + 0.04 * j + rng.random(len(sel)) * 0.01)
    m = 40
    x = 33000 + np.arange(m)
    y = rng.choice(np.array([53, 5353]), size=m)
    p0 = rng.random(m) * 0.7
    for j, (a, b) in enumerate([(x, y), (y, x), (x, y), (y, x)]):
        sel = np.flatnonzero(rng.random(m) < (1.0 if j < 2 else 0.6))
        add_(_hdrs6(A, A, a[sel], b[sel], np.full(len(sel), S.IPPROTO_UDP),
                    np.zeros(len(sel)), rng.integers(100, 1500, size=len(sel))),
             p0[sel] + 0.05 * j + rng.random(len(sel)) * 0.01)
    m = 30
    p0 = rng.random(m) * 0.8
    for j, ty in enumerate([128, 129, 128, 129]):
        add_(_hdrs6(A, A, np.full(m, ty), np.zeros(m), np.full(m, S.IPPROTO_ICMPV6),
                    np.zeros(m), rng.integers(100, 200, size=m)),
             p0 + 0.03 * j + rng.random(m) * 0.01)
    m = 40
    add_(_hdrs6(A, A, rng.choice(np.array([1, 3]), size=m), np.zeros(m),
                np.full(m, S.IPPROTO_ICMPV6), np.zeros(m), rng.integers(100, 200, size=m)),
         0.2 + rng.random(m) * 0.8)
    m = 150
    p0 = rng.random(m) * 0.6
    svc = svc_flows(45000 + np.arange(m), 0x02)
    add_(svc, p0)
    later = S.take(svc, np.arange(m))
    later.tcpflags = np.full(m, 0x10, np.uint8)
    add_(later, p0 + 0.1)
    plain = S.gen_headers_v6(rng, int(n * 0.3), ipc, S.local_v6_addrs(t), local_frac=0.3,
                             mark_host=0, mark_proxy=0, src_fixed=S.LXC_IPV6, ext=0,
                             exthdr_drop=0)
    add_(plain, rng.random(len(plain)))
    h = S.concat(parts)
    h = S.take(h, np.argsort(np.concatenate(pos), kind="stable"))
    h.hash = None
    # the service flows the endpoint itself serves: it answers from the
    # backend port (a dry run of the reference gives the translated port)
    dry = RefDatapath(t)
    try:
        res = run(dry, h, MODE_EGRESS, S.EP_LXC_ID)
    finally:
        dry.close()
    pk = res[8]
    dst = np.ascontiguousarray(pk[:, 4:8]).view(np.uint8).reshape(-1, 16)
    vis = (np.asarray(h.daddr) == vip).all(1)
    lo = np.flatnonzero(vis & (dst == A).all(1) & (h.proto == S.IPPROTO_TCP) & (res[0] != 2))
    _, first = np.unique(h.sport[lo], return_index=True)
    lo = lo[first]
    if len(lo):
        rp = _hdrs6(A, A, np.zeros(len(lo)), np.zeros(len(lo)),
                    np.full(len(lo), S.IPPROTO_TCP), np.full(len(lo), 0x12),
                    rng.integers(100, 1500, size=len(lo)))
        rp.sport = (pk[lo, 8] >> 16).astype(np.uint16)
        rp.dport = (pk[lo, 8] & 0xFFFF).astype(np.uint16)
        at = np.concatenate([np.arange(len(h)), lo + 0.5 + rng.random(len(lo)) * 40])
        h = S.concat([h, rp])
        h = S.take(h, np.argsort(at, kind="stable"))
        h.hash = None
    return t, h.slice(0, n), MODE_EGRESS, S.EP_LXC_ID, dp


SCENARIOS = {
    "edge_ingress_v4": sc_edge_ingress,
    "small_ingress_v4": sc_small_ingress,
    "c1_ingress_v4": sc_c1_ingress,
    "c2_ingress_v4": sc_c2_ingress,
    "c2_egress_v4": sc_c2_egress,
    "xdp_v4": sc_xdp,
    "full_v4": lambda: sc_xdp(seed=6, mode=MODE_FULL),
    "empty_ingress_v4": sc_empty,
    "edge_ingress_v6": sc_edge_ingress_v6,
    "c3_ingress_v6": sc_c3_ingress,
    "c3_egress_v6": sc_c3_egress,
    "xdp_v6": sc_xdp_v6,
    "full_v6": lambda: sc_xdp_v6(seed=12, mode=MODE_FULL),
    "ct_ingress_v4": lambda: _ct_scenario(4, MODE_INGRESS, 21),
    "ct_egress_v4": lambda: _ct_scenario(4, MODE_EGRESS, 22),
    "ct_ingress_v6": lambda: _ct_scenario(6, MODE_INGRESS, 23),
    "ct_egress_v6": lambda: _ct_scenario(6, MODE_EGRESS, 24),
    "ct_seq_ingress_v4": lambda: _ct_seq_scenario(4, MODE_INGRESS, 25),
    "ct_seq_egress_v4": lambda: _ct_seq_scenario(4, MODE_EGRESS, 26),
    "ct_seq_ingress_v6": lambda: _ct_seq_scenario(6, MODE_INGRESS, 27),
    "ct_seq_egress_v6": lambda: _ct_seq_scenario(6, MODE_EGRESS, 28),
    "nat46_egress_v6": sc_nat46_egress_v6,
    "nat46_reply_v4": sc_nat46_reply_v4,
    "nat64_local_v6": sc_nat64_local_v6,
    "lb_egress_v4": sc_lb_egress,
    "lb_reply_v4": sc_lb_reply,
    "lb_egress_v6": sc_lb_egress_v6,
    "lb_reply_v6": sc_lb_reply_v6,
    "self_egress_v4": sc_self_egress,
    "self_egress_v6": sc_self_egress_v6,
    "nat64_lb_v6": sc_nat64_lb_v6,
    "nat46_self_v4": sc_nat46_self_v4,
    "nat64_lb_lo_v6": lambda: sc_nat64_lb_v6(seed=68, loopback=True),
}
# fixtures that pin only the oracle (tests/golden_oracle): the engine has
# not been run against them on the GPU
ORACLE_ONLY = {"nat64_lb_v6", "nat46_self_v4", "nat64_lb_lo_v6"}


def main(names):
    for name in names or SCENARIOS:
        t0 = time.time()
        sc = SCENARIOS[name]()
        t, h, mode, ep = sc[:4]
        dp = sc[4] if len(sc) > 4 else RefDatapath(t)
        try:
            res = run(dp, h, mode, ep)
            path = save(name, t, h, mode, ep, res, dp)
        finally:
            dp.close()
        act = res[0]
        print(f"{name}: {len(h)} headers, mode {mode}, actions "
              f"{dict(zip(*np.unique(act, return_counts=True)))}, "
              f"{os.path.getsize(path) // 1024} KiB, {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main(sys.argv[1:])
