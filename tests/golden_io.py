"""Load the golden fixtures written by oracle/gen_golden.py."""
import glob
import os

import numpy as np

import oracle as O
from cilium_amd import synth as S

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# fixtures that pin only the oracle: streams the engine has not been run
# against on the GPU (the GPU tests take names(), golden/ alone)
ORACLE_ONLY_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_oracle")


def names():
    return sorted(os.path.basename(p)[:-4]
                  for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def oracle_only_names():
    return sorted(os.path.basename(p)[:-4]
                  for p in glob.glob(os.path.join(ORACLE_ONLY_DIR, "*.npz")))


class Golden:
    def pkt_addrs(self):
        """The packet's (saddr, daddr) as the programs left them, in the
        header batch's address format (IPv4 u32, IPv6 (n, 16) bytes)."""
        if self.headers.family == 4:
            return self.pkt[:, 0], self.pkt[:, 1]
        p = np.ascontiguousarray(self.pkt)
        return (np.ascontiguousarray(p[:, 0:4]).view(np.uint8).reshape(-1, 16),
                np.ascontiguousarray(p[:, 4:8]).view(np.uint8).reshape(-1, 16))

    def __init__(self, name):
        self.name = name
        path = os.path.join(GOLDEN_DIR, name + ".npz")
        if not os.path.exists(path):
            path = os.path.join(ORACLE_ONLY_DIR, name + ".npz")
        d = np.load(path, allow_pickle=False)
        self.mode = int(d["mode"])
        self.ep_lxc = int(d["ep_lxc"])
        policy = {int(k.split("_")[1]): d[k] for k in d.files
                  if k.startswith("policy_")}
        seclabel = {int(a): int(b) for a, b in d["seclabel"]}
        self.tables = S.Tables(d["ipcache"], d["endpoints"], policy,
                               d["prefilter"], seclabel,
                               d["ct"] if "ct" in d.files else None)
        if "lb4" in d.files:   # service load balancing (LB4_DT, REVNAT4_DT)
            self.tables.lb4 = d["lb4"]
            self.tables.revnat4 = d["revnat4"]
        if "lb6" in d.files:   # (LB6_DT, REVNAT6_DT)
            self.tables.lb6 = d["lb6"]
            self.tables.revnat6 = d["revnat6"]
        # CT maps after the stream, oracle row format (None: no CT state)
        self.ct_after = d["x_ct"] if "x_ct" in d.files else None
        self.headers = S.Headers(int(d["h_family"]), d["h_saddr"], d["h_daddr"],
                                 d["h_sport"], d["h_dport"], d["h_proto"],
                                 d["h_flags"], d["h_length"], d["h_mark"],
                                 d["h_tcpflags"] if "h_tcpflags" in d.files else None)
        # skb->hash of each header as the reference's records reported it
        # (lb4_select_slave's input), and the packet the program left:
        # (saddr, daddr, first L4 word); None in fixtures without a service
        self.hash_ok = d["x_hash_ok"] if "x_hash_ok" in d.files else None
        if self.hash_ok is not None:
            self.headers.hash = d["x_hash"]
        # ((n, 3) u32 for IPv4; (n, 9) for IPv6: saddr and daddr as four
        # raw words each, then the L4 word)
        self.pkt = d["x_pkt"] if "x_pkt" in d.files else None
        # the cilium_events perf-ring samples (trace_notify / drop_notify,
        # 32 bytes each, EVENT_DT) and the header of each; None in older
        # fixtures
        self.ev = (d["x_ev"].reshape(-1).view(O.EVENT_DT)
                   if "x_ev" in d.files else None)
        self.ev_hdr = d["x_ev_hdr"] if "x_ev_hdr" in d.files else None
        # bpf_ktime_get_sec() while each header ran (0xFFFFFFFF: a second
        # boundary fell inside its run); None in older fixtures
        self.clock = d["x_clock"] if "x_clock" in d.files else None
        self.action = d["x_action"]
        self.verdict = d["x_verdict"]
        self.identity = d["x_identity"]
        self.idmask = d["x_idmask"]
        self.metrics = d["x_metrics"]
        # skb->cb[0..4] after the reference ran (None in older fixtures)
        self.cb = d["x_cb"] if "x_cb" in d.files else None
        self.counters = {int(k.split("_")[2]): d[k] for k in d.files
                         if k.startswith("x_counters_")}
        # the kernel's own LPM of each header's addresses in cilium_ipcache
        # (oracle/pin_lpm.py, gen_golden.lpm_pin): (n, 4) labels and hits for
        # saddr, daddr, the packet's saddr, daddr (services: translated)
        self.lpm = d["x_lpm"] if "x_lpm" in d.files else None
        self.lpm_hit = d["x_lpm_hit"] if "x_lpm_hit" in d.files else None
        # (IPv6 fixtures) the IPv4 LPM of each daddr's low 32 bits: NAT64's
        # IPv4 egress lookup of a v4-mapped destination
        self.lpm_nat = d["x_lpm_nat"] if "x_lpm_nat" in d.files else None
        self.lpm_nat_hit = d["x_lpm_nat_hit"] if "x_lpm_nat_hit" in d.files else None
        # (IPv6 fixtures with IPv4 services) the IPv4 packet a NAT64 hop left:
        # (saddr, daddr, L4 word) after the IPv4 program's service step
        self.pkt4 = d["x_pkt4"] if "x_pkt4" in d.files else None
        self.pkt4_ok = d["x_pkt4_ok"].astype(bool) if "x_pkt4_ok" in d.files else None
        # what the reference reported itself (perf-ring records, drop cb[],
        # proxy map); identity / idmask below add the identities derived
        # from the kernel's LPM for every other tc-path header
        self.identity_reported = self.identity
        self.idmask_reported = self.idmask
        if self.lpm is not None:
            exp, applies = lpm_identity(self)
            full = np.uint32(0xFFFFFFFF)
            self.identity = np.where(applies, exp, self.identity).astype(np.uint32)
            self.idmask = np.where(applies, full, self.idmask).astype(np.uint32)
            self.lpm_expected, self.lpm_applies = exp, applies


# Drops that end a program before its ipcache lookup, so no identity is
# derived (common.h:239-265): egress DROP_INVALID_SIP (lxc.h:55),
# DROP_CT_UNKNOWN_PROTO (ct_lookup4/6 runs before the dstID lookup,
# bpf_lxc.c:497-532), DROP_INVALID_EXTHDR / DROP_FRAG_NOSUPPORT
# (ipv6_hdrlen), DROP_NO_SERVICE (lb4_local); ingress only the IPv6 header
# walk of handle_ipv6 (bpf_netdev.c:172-200) — its CT drops come after the
# source identity
NO_IDENTITY_EGRESS = (-132, -137, -156, -157, -158)
NO_IDENTITY_INGRESS = (-156, -157)


def no_identity(g):
    return np.isin(g.verdict, NO_IDENTITY_EGRESS if g.mode == 1 else NO_IDENTITY_INGRESS)


def identity_from_mark(mark):
    """handle_identity_from_host (bpf_netdev.c:128-153) on skb->mark"""
    m = np.asarray(mark, np.uint64)
    magic = m & 0x0F00
    proxy = (magic == 0x0A00) | (magic == 0x0B00)   # MARK_MAGIC_PROXY_{INGRESS,EGRESS}
    return np.where(proxy, ((m & 0xFF) << 16) | (m >> 16),
                    np.where(magic == 0x0C00, 1, 2)).astype(np.uint32)   # HOST / WORLD


def lpm_identity(g: Golden):
    """The identity of every tc-path header from the kernel's own LPM
    results (g.lpm) by the reference's derivation -> (identity u32, applies):
    ingress (bpf_netdev.c:374-398, v6 :202-213): the mark's identity; if it
    is reserved (policy.h:41-44, < HEALTH_ID) the LPM label of saddr when
    != 0, != CLUSTER_ID (v4 also != HOST_ID); egress (bpf_lxc.c:516-532, v6
    :206-221): the LPM label of the tuple's daddr (the service's backend,
    or the VIP for a looped-back flow) when != 0, else CLUSTER_ID inside
    IPV4_CLUSTER_RANGE/MASK (v6: the /64 of ROUTER_IP), else WORLD_ID.
    applies: tc-path headers (not XDP, not an XDP drop of FULL mode) whose
    program reached the lookup (no_identity)."""
    n = len(g.verdict)
    v4 = g.headers.family == 4
    tc = np.full(n, g.mode != 2)
    if g.mode == 3:
        tc &= ~((g.action == 1) & (g.verdict == -1))   # XDP_DROP
    applies = tc & ~no_identity(g)
    lab, hit = g.lpm.astype(np.uint32), g.lpm_hit.astype(bool)
    nat = np.zeros(n, bool)
    if g.mode == 1 and not v4:
        # NAT64 (bpf_lxc.c:353-360): a peer outside the cluster in
        # ::ffff:0:0/96 leaves through the IPv4 egress program, whose dstID
        # is the IPv4 derivation of the low 32 bits (:516-532)
        da = np.asarray(g.headers.daddr, np.uint8)
        mapped = (da[:, :10] == 0).all(1) & (da[:, 10] == 0xff) & (da[:, 11] == 0xff)
        cl = hit[:, 1] & (lab[:, 1] == S.CLUSTER_ID)
        nat = mapped & ~cl
        if g.lpm_nat is None:
            applies &= ~nat
    if g.mode == 1:
        col = np.full(n, 1)
        da = np.asarray(g.headers.daddr)
        if g.pkt is not None and v4:   # lb4_local: the tuple's daddr is the backend
            loop = g.pkt[:, 0] == S.IPV4_LOOPBACK
            col = np.where(loop, 1, 3)
            da = np.where(loop, np.asarray(g.headers.daddr, np.uint32), g.pkt[:, 1])
        elif g.pkt is not None:        # lb6_local (no loopback case)
            col = np.full(n, 3)
            da = g.pkt_addrs()[1]
        l, h = lab[np.arange(n), col], hit[np.arange(n), col]
        if v4:
            cluster = (np.asarray(da, np.uint32) & 0xFF0000) == 0x100000
        else:
            cluster = (np.asarray(da, np.uint8)[:, :8] ==
                       np.asarray(S.ROUTER_IPV6, np.uint8)[:8]).all(axis=1)
        exp = np.where(h & (l != 0), l, np.where(cluster, S.CLUSTER_ID, S.WORLD_ID))
        if nat.any() and g.lpm_nat is not None:
            d4 = np.ascontiguousarray(np.asarray(g.headers.daddr, np.uint8)[:, 12:16]
                                      ).view("<u4").ravel()
            if g.pkt4 is not None:   # the service step's backend (bpf_lxc.c:476-501)
                d4 = np.where(g.pkt4_ok, g.pkt4[:, 1], d4).astype(np.uint32)
            l4, h4 = g.lpm_nat.astype(np.uint32), g.lpm_nat_hit.astype(bool)
            e4 = np.where(h4 & (l4 != 0), l4,
                          np.where((d4 & 0xFF0000) == 0x100000, S.CLUSTER_ID, S.WORLD_ID))
            exp = np.where(nat, e4, exp)
    else:
        ident = identity_from_mark(g.headers.mark)
        l, h = lab[:, 0], hit[:, 0]
        ok = h & (l != 0) & (l != S.CLUSTER_ID)
        if v4:
            ok &= l != 1   # HOST_ID
        exp = np.where((ident < 4) & ok, l, ident)
    return exp.astype(np.uint32), applies


def mismatches(g: Golden, action, verdict, identity):
    """Indices where (action, verdict, pinned identity bits) differ."""
    bad = (action != g.action) | (verdict != g.verdict) | \
          ((identity & g.idmask) != (g.identity & g.idmask))
    return np.nonzero(bad)[0]


# ct_entry bytes the comparison ignores: lifetime (offset 32, clock),
# seen_non_syn (bit 4 of offset 36) and the seen-TCP-flag bytes (42, 43:
# TCP flag bits the header batch does not carry), last_{tx,rx}_report
# (48-55, clock).  Row offsets: entry starts at 44.
def ct_masked(rows):
    r = np.array(rows, np.uint8).reshape(-1, S.CT_ROW).copy()
    e = 44
    r[:, e + 32:e + 36] = 0
    r[:, e + 36] &= 0xEF
    r[:, e + 42:e + 44] = 0
    r[:, e + 48:e + 56] = 0
    return r


def expected_drop_notify(g: Golden):
    """(header indices, fields) of the drop notifications the reference's
    send_drop_notify armed (drop.h:98-102): cb[1] = src << 16 | dst & 0xFFFF,
    cb[2] = reason, cb[3] = dst_id, cb[4] = ifindex.  XDP drops notify
    nothing (bpf_xdp.c has no send_drop_notify)."""
    tc = g.mode != 2
    idx = np.flatnonzero((g.action == 2) & (g.verdict < 0) & (g.verdict != -1)
                         if tc else np.zeros(len(g.action), bool))
    cb = g.cb[idx].astype(np.int64)
    f = dict(subtype=(-cb[:, 2]) & 0xFF,
             src_label=(cb[:, 1] >> 16) & 0xFFFF,
             dst_label=cb[:, 1] & 0xFFFF,
             dst_id=cb[:, 3] & 0xFFFFFFFF,
             ifindex=cb[:, 4] & 0xFFFFFFFF)
    return idx.astype(np.uint64), f
