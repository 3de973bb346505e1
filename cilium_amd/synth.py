"""Synthetic tables and header streams for the BASELINE.json configurations.

The reference has no traffic generator for the verdict path; SURVEY.md §8d
defines the workloads (C1..C5).  Everything here is plain numpy and seeded,
so the golden-vector script (oracle/gen_golden.py), the parity tests and
bench.py all see byte-identical inputs for a given seed.

Byte conventions follow the reference datapath:
  * IPv4 addresses are `__be32` as the BPF program loads them: the four
    network-order bytes read as a little-endian u32 (so 10.0.0.1 -> 0x0100000a).
  * Ports are `__be16` raw (network-order bytes read little-endian), the form
    stored in PolicyKey.DestPort (pkg/maps/policymap/policymap.go:64-69).
  * For ICMP the "sport" word carries the first two ICMP bytes (type, code),
    "dport" the checksum — exactly what ct_lookup4 reads
    (bpf/lib/conntrack.h:496-526).
"""
from __future__ import annotations

import dataclasses
import numpy as np

# reserved identities, bpf/node_config.h
HOST_ID, WORLD_ID, CLUSTER_ID, HEALTH_ID, INIT_ID = 1, 2, 3, 4, 5
# header flag bits (cfc.h CFC_HF_*)
HF_FRAG = 1          # ipv4_is_fragment(): frag_off & htons(0xBFFF)
HF_TCP_CLOSE = 2     # ct_lookup's "rst || fin" (conntrack.h:533): bit 0 of
                     # TCP byte 12, where union tcp_flags' bitfields all sit
HF_EXTHDR = 4        # IPv6: extension headers precede `proto`
IPPROTO_ICMP, IPPROTO_TCP, IPPROTO_UDP, IPPROTO_ICMPV6 = 1, 6, 17, 58

IPCACHE_DT = np.dtype([("family", "u1"), ("plen", "u1"), ("addr", "u1", 16),
                       ("label", "<u4"), ("tunnel", "<u4")])
ENDPOINT_DT = np.dtype([("family", "u1"), ("addr", "u1", 16),
                        ("ifindex", "<u4"), ("lxc_id", "<u2"),
                        ("flags", "<u4")])
POLICY_DT = np.dtype([("identity", "<u4"), ("dport", "<u2"), ("proto", "u1"),
                      ("egress", "u1"), ("proxy_port", "<u2")])
PREFILTER_DT = np.dtype([("family", "u1"), ("plen", "u1"),
                         ("addr", "u1", 16), ("dyn", "u1")])


# one conntrack entry: which map (global or an endpoint's local maps, TCP or
# ANY) and the raw struct ipv{4,6}_ct_tuple / struct ct_entry bytes
# (bpf/lib/common.h:338-406)
CT_DT = np.dtype([("family", "u1"), ("lxc", "<i4"), ("any", "u1"),
                  ("tuple", "u1", 38), ("entry", "u1", 56)])

# cilium_lb4_services: struct lb4_key {address, dport, slave} and struct
# lb4_service {target, port, count, rev_nat_index, weight} (bpf/lib/common.h:
# 427-439; addresses be32 raw, ports be16 raw); cilium_lb4_reverse_nat: key
# rev_nat_index, struct lb4_reverse_nat {address, port} (:441-444)
LB4_DT = np.dtype([("addr", "<u4"), ("dport", "<u2"), ("slave", "<u2"),
                   ("target", "<u4"), ("port", "<u2"), ("count", "<u2"),
                   ("rev_nat", "<u2"), ("weight", "<u2")])
REVNAT4_DT = np.dtype([("index", "<u2"), ("addr", "<u4"), ("port", "<u2")])
# struct lb6_key + struct lb6_service (common.h:408-420), packed; struct
# lb6_reverse_nat (:422-425) behind its u16 index
LB6_DT = np.dtype([("addr", "u1", 16), ("dport", "<u2"), ("slave", "<u2"),
                   ("target", "u1", 16), ("port", "<u2"), ("count", "<u2"),
                   ("rev_nat", "<u2"), ("weight", "<u2")])
REVNAT6_DT = np.dtype([("index", "<u2"), ("addr", "u1", 16), ("port", "<u2")])


def htons(x):
    x = np.asarray(x, dtype=np.uint32)
    return (((x & 0xFF) << 8) | ((x >> 8) & 0xFF)).astype(np.uint16)


def ntohs(x):
    return htons(x)


def ip4(s: str) -> int:
    """'10.0.0.1' -> be32 raw (little-endian load of network bytes)."""
    b = bytes(int(p) for p in s.split("."))
    return int.from_bytes(b, "little")


def be32_to_bytes(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a.astype("<u4")).view(np.uint8).reshape(-1, 4)


def mask_be32(plen: np.ndarray) -> np.ndarray:
    """Network-order prefix mask as a be32-raw u32 (GET_PREFIX, ipv6.h:136)."""
    plen = np.asarray(plen, dtype=np.uint64)
    host = np.where(plen == 0, 0, (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF)
    return byteswap32(host.astype(np.uint32))


def byteswap32(x):
    x = np.asarray(x, dtype=np.uint32)
    return (((x & 0xFF) << 24) | ((x & 0xFF00) << 8) | ((x >> 8) & 0xFF00)
            | (x >> 24)).astype(np.uint32)


@dataclasses.dataclass
class Tables:
    ipcache: np.ndarray                      # IPCACHE_DT
    endpoints: np.ndarray                    # ENDPOINT_DT
    policy: dict                             # lxc_id -> POLICY_DT array
    prefilter: np.ndarray                    # PREFILTER_DT
    seclabel: dict                           # lxc_id -> u32 (endpoint SECLABEL)
    ct: np.ndarray = None                    # CT_DT pre-populated conntrack
    # node_config.h (IPV4_CLUSTER_RANGE, IPV4_CLUSTER_MASK, ROUTER_IP); None =
    # the reference's compiled-in values
    node: tuple = None
    lb4: np.ndarray = None                   # LB4_DT service / backend slots
    revnat4: np.ndarray = None               # REVNAT4_DT


@dataclasses.dataclass
class Headers:
    family: int                              # 4 or 6 (whole batch)
    saddr: np.ndarray                        # v4: (n,) <u4 be32 raw; v6: (n,16) u8
    daddr: np.ndarray
    sport: np.ndarray                        # (n,) <u2 be16 raw
    dport: np.ndarray
    proto: np.ndarray                        # (n,) u1
    flags: np.ndarray                        # (n,) u1 HF_*
    length: np.ndarray                       # (n,) <u2 skb->len
    mark: np.ndarray                         # (n,) <u4 skb->mark
    # (n,) u1 TCP header byte 13 (the flag bits ct_lookup accumulates into
    # the CT entry's seen flags, conntrack.h:137-185); None = the default
    # the packet builders use: FIN|ACK with HF_TCP_CLOSE, else SYN
    tcpflags: np.ndarray = None
    # (n,) <u4 skb->hash (what lb4_select_slave reduces modulo the backend
    # count, lb.h:158-190); None = the engine's flow hash (cfc.h)
    hash: np.ndarray = None

    def __len__(self):
        return len(self.proto)

    def slice(self, a, b):
        return Headers(self.family, self.saddr[a:b], self.daddr[a:b],
                       self.sport[a:b], self.dport[a:b], self.proto[a:b],
                       self.flags[a:b], self.length[a:b], self.mark[a:b],
                       None if self.tcpflags is None else self.tcpflags[a:b],
                       None if self.hash is None else self.hash[a:b])


def tcp_flags_of(h) -> np.ndarray:
    """TCP header byte 13 of every header (0 for other protocols)."""
    if h.tcpflags is not None:
        return np.asarray(h.tcpflags, np.uint8)
    tcp = np.asarray(h.proto) == IPPROTO_TCP
    close = (np.asarray(h.flags) & HF_TCP_CLOSE) != 0
    return np.where(tcp, np.where(close, 0x11, 0x02), 0).astype(np.uint8)


def _v4_entries(addr_be32, plen, label):
    n = len(addr_be32)
    e = np.zeros(n, IPCACHE_DT)
    e["family"] = 1
    e["plen"] = plen
    e["addr"][:, :4] = be32_to_bytes(addr_be32)
    e["label"] = label
    return e


def gen_ipcache_v4(rng, n, label_base=256, label_mod=16384,
                   lengths=((8, .01), (12, .02), (16, .07), (20, .10),
                            (24, .40), (28, .10), (32, .30))):
    """C2 ipcache: n unique IPv4 prefixes, length mix of SURVEY.md §8d."""
    ls = np.array([l for l, _ in lengths])
    ps = np.array([p for _, p in lengths], dtype=np.float64)
    ps /= ps.sum()
    out_a, out_l = [], []
    seen = set()
    need = n
    while need > 0:
        m = int(need * 1.3) + 16
        plen = rng.choice(ls, size=m, p=ps).astype(np.uint32)
        host = rng.integers(0, 1 << 32, size=m, dtype=np.uint64).astype(np.uint32)
        # keep away from 64.48.32.16 (LXC_IPV4) /8 and the 10/8 endpoint space
        top = host >> 24
        ok = (top != 10) & (top != 64) & (top != 0) & (top < 224)
        plen, host = plen[ok], host[ok]
        hmask = np.where(plen == 0, 0,
                         (np.uint64(0xFFFFFFFF) << (32 - plen.astype(np.uint64)))
                         & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        host &= hmask
        for h, l in zip(host.tolist(), plen.tolist()):
            if (h, l) in seen:
                continue
            seen.add((h, l))
            out_a.append(h)
            out_l.append(l)
            need -= 1
            if need == 0:
                break
    host = np.array(out_a, dtype=np.uint32)
    plen = np.array(out_l, dtype=np.uint8)
    label = (label_base + (np.arange(n) % label_mod)).astype(np.uint32)
    return _v4_entries(byteswap32(host), plen, label)


# ------------------------------------------------------------------ IPv6
def ip6(s: str) -> np.ndarray:
    """'beef::1' -> 16 network-order bytes."""
    import ipaddress
    return np.frombuffer(ipaddress.IPv6Address(s).packed, np.uint8).copy()


LXC_IPV6 = np.array([0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x01, 0x01, 0x65,
                     0x82, 0xbc], np.uint8)        # bpf/lxc_config.h LXC_IP
ROUTER_IPV6 = np.array([0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 0],
                       np.uint8)                   # bpf/node_config.h ROUTER_IP


def mask_v6(addrs: np.ndarray, plen) -> np.ndarray:
    """Clear the bits past plen of (m,16) network-order addresses
    (ipv6_addr_clear_suffix, ipv6.h:140-150)."""
    addrs = np.asarray(addrs, np.uint8).reshape(-1, 16)
    plen = np.broadcast_to(np.asarray(plen, np.int64), (len(addrs),))
    bit = np.arange(16)[None, :] * 8
    keep = np.clip(plen[:, None] - bit, 0, 8)
    m = (0xFF << (8 - keep)) & 0xFF
    return (addrs & m.astype(np.uint8)).astype(np.uint8)


def _v6_entries(addrs, plen, label):
    n = len(addrs)
    e = np.zeros(n, IPCACHE_DT)
    e["family"] = 2
    e["plen"] = plen
    e["addr"] = mask_v6(addrs, plen)
    e["label"] = label
    return e


def gen_ipcache_v6(rng, n, label_base=256, label_mod=16384,
                   lengths=((32, .02), (40, .03), (48, .30), (56, .20),
                            (64, .25), (96, .05), (128, .15))):
    """C3 ipcache: n unique IPv6 prefixes, mass at /48, /56, /64 and /128
    (SURVEY.md §8d), inside 2000::/4 and away from the node's beef::/16."""
    ls = np.array([l for l, _ in lengths])
    ps = np.array([p for _, p in lengths], dtype=np.float64)
    ps /= ps.sum()
    out_a, out_l, seen = [], [], set()
    need = n
    while need > 0:
        m = int(need * 1.2) + 16
        plen = rng.choice(ls, size=m, p=ps)
        a = rng.integers(0, 256, size=(m, 16), dtype=np.uint16).astype(np.uint8)
        a[:, 0] = 0x20 | (a[:, 0] & 0x0F)
        a = mask_v6(a, plen)
        for row, l in zip(a, plen.tolist()):
            k = (row.tobytes(), l)
            if k in seen:
                continue
            seen.add(k)
            out_a.append(row)
            out_l.append(l)
            need -= 1
            if need == 0:
                break
    addrs = np.stack(out_a)
    label = (label_base + (np.arange(n) % label_mod)).astype(np.uint32)
    return _v6_entries(addrs, np.array(out_l, np.uint8), label)


def endpoint_v6(addr16, ifindex, lxc_id, flags=0):
    e = np.zeros(1, ENDPOINT_DT)
    e["family"] = 2
    e["addr"][0] = np.asarray(addr16, np.uint8)
    e["ifindex"] = ifindex
    e["lxc_id"] = lxc_id
    e["flags"] = flags
    return e


def _addr_in_prefix_v6(rng, ipc, idx):
    base = ipc["addr"][idx]
    plen = ipc["plen"][idx].astype(np.int64)
    rnd = rng.integers(0, 256, size=(len(idx), 16), dtype=np.uint16).astype(np.uint8)
    host = rnd & ~mask_v6(np.full((len(idx), 16), 0xFF, np.uint8), plen)
    return (base | host).astype(np.uint8)


ICMP6_TYPES = np.array([128, 128, 129, 1, 3, 136], np.uint32)


def gen_headers_v6(rng, n, ipc, dst_addrs, in_prefix=0.9, local_frac=0.97,
                   ports=None, ext=0.01, exthdr_drop=0.005,
                   mark_host=0.03, mark_proxy=0.02, other_proto=0.005,
                   proxy_ident=None, src_fixed=None, icmp_types=ICMP6_TYPES):
    """IPv6 header batch, the C3 analogue of gen_headers_v4.  `proto` is the
    next header ipv6_hdrlen() stops at: a fraction `exthdr_drop` stops at
    FRAGMENT (44) or NONE (59), which the datapath drops."""
    ports = PORT_SET if ports is None else ports
    if src_fixed is not None:
        saddr = np.tile(np.asarray(src_fixed, np.uint8), (n, 1))
    else:
        pick = rng.integers(0, len(ipc), size=n)
        saddr = _addr_in_prefix_v6(rng, ipc, pick)
        uni = rng.random(n) >= in_prefix
        saddr[uni] = rng.integers(0, 256, size=(int(uni.sum()), 16),
                                  dtype=np.uint16).astype(np.uint8)
    dst_addrs = np.asarray(dst_addrs, np.uint8).reshape(-1, 16)
    daddr = dst_addrs[rng.integers(0, len(dst_addrs), size=n)].copy()
    nonlocal_ = rng.random(n) >= local_frac
    daddr[nonlocal_] = rng.integers(0, 256, size=(int(nonlocal_.sum()), 16),
                                    dtype=np.uint16).astype(np.uint8)
    r = rng.random(n)
    proto = np.where(r < 0.70, IPPROTO_TCP,
                     np.where(r < 0.95, IPPROTO_UDP, IPPROTO_ICMPV6)).astype(np.uint8)
    oth = rng.random(n) < other_proto
    proto[oth] = rng.choice(np.array([47, 132, 50], np.uint8), size=int(oth.sum()))
    dr = rng.random(n) < exthdr_drop
    proto[dr] = rng.choice(np.array([44, 59], np.uint8), size=int(dr.sum()))
    dp = np.where(rng.random(n) < 0.6, rng.choice(ports, size=n),
                  rng.integers(1, 65536, size=n)).astype(np.uint32)
    sp = rng.integers(32768, 65536, size=n).astype(np.uint32)
    sport, dport = htons(sp), htons(dp)
    icmp = proto == IPPROTO_ICMPV6
    sport[icmp] = rng.choice(np.asarray(icmp_types, np.uint32),
                             size=int(icmp.sum())).astype(np.uint16)
    dport[icmp] = rng.integers(0, 65536, size=int(icmp.sum())).astype(np.uint16)
    flags = np.zeros(n, np.uint8)
    flags[rng.random(n) < ext] |= HF_EXTHDR
    tcp = proto == IPPROTO_TCP
    flags[tcp & (rng.random(n) < 0.02)] |= HF_TCP_CLOSE
    length = rng.integers(100, 1501, size=n).astype(np.uint16)
    mark = np.zeros(n, np.uint32)
    rm = rng.random(n)
    mark[rm < mark_host] = 0xC00
    if proxy_ident is not None and len(proxy_ident):
        sel = (rm >= mark_host) & (rm < mark_host + mark_proxy)
        ids = rng.choice(np.asarray(proxy_ident, np.uint32), size=int(sel.sum()))
        magic = np.where(rng.random(int(sel.sum())) < 0.5, 0xA00, 0xB00)
        mark[sel] = ((ids & 0xFFFF) << 16) | ((ids >> 16) & 0xFF) | magic
    return Headers(6, saddr, daddr, sport, dport, proto, flags, length, mark)


def local_v6_addrs(t: Tables):
    e = t.endpoints[t.endpoints["family"] == 2]
    return e["addr"].copy()


def config_c3(seed=3, n_prefixes=1_000_000, n_v4_prefixes=100_000,
              n_policy=16384, n_endpoints=1, n_prefilter=50_000):
    """C3 (dual stack): 1M IPv6 /32-/128 ipcache prefixes next to C2's IPv4
    ones, endpoints with both addresses, and a 50k-entry prefilter (half v4
    /32, half v6 /128 exact entries)."""
    t = config_c2(seed, n_prefixes=n_v4_prefixes, n_policy=n_policy,
                  n_endpoints=n_endpoints)
    rng = np.random.default_rng(seed + 77)
    ipc6 = gen_ipcache_v6(rng, n_prefixes)
    t.ipcache = np.concatenate([t.ipcache, ipc6])
    eps = [endpoint_v6(LXC_IPV6, 100, EP_LXC_ID)]
    for i in range(1, n_endpoints):
        a = LXC_IPV6.copy()
        a[12:] = [0, 0, i >> 8, i & 255]
        eps.append(endpoint_v6(a, 100 + i, EP_LXC_ID + i))
    host = LXC_IPV6.copy()
    host[12:] = [0xff, 0xff, 0xff, 0xfe]
    eps.append(endpoint_v6(host, 0, 0xFFF0, flags=1))
    t.endpoints = np.concatenate([t.endpoints] + eps)
    half = n_prefilter // 2
    pf = np.zeros(n_prefilter, PREFILTER_DT)
    v4 = np.unique(rng.integers(1 << 24, 224 << 24, size=half,
                                dtype=np.uint64).astype(np.uint32))
    pf = pf[:len(v4) + (n_prefilter - half)]
    pf["family"][:len(v4)] = 1
    pf["plen"][:len(v4)] = 32
    pf["addr"][:len(v4), :4] = be32_to_bytes(byteswap32(v4))
    a6 = rng.integers(0, 256, size=(n_prefilter - half, 16),
                      dtype=np.uint16).astype(np.uint8)
    a6[:, 0] = 0x20 | (a6[:, 0] & 0x0F)
    pf["family"][len(v4):] = 2
    pf["plen"][len(v4):] = 128
    pf["addr"][len(v4):] = a6
    t.prefilter = pf
    return t


def headers_c3(t: Tables, n, seed=3, **kw):
    rng = np.random.default_rng(seed + 3000)
    ipc6 = t.ipcache[t.ipcache["family"] == 2]
    return gen_headers_v6(rng, n, ipc6, local_v6_addrs(t),
                          proxy_ident=proxy_identities(t), **kw)


def endpoint_v4(addr_be32, ifindex, lxc_id, flags=0):
    e = np.zeros(1, ENDPOINT_DT)
    e["family"] = 1
    e["addr"][0, :4] = be32_to_bytes(np.array([addr_be32], np.uint32))[0]
    e["ifindex"] = ifindex
    e["lxc_id"] = lxc_id
    e["flags"] = flags
    return e


PORT_SET = np.array([22, 25, 53, 80, 110, 123, 143, 389, 443, 445, 465, 587,
                     636, 853, 993, 995, 1433, 1521, 2049, 2379, 3000, 3306,
                     5000, 5432, 5672, 6379, 6443, 8000, 8080, 8443, 9090,
                     9200], dtype=np.uint32)
PROXY_PORTS = np.array([10001, 10002, 10003, 10004], dtype=np.uint32)


def gen_policy(rng, n, identities, ports=PORT_SET, l3_frac=0.5,
               wildcard=8, proxy_frac=0.05, both_dirs=True):
    """C2 policymap: n unique keys (half L3 {id,0,0,dir}, half L4
    {id,port,proto,dir}), a few wildcard-port keys {0,port,proto,dir} and
    some proxy redirects."""
    keys = set()
    rows = []
    identities = np.asarray(identities, dtype=np.uint32)
    # wildcard-port entries first (policy.h:85-96 fallback)
    for _ in range(wildcard):
        p = int(rng.choice(ports))
        pr = int(rng.choice([IPPROTO_TCP, IPPROTO_UDP]))
        d = int(rng.integers(0, 2)) if both_dirs else 0
        k = (0, int(htons(p)), pr, d)
        if k not in keys:
            keys.add(k)
            rows.append(k + (0,))
    while len(rows) < n:
        ident = int(rng.choice(identities))
        d = int(rng.integers(0, 2)) if both_dirs else 0
        if rng.random() < l3_frac:
            k = (ident, 0, 0, d)
        else:
            p = int(rng.choice(ports))
            pr = IPPROTO_TCP if rng.random() < 0.75 else IPPROTO_UDP
            k = (ident, int(htons(p)), pr, d)
        if k in keys:
            continue
        keys.add(k)
        proxy = 0
        if k[1] != 0 and rng.random() < proxy_frac:
            proxy = int(htons(int(rng.choice(PROXY_PORTS))))
        rows.append(k + (proxy,))
    out = np.zeros(len(rows), POLICY_DT)
    a = np.array(rows, dtype=np.int64)
    out["identity"], out["dport"], out["proto"] = a[:, 0], a[:, 1], a[:, 2]
    out["egress"], out["proxy_port"] = a[:, 3], a[:, 4]
    return out


def _addr_in_prefix_v4(rng, ipc, idx):
    """Random address inside prefix idx (be32 raw)."""
    base = byteswap32(ipc["addr"][idx, :4].copy().view("<u4").ravel())
    plen = ipc["plen"][idx].astype(np.uint64)
    hostbits = (rng.integers(0, 1 << 32, size=len(idx), dtype=np.uint64)
                & ((np.uint64(1) << (np.uint64(32) - plen)) - np.uint64(1)))
    return byteswap32((base.astype(np.uint64) | hostbits).astype(np.uint32))


def gen_headers_v4(rng, n, ipc, dst_addrs, in_prefix=0.9, local_frac=0.97,
                   ports=PORT_SET, frag=0.01, mark_host=0.03, mark_proxy=0.02,
                   other_proto=0.005, proxy_ident=None, src_fixed=None):
    """IPv4 header batch.  src: `in_prefix` inside a random ipcache prefix,
    rest uniform (WORLD); dst: a local endpoint with prob `local_frac`."""
    if src_fixed is not None:
        saddr = np.full(n, src_fixed, np.uint32)
    else:
        pick = rng.integers(0, len(ipc), size=n)
        saddr = _addr_in_prefix_v4(rng, ipc, pick)
        uni = rng.random(n) >= in_prefix
        saddr[uni] = rng.integers(0, 1 << 32, size=int(uni.sum()),
                                  dtype=np.uint64).astype(np.uint32)
    dst_addrs = np.asarray(dst_addrs, dtype=np.uint32)
    daddr = dst_addrs[rng.integers(0, len(dst_addrs), size=n)]
    nonlocal_ = rng.random(n) >= local_frac
    daddr[nonlocal_] = rng.integers(0, 1 << 32, size=int(nonlocal_.sum()),
                                    dtype=np.uint64).astype(np.uint32)
    r = rng.random(n)
    proto = np.where(r < 0.70, IPPROTO_TCP,
                     np.where(r < 0.95, IPPROTO_UDP, IPPROTO_ICMP)).astype(np.uint8)
    oth = rng.random(n) < other_proto
    proto[oth] = rng.choice(np.array([47, 132, 50], np.uint8), size=int(oth.sum()))
    # ports: 60% from the policy port set, 40% uniform
    dp = np.where(rng.random(n) < 0.6, rng.choice(ports, size=n),
                  rng.integers(1, 65536, size=n)).astype(np.uint32)
    sp = rng.integers(32768, 65536, size=n).astype(np.uint32)
    sport, dport = htons(sp), htons(dp)
    icmp = proto == IPPROTO_ICMP
    itype = rng.choice(np.array([0, 8, 8, 8, 3, 11, 13], np.uint32),
                       size=int(icmp.sum()))
    sport[icmp] = itype.astype(np.uint16)          # bytes [type, code=0]
    dport[icmp] = rng.integers(0, 65536, size=int(icmp.sum())).astype(np.uint16)
    flags = np.zeros(n, np.uint8)
    flags[rng.random(n) < frag] |= HF_FRAG
    tcp = proto == IPPROTO_TCP
    flags[tcp & (rng.random(n) < 0.02)] |= HF_TCP_CLOSE
    minlen = np.where(proto == IPPROTO_TCP, 54,
                      np.where(proto == IPPROTO_UDP, 42, 42)).astype(np.uint32)
    length = np.maximum(rng.integers(60, 1501, size=n), minlen).astype(np.uint16)
    mark = np.zeros(n, np.uint32)
    rm = rng.random(n)
    mark[rm < mark_host] = 0xC00                              # MARK_MAGIC_HOST
    if proxy_ident is not None and len(proxy_ident):
        sel = (rm >= mark_host) & (rm < mark_host + mark_proxy)
        ids = rng.choice(np.asarray(proxy_ident, np.uint32), size=int(sel.sum()))
        magic = np.where(rng.random(int(sel.sum())) < 0.5, 0xA00, 0xB00)
        # identity = ((mark & 0xFF) << 16) | mark >> 16  (common.h get_identity_via_proxy)
        mark[sel] = ((ids & 0xFFFF) << 16) | ((ids >> 16) & 0xFF) | magic
    return Headers(4, saddr, daddr, sport, dport, proto, flags, length, mark)


def ensure_no_reverse(h: Headers):
    """Drop headers whose reverse 5-tuple appeared earlier (CT_REPLY would
    change the verdict: SURVEY.md §8c 'Streams must avoid intra-batch
    reverse packets').  Returns a boolean keep-mask."""
    fwd = {}
    keep = np.ones(len(h), bool)
    if h.saddr.ndim == 2:    # IPv6: (n, 16) bytes
        s = [bytes(a) for a in h.saddr]
        d = [bytes(a) for a in h.daddr]
    else:
        s, d = h.saddr.tolist(), h.daddr.tolist()
    sp, dp, pr = h.sport.tolist(), h.dport.tolist(), h.proto.tolist()
    for i in range(len(h)):
        if (d[i], s[i], dp[i], sp[i], pr[i]) in fwd:
            keep[i] = False
            continue
        fwd[(s[i], d[i], sp[i], dp[i], pr[i])] = 1
    return keep


# ---------------------------------------------------------------- configs
LXC_IPV4 = ip4("64.48.32.16")       # bpf/lxc_config.h LXC_IPV4 0x10203040
EP_LXC_ID = 0x1010                  # bpf/lxc_config.h LXC_ID
EP_SECLABEL = 2                     # bpf/node_config.h SECLABEL


def config_c2(seed=2, n_prefixes=100_000, n_policy=16384, n_endpoints=1):
    """C2 tables: 100k IPv4 prefixes + 16k-entry policymap for one endpoint
    (SURVEY.md §8d).  Endpoint 0 is the reference's own LXC (64.48.32.16,
    LXC_ID 0x1010); a host endpoint (ENDPOINT_F_HOST) is added too."""
    rng = np.random.default_rng(seed)
    ipc = gen_ipcache_v4(rng, n_prefixes)
    eps = [endpoint_v4(LXC_IPV4, 100, EP_LXC_ID)]
    for i in range(1, n_endpoints):
        eps.append(endpoint_v4(ip4(f"10.1.{i >> 8}.{i & 255}"), 100 + i,
                               EP_LXC_ID + i))
    eps.append(endpoint_v4(ip4("10.0.255.254"), 0, 0xFFF0, flags=1))  # host
    eps = np.concatenate(eps)
    idents = np.unique(ipc["label"])
    pol = {}
    for e in eps:
        if e["flags"] & 1:
            continue
        pol[int(e["lxc_id"])] = gen_policy(rng, n_policy, idents)
    pf = np.zeros(0, PREFILTER_DT)
    seclabel = {int(e["lxc_id"]): EP_SECLABEL for e in eps}
    return Tables(ipc, eps, pol, pf, seclabel)


def local_v4_addrs(t: Tables):
    e = t.endpoints[t.endpoints["family"] == 1]
    return e["addr"][:, :4].copy().view("<u4").ravel()


def proxy_identities(t: Tables):
    return np.unique(t.ipcache["label"])[:64]


def headers_c2(t: Tables, n, seed=2, **kw):
    rng = np.random.default_rng(seed + 1000)
    return gen_headers_v4(rng, n, t.ipcache, local_v4_addrs(t),
                          proxy_ident=proxy_identities(t), **kw)


# ------------------------------------------------------- device generator
def gen_batch_v4_torch(t: Tables, n, seed, device, in_prefix=0.9,
                       local_frac=0.97, deny_frac=0.02, frag=0.01):
    """C2/C4 header batch generated directly on the GPU in the packed SoA
    form of cfc_hdr_v4 (saddr, daddr, ports, meta), same distribution as
    gen_headers_v4: 90% sources inside a random ipcache
    prefix, the rest uniform; 97% destinations on a local endpoint; TCP 70% /
    UDP 25% / ICMP 5% (+0.5% other protocols); 60% of dports from the policy
    port set; 1% fragments; len U[60,1500].  `deny_frac` of the sources are
    taken from the prefilter's /32 deny set when one is configured."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    i64 = torch.int64

    def rint(lo, hi, size=n):
        return torch.randint(lo, hi, (size,), generator=g, device=device, dtype=i64)

    def rnd(size=n):
        return torch.rand((size,), generator=g, device=device)

    def bswap(x):
        return (((x & 0xFF) << 24) | ((x & 0xFF00) << 8) | ((x >> 8) & 0xFF00)
                | ((x >> 24) & 0xFF))

    ipc = t.ipcache[t.ipcache["family"] == 1]
    base = torch.from_numpy(byteswap32(ipc["addr"][:, :4].copy().view("<u4")
                                       .ravel()).astype(np.int64)).to(device)
    plen = torch.from_numpy(ipc["plen"].astype(np.int64)).to(device)
    pick = rint(0, len(ipc))
    host = base[pick] | (rint(0, 1 << 32) & ((1 << (32 - plen[pick])) - 1))
    host = torch.where(rnd() < in_prefix, host, rint(0, 1 << 32))
    pf = t.prefilter
    fix = pf[(pf["family"] == 1) & (pf["dyn"] == 0) & (pf["plen"] == 32)] if len(pf) else pf
    if len(fix) and deny_frac > 0:
        deny = torch.from_numpy(byteswap32(fix["addr"][:, :4].copy().view("<u4")
                                           .ravel()).astype(np.int64)).to(device)
        host = torch.where(rnd() < deny_frac, deny[rint(0, len(fix))], host)
    saddr = bswap(host)
    eps = t.endpoints[(t.endpoints["family"] == 1) & ((t.endpoints["flags"] & 1) == 0)]
    loc = torch.from_numpy(eps["addr"][:, :4].copy().view("<u4").ravel()
                           .astype(np.int64)).to(device)
    daddr = torch.where(rnd() < local_frac, loc[rint(0, len(loc))],
                        rint(0, 1 << 32))
    r = rnd()
    proto = torch.where(r < 0.70, 6, torch.where(r < 0.95, 17, 1))
    proto = torch.where(rnd() < 0.005, 47, proto)
    ports_set = torch.from_numpy(PORT_SET.astype(np.int64)).to(device)
    dp = torch.where(rnd() < 0.6, ports_set[rint(0, len(PORT_SET))], rint(1, 65536))
    sp = rint(32768, 65536)

    def hs(x):
        return ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)
    ports = hs(sp) | (hs(dp) << 16)
    itype = torch.tensor([0, 8, 8, 8, 3, 11, 13], device=device, dtype=i64)[rint(0, 7)]
    ports = torch.where(proto == 1, itype | (rint(0, 65536) << 16), ports)
    flags = (rnd() < frag).to(i64) * HF_FRAG
    flags |= ((proto == 6) & (rnd() < 0.02)).to(i64) * HF_TCP_CLOSE
    minlen = torch.where(proto == 6, 54, 42)
    length = torch.maximum(rint(60, 1501), minlen)
    meta = proto | (flags << 8) | (length << 16)

    def i32(x):
        return (x & 0xFFFFFFFF).to(torch.int64).sub_(
            ((x & 0xFFFFFFFF) >= (1 << 31)).to(i64) << 32).to(torch.int32)
    return i32(saddr), i32(daddr), i32(ports), i32(meta)


def unpack_v4(saddr, daddr, ports, meta, mark=None) -> Headers:
    """Packed numpy int32/uint32 SoA -> Headers (for the oracle)."""
    u = lambda a: np.ascontiguousarray(a).view(np.uint32)   # noqa: E731
    s, d, p, m = u(saddr), u(daddr), u(ports), u(meta)
    return Headers(4, s, d, (p & 0xFFFF).astype(np.uint16),
                   (p >> 16).astype(np.uint16), (m & 0xFF).astype(np.uint8),
                   ((m >> 8) & 0xFF).astype(np.uint8),
                   (m >> 16).astype(np.uint16),
                   u(mark) if mark is not None else np.zeros(len(s), np.uint32))


def config_c2_bench(seed=2, n_prefilter=25_000):
    """The bench tables: C2 (100k prefixes, 16k-entry policymap) plus a
    production-shaped prefilter (fixed /32 deny-list only, dyn disabled as
    in pkg/policy/prefilter.go:282-289)."""
    t = config_c2(seed)
    rng = np.random.default_rng(seed + 500)
    host = np.unique(rng.integers(1 << 24, 224 << 24, size=n_prefilter,
                                  dtype=np.uint64).astype(np.uint32))
    pf = np.zeros(len(host), PREFILTER_DT)
    pf["family"] = 1
    pf["plen"] = 32
    pf["addr"][:, :4] = be32_to_bytes(byteswap32(host))
    t.prefilter = pf
    return t


# ------------------------------------------------------------ conntrack
def take(h: Headers, idx) -> Headers:
    return Headers(h.family, h.saddr[idx], h.daddr[idx], h.sport[idx],
                   h.dport[idx], h.proto[idx], h.flags[idx], h.length[idx],
                   h.mark[idx], None if h.tcpflags is None else h.tcpflags[idx],
                   None if h.hash is None else h.hash[idx])


def concat(hs) -> Headers:
    f = hs[0].family
    cat = lambda k: np.concatenate([getattr(h, k) for h in hs])   # noqa: E731
    tf = None
    if any(h.tcpflags is not None for h in hs):
        tf = np.concatenate([tcp_flags_of(h) for h in hs])
    hs_ = None
    if any(h.hash is not None for h in hs):
        hs_ = np.concatenate([h.hash if h.hash is not None
                              else np.zeros(len(h), np.uint32) for h in hs])
    return Headers(f, cat("saddr"), cat("daddr"), cat("sport"), cat("dport"),
                   cat("proto"), cat("flags"), cat("length"), cat("mark"), tf, hs_)


def reverse(h: Headers) -> Headers:
    """The packets travelling the other way: addresses and L4 ports swapped,
    ICMP echo requests answered by echo replies (type 0 / 129)."""
    icmp = h.proto == (IPPROTO_ICMP if h.family == 4 else IPPROTO_ICMPV6)
    echo, reply = (8, 0) if h.family == 4 else (128, 129)
    sport = np.where(icmp, h.sport, h.dport).astype(np.uint16)
    dport = np.where(icmp, h.dport, h.sport).astype(np.uint16)
    sport[icmp & ((h.sport & 0xFF) == echo)] = reply
    return Headers(h.family, h.daddr.copy(), h.saddr.copy(), sport, dport,
                   h.proto.copy(), (h.flags & np.uint8(0xFF ^ HF_TCP_CLOSE)).astype(np.uint8),
                   h.length.copy(), np.zeros(len(h), np.uint32))


CT_ROW = 104


def ct_from_rows(rows: np.ndarray) -> np.ndarray:
    """CT dump rows (u16 owner = lxc_id + 1 or 0 for the global maps,
    u8 map (0 TCP / 1 ANY), u8 family, tuple[40], ct_entry[56], pad[4]) ->
    CT_DT records."""
    rows = np.asarray(rows, np.uint8).reshape(-1, CT_ROW)
    ct = np.zeros(len(rows), CT_DT)
    owner = rows[:, 0].astype(np.int32) | (rows[:, 1].astype(np.int32) << 8)
    ct["lxc"] = owner - 1
    ct["any"] = rows[:, 2]
    ct["family"] = rows[:, 3]
    ct["tuple"] = rows[:, 4:42]
    ct["entry"] = rows[:, 44:100]
    return ct


def _zipf_ranks(rng, n_items, n, s=1.1):
    """n draws of ranks 0..n_items-1 with P(k) ~ 1 / (k + 1)^s."""
    w = 1.0 / np.power(np.arange(1, n_items + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, rng.random(n)), n_items - 1)


def ct_entries_v4(daddr, saddr, dport, sport, proto, flags, dir_ingress,
                  length, src_sec_id, lxc=-1, now=0):
    """CT_DT records of flows as ct_create4 writes them (conntrack.h:
    691-772) at clock `now` (bpf_ktime_get_sec): the flow's entry (tuple k2,
    rx or tx packets = 1, bytes = len, src_sec_id, lifetime now + 60 —
    CT_SYN_TIMEOUT / CT_LIFETIME_NONTCP — and the direction's report time)
    plus its ICMP 'related' entry ({daddr, saddr, 0, 0, ICMP, flags |
    TUPLE_F_RELATED}, seen_non_syn) in the same map."""
    n = len(daddr)
    tu = np.zeros((n, 38), np.uint8)
    tu[:, 0:4] = be32_to_bytes(byteswap32(np.asarray(daddr, np.uint32)))
    tu[:, 4:8] = be32_to_bytes(byteswap32(np.asarray(saddr, np.uint32)))
    tu[:, 8:10] = np.asarray(dport, np.uint16).view(np.uint8).reshape(n, 2)
    tu[:, 10:12] = np.asarray(sport, np.uint16).view(np.uint8).reshape(n, 2)
    tu[:, 12] = proto
    tu[:, 13] = flags
    ent = np.zeros((n, 56), np.uint8)
    ev = ent.view("<u8")[:, :4]
    one = np.ones(n, np.uint64)
    ev[:, 0] = np.where(dir_ingress, one, 0)
    ev[:, 1] = np.where(dir_ingress, length, 0)
    ev[:, 2] = np.where(dir_ingress, 0, one)
    ev[:, 3] = np.where(dir_ingress, 0, length)
    ent[:, 44:48] = np.asarray(src_sec_id, np.uint32).view(np.uint8).reshape(n, 4)
    ent[:, 32:36] = np.full(n, now + 60, np.uint32).view(np.uint8).reshape(n, 4)
    if now > 5:   # __ct_update_timeout: last_report + 5 < now (from 0)
        rep = np.full(n, now, np.uint32).view(np.uint8).reshape(n, 4)
        ing = np.asarray(dir_ingress, bool)
        ent[ing, 52:56] = rep[ing]       # last_rx_report
        ent[~ing, 48:52] = rep[~ing]     # last_tx_report
    ct = np.zeros(2 * n, CT_DT)
    ct["family"] = 1
    ct["lxc"] = lxc
    ct["any"][:n] = np.asarray(proto) != IPPROTO_TCP
    ct["any"][n:] = ct["any"][:n]
    ct["tuple"][:n] = tu
    rel = tu.copy()
    rel[:, 8:12] = 0
    rel[:, 12] = IPPROTO_ICMP
    rel[:, 13] = np.asarray(flags, np.uint8) | 2
    ct["tuple"][n:] = rel
    ct["entry"][:n] = ent
    ent2 = ent.copy()
    ent2[:, 36] = 16                                   # seen_non_syn
    ct["entry"][n:] = ent2
    # one entry per key (a later flow's related entry overwrites, like
    # map_update_elem)
    import pandas as pd
    tu = np.ascontiguousarray(ct["tuple"][:, :16])
    k0 = tu[:, :8].copy().view("<u8").ravel()
    k1 = (tu[:, 8:16].copy().view("<u8").ravel() & np.uint64((1 << 48) - 1)) | \
        (ct["any"].astype(np.uint64) << np.uint64(48))
    dup = pd.DataFrame({"a": k0, "b": k1}).duplicated(keep="last").to_numpy()
    return ct[~dup]


def config_c5(seed=5, n_flows=10_000_000, n_prefixes=100_000, n_policy=16384,
              n_prefilter=25_000, now=0):
    """C5: the C2 tables and prefilter plus n_flows live
    conntrack flows into / out of the endpoint (global CT maps), half opened
    from outside (ingress-created, TUPLE_F_IN) and half by the endpoint
    (egress-created, TUPLE_F_OUT); TCP 70% / UDP 30%.  Returns (tables,
    flows) where flows holds each flow's inbound header fields."""
    t = config_c2_bench(seed, n_prefilter=n_prefilter) if n_prefixes == 100_000 \
        else config_c2(seed, n_prefixes=n_prefixes, n_policy=n_policy)
    rng = np.random.default_rng(seed + 501)
    ipc = t.ipcache[t.ipcache["family"] == 1]
    r_addr = _addr_in_prefix_v4(rng, ipc, rng.integers(0, len(ipc), size=n_flows))
    c_addr = np.full(n_flows, LXC_IPV4, np.uint32)
    proto = np.where(rng.random(n_flows) < 0.7, IPPROTO_TCP, IPPROTO_UDP).astype(np.uint8)
    inbound = rng.random(n_flows) < 0.5            # opened from outside
    svc = htons(rng.choice(PORT_SET, size=n_flows).astype(np.uint32))
    eph = htons(rng.integers(1024, 65536, size=n_flows).astype(np.uint32))
    # inbound packet of the flow: r -> c.  Ingress-created: (eph -> svc);
    # egress-created reply: remote service port -> the endpoint's eph port
    sport = np.where(inbound, eph, svc).astype(np.uint16)
    dport = np.where(inbound, svc, eph).astype(np.uint16)
    length = rng.integers(60, 1501, size=n_flows).astype(np.uint64)
    # ct_create4 keys: ingress-created k2 = {r, c, dport, sport, IN};
    # egress-created (pkt c -> r, sport=eph, dport=svc):
    # k2 = {c, r, svc, eph, OUT}
    d = np.where(inbound, r_addr, c_addr)
    s = np.where(inbound, c_addr, r_addr)
    kd = np.where(inbound, dport, sport)
    ks = np.where(inbound, sport, dport)
    sec = np.where(inbound, rng.integers(256, 256 + 16384, size=n_flows),
                   EP_SECLABEL).astype(np.uint32)
    t.ct = ct_entries_v4(byteswap32(d), byteswap32(s), kd, ks, proto,
                         np.where(inbound, 1, 0).astype(np.uint8), inbound,
                         length, sec, now=now)
    flows = Headers(4, r_addr, c_addr, sport, dport, proto,
                    np.zeros(n_flows, np.uint8), length.astype(np.uint16),
                    np.zeros(n_flows, np.uint32))
    return t, flows


def ct_entries_v6(daddr, saddr, dport, sport, proto, flags, dir_ingress,
                  length, src_sec_id, rev_nat, lxc=-1, now=0):
    """CT_DT records of IPv6 flows as ct_create6 writes them (conntrack.h:
    615-662): as ct_entries_v4, 16-byte addresses, rev_nat_index (ipv6_policy
    sets it from daddr.s6_addr32[3] for flows it creates, bpf_lxc.c:787-788)
    and an ICMPv6 related entry."""
    n = len(daddr)
    tu = np.zeros((n, 38), np.uint8)
    tu[:, 0:16] = np.asarray(daddr, np.uint8).reshape(n, 16)
    tu[:, 16:32] = np.asarray(saddr, np.uint8).reshape(n, 16)
    tu[:, 32:34] = np.asarray(dport, np.uint16).view(np.uint8).reshape(n, 2)
    tu[:, 34:36] = np.asarray(sport, np.uint16).view(np.uint8).reshape(n, 2)
    tu[:, 36] = proto
    tu[:, 37] = flags
    ent = np.zeros((n, 56), np.uint8)
    ev = ent.view("<u8")[:, :4]
    one = np.ones(n, np.uint64)
    ev[:, 0] = np.where(dir_ingress, one, 0)
    ev[:, 1] = np.where(dir_ingress, length, 0)
    ev[:, 2] = np.where(dir_ingress, 0, one)
    ev[:, 3] = np.where(dir_ingress, 0, length)
    ent[:, 38:40] = np.asarray(rev_nat, np.uint16).view(np.uint8).reshape(n, 2)
    ent[:, 44:48] = np.asarray(src_sec_id, np.uint32).view(np.uint8).reshape(n, 4)
    ent[:, 32:36] = np.full(n, now + 60, np.uint32).view(np.uint8).reshape(n, 4)
    if now > 5:
        rep = np.full(n, now, np.uint32).view(np.uint8).reshape(n, 4)
        ing = np.asarray(dir_ingress, bool)
        ent[ing, 52:56] = rep[ing]
        ent[~ing, 48:52] = rep[~ing]
    ct = np.zeros(2 * n, CT_DT)
    ct["family"] = 2
    ct["lxc"] = lxc
    ct["any"][:n] = np.asarray(proto) != IPPROTO_TCP
    ct["any"][n:] = ct["any"][:n]
    ct["tuple"][:n] = tu
    rel = tu.copy()
    rel[:, 32:36] = 0
    rel[:, 36] = IPPROTO_ICMPV6
    rel[:, 37] = np.asarray(flags, np.uint8) | 2
    ct["tuple"][n:] = rel
    ct["entry"][:n] = ent
    ent2 = ent.copy()
    ent2[:, 36] = 16                                   # seen_non_syn
    ct["entry"][n:] = ent2
    import pandas as pd
    key = np.ascontiguousarray(ct["tuple"]).view(np.dtype((np.void, 38))).ravel()
    df = pd.DataFrame({"k": [bytes(k) for k in key], "a": ct["any"]})
    return ct[~df.duplicated(keep="last").to_numpy()]


def config_c5_v6(seed=6, n_flows=300_000, n_prefixes=100_000, n_policy=16384, now=0):
    """The C5 shape for IPv6: C3's tables (n_prefixes IPv6 ipcache prefixes,
    no prefilter) plus n_flows live flows into / out of the endpoint's IPv6
    address in the global CT6 maps, half opened from outside, TCP 70% /
    UDP 30%.  Returns (tables, flows) as config_c5."""
    t = config_c3(seed, n_prefixes=n_prefixes, n_v4_prefixes=1000, n_policy=n_policy,
                  n_prefilter=0)
    rng = np.random.default_rng(seed + 601)
    ipc = t.ipcache[t.ipcache["family"] == 2]
    r_addr = _addr_in_prefix_v6(rng, ipc, rng.integers(0, len(ipc), size=n_flows))
    c_addr = np.tile(LXC_IPV6, (n_flows, 1))
    proto = np.where(rng.random(n_flows) < 0.7, IPPROTO_TCP, IPPROTO_UDP).astype(np.uint8)
    inbound = rng.random(n_flows) < 0.5
    svc = htons(rng.choice(PORT_SET, size=n_flows).astype(np.uint32))
    eph = htons(rng.integers(1024, 65536, size=n_flows).astype(np.uint32))
    sport = np.where(inbound, eph, svc).astype(np.uint16)
    dport = np.where(inbound, svc, eph).astype(np.uint16)
    length = rng.integers(60, 1501, size=n_flows).astype(np.uint64)
    ib = inbound[:, None]
    d = np.where(ib, r_addr, c_addr)
    s = np.where(ib, c_addr, r_addr)
    kd = np.where(inbound, dport, sport)
    ks = np.where(inbound, sport, dport)
    sec = np.where(inbound, rng.integers(256, 256 + 16384, size=n_flows),
                   EP_SECLABEL).astype(np.uint32)
    # ingress-created entries: rev_nat_index from the packet's daddr (c)
    rev = np.where(inbound, c_addr[:, 12].astype(np.uint16) |
                   (c_addr[:, 13].astype(np.uint16) << 8), 0).astype(np.uint16)
    t.ct = ct_entries_v6(d, s, kd, ks, proto, np.where(inbound, 1, 0).astype(np.uint8),
                         inbound, length, sec, rev, now=now)
    flows = Headers(6, r_addr, c_addr, sport, dport, proto,
                    np.zeros(n_flows, np.uint8), length.astype(np.uint16),
                    np.zeros(n_flows, np.uint32))
    return t, flows


def headers_c5_v6(t: Tables, flows: Headers, n, seed=6, new_frac=0.05, s=1.1,
                  return_new=False):
    """IPv6 C5 stream: Zipf packets of live flows plus new flows (C3
    generator, every one to the endpoint).  return_new: also the mask of
    the new flows' headers."""
    rng = np.random.default_rng(seed + 777)
    m = int(n * (1 - new_frac))
    old = take(flows, _zipf_ranks(rng, len(flows), m, s))
    old.length = rng.integers(60, 1501, size=m).astype(np.uint16)
    ipc6 = t.ipcache[t.ipcache["family"] == 2]
    new = gen_headers_v6(rng, n - m, ipc6, local_v6_addrs(t)[:1], local_frac=1.0,
                         proxy_ident=proxy_identities(t))
    h = concat([old, new])
    perm = rng.permutation(n)
    if return_new:
        return take(h, perm), perm >= m
    return take(h, perm)


def headers_c5(t: Tables, flows: Headers, n, seed=5, new_frac=0.05, s=1.1,
               return_new=False, owner=None):
    """C5 stream into the endpoint: 95% packets of live flows drawn
    Zipf(s) by flow (ESTABLISHED for flows opened from outside, REPLY for
    flows the endpoint opened), 5% packets of new flows (C2 generator).
    return_new: also the mask of the new flows' headers.  owner = (rank,
    world): only new flows whose address pair that rank owns
    (distributed.pair_owner; flows should be the rank's own already)."""
    rng = np.random.default_rng(seed + 777)
    m = int(n * (1 - new_frac))
    pick = _zipf_ranks(rng, len(flows), m, s)
    old = take(flows, pick)
    old.length = rng.integers(60, 1501, size=m).astype(np.uint16)
    if owner is None or owner[1] == 1:
        new = gen_headers_v4(rng, n - m, t.ipcache, local_v4_addrs(t)[:1],
                             local_frac=1.0, proxy_ident=proxy_identities(t))
    else:
        from .distributed import addr_keys, pair_owner
        parts, got = [], 0
        while got < n - m:
            c = gen_headers_v4(rng, (n - m - got) * owner[1] * 5 // 4 + 1024, t.ipcache,
                               local_v4_addrs(t)[:1], local_frac=1.0,
                               proxy_ident=proxy_identities(t))
            keep = pair_owner(addr_keys(c.saddr, 4), addr_keys(c.daddr, 4),
                              owner[1]) == owner[0]
            c = take(c, np.flatnonzero(keep)[:n - m - got])
            parts.append(c)
            got += len(c)
        new = concat(parts)
    h = concat([old, new])
    perm = rng.permutation(n)
    if return_new:
        return take(h, perm), perm >= m
    return take(h, perm)


def headers_c5_seq(t: Tables, flows: Headers, n, seed=5, new_frac=0.08, s=1.1,
                   return_new=False):
    """C5 stream with the intra-batch conntrack dependencies a real batch
    holds (the reference applies each packet's CT writes before the next
    packet's lookup, conntrack.h:221-285, 615-772): 92% Zipf(s) packets of
    live flows (ACK / PSH-ACK, 2% FIN or RST; flows the policy now denies
    lose their entry to their first packet, bpf_lxc.c:963-970, and find
    none after), and new flows with several packets in order — SYN, then
    ACK and data, an ICMP error about a UDP flow, a FIN or RST, a packet
    after the close.  return_new: also the mask of the new flows' headers."""
    rng = np.random.default_rng(seed + 919)
    m = int(n * (1 - new_frac))
    old = take(flows, _zipf_ranks(rng, len(flows), m, s))
    old.length = rng.integers(60, 1501, size=m).astype(np.uint16)
    tf = rng.choice(np.array([0x10, 0x18], np.uint8), size=m)
    close = rng.random(m) < 0.02
    tf[close] = rng.choice(np.array([0x11, 0x04], np.uint8), size=int(close.sum()))
    old.flags[close] |= np.uint8(HF_TCP_CLOSE)
    old.tcpflags = np.where(old.proto == IPPROTO_TCP, tf, 0).astype(np.uint8)
    parts, pos = [old], [rng.random(m)]
    k = max(1, (n - m) // 3)
    base = gen_headers_v4(rng, k, t.ipcache, local_v4_addrs(t)[:1], local_frac=1.0,
                          mark_host=0, mark_proxy=0, other_proto=0, frag=0)
    # most new flows from identities the endpoint's policy admits on L3
    pol = t.policy[EP_LXC_ID]
    l3 = pol["identity"][(pol["dport"] == 0) & (pol["proto"] == 0) & (pol["egress"] == 0)]
    okp = np.flatnonzero(np.isin(t.ipcache["label"], l3) & (t.ipcache["family"] == 1))
    if len(okp):
        sel = np.flatnonzero(rng.random(k) < 0.8)
        base.saddr[sel] = _addr_in_prefix_v4(rng, t.ipcache, okp[rng.integers(0, len(okp),
                                                                              size=len(sel))])
    ic = base.proto == IPPROTO_ICMP
    base.sport[ic] = 8            # echo request
    base.dport[ic] = 0
    base.flags[:] = 0
    at = rng.random(k) * 0.9
    script = [(1.0, 0x02, False, False), (0.8, 0x10, False, False), (0.5, 0x18, False, False),
              (0.3, 0, False, True), (0.2, 0x11, True, False), (0.1, 0x10, False, False)]
    left = n - m
    for p_, f, cl, err in script:
        sel = np.flatnonzero(rng.random(k) < p_)
        if err:   # an ICMP error about a UDP flow (destination unreachable)
            sel = sel[base.proto[sel] == IPPROTO_UDP]
        sel = sel[:left]
        left -= len(sel)
        h = take(base, sel)
        h.length = rng.integers(60, 1501, size=len(h)).astype(np.uint16)
        if err:
            h.proto[:] = IPPROTO_ICMP
            h.sport[:] = 3
            h.dport[:] = 0
            h.tcpflags = np.zeros(len(h), np.uint8)
        else:
            h.tcpflags = np.where(h.proto == IPPROTO_TCP, f, 0).astype(np.uint8)
            if cl:
                h.flags[h.proto == IPPROTO_TCP] |= np.uint8(HF_TCP_CLOSE)
        parts.append(h)
        pos.append(at[sel])
        at = at + rng.random(k) * 0.01
    h = concat(parts)
    order = np.argsort(np.concatenate(pos), kind="stable")
    h = take(h, order)
    if return_new:
        isnew = np.concatenate([np.zeros(m, bool), np.ones(len(h) - m, bool)])[order]
        return h.slice(0, n), isnew[:n]
    return h.slice(0, n)


# ------------------------------------------------------------ C1
C1_POLICIES = "tests/golden/c1_policies.json"
C1_PORTS = np.array([80, 443, 53, 8080], dtype=np.uint32)
# label values the example policies select on (examples/policies/{l3,l4})
C1_LABELS = {"role": ["frontend", "backend", "crawler", "restricted", "public",
                      "victim", "db"],
             "app": ["myService", "test-app", "web"],
             "env": ["dev", "prod"],
             "app-type": ["dns"],
             "id": ["app2"]}
# the local endpoints: one per label set some example rule selects
C1_LOCAL = [{"role": "backend"}, {"app": "myService"}, {"role": "frontend"},
            {"role": "crawler"}, {"env": "prod", "role": "backend"},
            {"role": "public"}, {"role": "victim"}, {"env": "dev"},
            {"role": "restricted"}, {"id": "app2"}, {"app": "test-app"}]


def config_c1(seed=1, n_pods=100, policies=None):
    """C1 (BASELINE.json configs[0]): the MapState of every
    local endpoint under the example policies of examples/policies/{l3,l4}
    (cilium_amd.policy_resolver), ~100 pod identities 256-355 plus the
    reserved ones and one CIDR identity per prefix the rules name; ipcache:
    /32s of every pod (1-4 each) and local endpoint, plus the CIDR prefixes.
    Returns (tables, resolver context {identities, local labels})."""
    import os
    from . import policy_resolver as R
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    repo = R.Repository(R.load_fixture(policies or os.path.join(root, C1_POLICIES)))
    rng = np.random.default_rng(seed)
    pods = {}
    for i, lb in enumerate(C1_LOCAL):          # the local endpoints' identities
        pods[256 + i] = lb
    while len(pods) < n_pods:
        d = {}
        for k, vals in C1_LABELS.items():
            p = {"role": 0.85, "app": 0.5, "env": 0.6}.get(k, 0.08)
            if rng.random() < p:
                d[k] = str(rng.choice(vals))
        if d:
            pods[256 + len(pods)] = d
    pod_ids = {i: R.pod_labels(d) for i, d in pods.items()}
    cidrs = repo.cidrs()
    cidr_ids = {R.LOCAL_IDENTITY_FLAG + 1 + j: R.cidr_labels(c) for j, c in enumerate(cidrs)}
    idents = R.identity_cache(pod_ids, cidr_ids)
    # local endpoints: EP_LXC_ID first (the reference harness's own LXC)
    eps, pol, sec = [], {}, {}
    for i, lb in enumerate(C1_LOCAL):
        lxc = EP_LXC_ID if i == 0 else 0x2000 + i
        addr = LXC_IPV4 if i == 0 else ip4(f"10.0.1.{i}")
        eps.append(endpoint_v4(addr, 100 + i, lxc))
        ms = repo.map_state(R.pod_labels(lb), idents)
        rows = np.zeros(len(ms), POLICY_DT)
        for j, (k, proxy) in enumerate(sorted(ms.items())):
            rows[j] = (k[0], int(htons(k[1])), k[2], k[3], proxy)
        pol[lxc] = rows
        sec[lxc] = 256 + i
    eps.append(endpoint_v4(ip4("10.0.255.254"), 0, 0xFFF0, flags=1))   # host
    sec[0xFFF0] = EP_SECLABEL
    eps = np.concatenate(eps)
    # ipcache: pods' /32s (in 10.1.0.0/16 and 172.20.0.0/16), the local
    # endpoints, the CIDR prefixes with their CIDR identities
    a, l, ident = [], [], []
    for pid in range(256 + len(C1_LOCAL), 256 + len(pods)):
        for _ in range(int(rng.integers(1, 5))):
            base = ip4("10.1.0.0") if rng.random() < 0.7 else ip4("172.20.0.0")
            a.append(byteswap32(np.uint32(byteswap32(np.uint32(base)) +
                                          int(rng.integers(1, 65535)))))
            l.append(32)
            ident.append(pid)
    for e, lxc in zip(eps, [int(x) for x in eps["lxc_id"]]):
        if lxc in sec and lxc != 0xFFF0:
            a.append(e["addr"][:4].copy().view("<u4")[0])
            l.append(32)
            ident.append(sec[lxc])
    for j, c in enumerate(cidrs):
        net = c.split("/")
        a.append(ip4(net[0]))
        l.append(int(net[1]))
        ident.append(R.LOCAL_IDENTITY_FLAG + 1 + j)
    a = np.array(a, np.uint32)
    _, first = np.unique(np.stack([a, np.array(l)]), axis=1, return_index=True)
    first = np.sort(first)
    ipc = _v4_entries(a[first], np.array(l)[first], np.array(ident, np.uint32)[first])
    t = Tables(ipc, eps, pol, np.zeros(0, PREFILTER_DT), sec)
    return t, {"identities": idents, "local": C1_LOCAL}


def headers_c1(t: Tables, n, seed=1):
    """C1 stream: sources 90% inside an ipcache prefix,
    10% uniform; destinations the local endpoints (97%); dport from
    {80, 443, 53, 8080} (60%) or uniform; TCP 70% / UDP 25% / ICMP 5%;
    1% fragments; len U[60, 1500]."""
    rng = np.random.default_rng(seed + 1000)
    loc = local_v4_addrs(t)[:len(C1_LOCAL)]
    return gen_headers_v4(rng, n, t.ipcache, loc, ports=C1_PORTS, other_proto=0.0,
                          mark_host=0.02, mark_proxy=0.0)


# ------------------------------------------------------------ load balancing
SVC_NET = ip4("172.20.0.0")          # service VIPs: 172.20.x.y
IPV4_LOOPBACK = 0x1FFFF50A           # bpf/node_config.h:45


def lb4_services(rng, t: Tables, n_services=24, loopback=True, n_backend_pool=None):
    """Services for cilium_lb4_services (pkg/maps/lbmap shape): per service a
    master slot {vip, dport, slave 0} -> {count, rev_nat_index} and backend
    slots 1..count -> {target, port}.  Backends are remote addresses inside
    ipcache prefixes and the local endpoints; with loopback one service's
    backend is the endpoint itself (LXC_IPV4, lb4_local's loopback case).
    Edge services: an L3 service (dport 0: every port and ICMP), a service
    whose master has count 0 (not a service), one with a missing backend
    slot (the fall-back lookup, DROP_NO_SERVICE), and one whose missing slot
    the L3 fall-back key holds.  -> (LB4_DT, REVNAT4_DT, vips u32 array,
    ports be16 array per service, proto per service)."""
    ipc = t.ipcache[t.ipcache["family"] == 1]
    loc = local_v4_addrs(t)
    loc = loc[loc != LXC_IPV4]
    pool_n = n_backend_pool or 4 * n_services
    remote = _addr_in_prefix_v4(rng, ipc, rng.integers(0, len(ipc), size=pool_n))
    rows, rn = [], []
    vips = np.zeros(n_services, np.uint32)
    ports = np.zeros(n_services, np.uint16)
    protos = np.zeros(n_services, np.uint8)

    def row(addr, dport, slave, target=0, port=0, count=0, rev=0, weight=0):
        r = np.zeros(1, LB4_DT)
        r["addr"], r["dport"], r["slave"] = addr, dport, slave
        r["target"], r["port"], r["count"] = target, port, count
        r["rev_nat"], r["weight"] = rev, weight
        rows.append(r)

    for k in range(n_services):
        vip = (SVC_NET + ((k + 1) << 24)) & 0xFFFFFFFF   # 172.20.0.(k+1)
        vips[k] = vip
        protos[k] = IPPROTO_UDP if k % 4 == 3 else IPPROTO_TCP
        dp = htons(int(rng.choice(np.array([80, 443, 53, 8080, 9090]))))
        l3 = k == 1                                   # L3 service: dport 0
        ports[k] = 0 if l3 else dp
        key_dp = 0 if l3 else int(dp)
        rev = k + 1
        count = int(rng.integers(1, 5))
        if k == 2:
            count = 0                                 # not a service
        row(vip, key_dp, 0, count=count, rev=rev)
        rnr = np.zeros(1, REVNAT4_DT)
        rnr["index"], rnr["addr"], rnr["port"] = rev, vip, key_dp
        rn.append(rnr)
        for j in range(1, max(count, 1) + 1):
            if k == 4 and j == 2:
                continue                              # missing backend slot
            tgt = int(loc[j % len(loc)]) if (k % 5 == 0 and len(loc)) else \
                int(remote[(4 * k + j) % pool_n])
            if loopback and k == 6 and j == 1:
                tgt = LXC_IPV4
            port = int(htons(8000 + k)) if k % 3 == 0 else 0
            row(vip, key_dp, j, target=tgt, port=port, rev=rev)
        if k == 5 and count >= 2:
            # slot 2 lives only under the L3 key: lb4_lookup_slave misses,
            # the fall-back lb4_lookup_service finds {vip, 0, 2}
            rows = [r for r in rows if not (int(r["addr"][0]) == vip and
                                            int(r["slave"][0]) == 2)]
            row(vip, 0, 2, target=int(remote[0]), count=2, rev=rev)
    return (np.concatenate(rows), np.concatenate(rn), vips, ports, protos)


SVC6_NET = np.array([0xfd, 0x00, 0x5e, 0xc0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0], np.uint8)


def lb6_services(rng, t: Tables, n_services=24, n_backend_pool=None):
    """IPv6 services for cilium_lb6_services, the lb4_services shapes: per
    service a master slot {vip, dport, 0} -> {count, rev_nat_index} and
    backend slots 1..count; backends remote (inside IPv6 ipcache prefixes)
    or local endpoints; one service's backend is the sending endpoint itself
    (lb6_local has no loopback translation: the packet comes back to it);
    an L3 service, a count-0 master, a missing backend slot and one held
    under the L3 key.  -> (LB6_DT, REVNAT6_DT, vips (n, 16) u8, ports be16,
    protos)."""
    ipc = t.ipcache[t.ipcache["family"] == 2]
    loc = local_v6_addrs(t)
    loc = loc[~(loc == LXC_IPV6).all(1)]
    pool_n = n_backend_pool or 4 * n_services
    remote = _addr_in_prefix_v6(rng, ipc, rng.integers(0, len(ipc), size=pool_n))
    rows, rn = [], []
    vips = np.zeros((n_services, 16), np.uint8)
    ports = np.zeros(n_services, np.uint16)
    protos = np.zeros(n_services, np.uint8)

    def row(addr, dport, slave, target=None, port=0, count=0, rev=0, weight=0):
        r = np.zeros(1, LB6_DT)
        r["addr"][0], r["dport"], r["slave"] = addr, dport, slave
        if target is not None:
            r["target"][0] = target
        r["port"], r["count"], r["rev_nat"], r["weight"] = port, count, rev, weight
        rows.append(r)

    for k in range(n_services):
        vip = SVC6_NET.copy()
        vip[14], vip[15] = (k + 1) >> 8, (k + 1) & 255
        vips[k] = vip
        protos[k] = IPPROTO_UDP if k % 4 == 3 else IPPROTO_TCP
        dp = htons(int(rng.choice(np.array([80, 443, 53, 8080, 9090]))))
        l3 = k == 1
        ports[k] = 0 if l3 else dp
        key_dp = 0 if l3 else int(dp)
        rev = k + 1
        count = int(rng.integers(1, 5))
        if k == 2:
            count = 0
        row(vip, key_dp, 0, count=count, rev=rev)
        rnr = np.zeros(1, REVNAT6_DT)
        rnr["index"], rnr["addr"][0], rnr["port"] = rev, vip, key_dp
        rn.append(rnr)
        for j in range(1, max(count, 1) + 1):
            if k == 4 and j == 2:
                continue
            tgt = loc[j % len(loc)] if (k % 5 == 0 and len(loc)) else \
                remote[(4 * k + j) % pool_n]
            if k == 6 and j == 1:
                tgt = LXC_IPV6
            port = int(htons(8000 + k)) if k % 3 == 0 else 0
            row(vip, key_dp, j, target=tgt, port=port, rev=rev)
        if k == 5 and count >= 2:
            rows = [r for r in rows if not ((r["addr"][0] == vip).all() and
                                            int(r["slave"][0]) == 2)]
            row(vip, 0, 2, target=remote[0], count=2, rev=rev)
    # ipv6_policy stores daddr.s6_addr32[3] & 0xFFFF as the rev_nat_index of
    # the flows it creates (bpf_lxc.c:787-788) and reverse-NATs every later
    # hit whose index cilium_lb6_reverse_nat holds (:808-815): an entry under
    # the endpoint's own index exercises that
    rnr = np.zeros(1, REVNAT6_DT)
    rnr["index"] = int(LXC_IPV6[12]) | int(LXC_IPV6[13]) << 8
    rnr["addr"][0] = vips[0]
    rnr["port"] = 0
    rn.append(rnr)
    return (np.concatenate(rows), np.concatenate(rn), vips, ports, protos)


# ---- LXC_NAT46 (lxc_config.h:28, nat46.h:30-32) -----------------------------


def config_nat(seed=61, n_prefixes=2000, n_v4_prefixes=500, n_policy=300,
               n_endpoints=2):
    """Dual-stack tables for the NAT hops (oracle/gen_golden.py _nat_setup,
    same recipe): IPv4 peers reached from the endpoint's IPv6 side through
    ::ffff:0:0/96; EP_LXC_ID's egress policy admits WORLD (the IPv6 stage)
    and 70% of the IPv4 identities (the IPv4 stage after NAT64), its ingress
    policy half of them (the replies after NAT46); ::ffff:10.0.0.0/104 is
    CLUSTER_ID (not translated, bpf_lxc.c:353-354).  -> (tables, IPv4
    ipcache rows)"""
    t = config_c3(seed, n_prefixes=n_prefixes, n_v4_prefixes=n_v4_prefixes,
                  n_policy=n_policy, n_endpoints=n_endpoints, n_prefilter=0)
    rng = np.random.default_rng(seed + 1)
    cl = np.zeros(1, IPCACHE_DT)
    cl["family"] = 2
    cl["plen"] = 104
    cl["addr"][0, 10:13] = [0xff, 0xff, 10]
    cl["label"] = CLUSTER_ID
    t.ipcache = np.concatenate([t.ipcache, cl])
    ipc4 = t.ipcache[t.ipcache["family"] == 1]
    ids4 = np.unique(ipc4["label"])
    out_ok = rng.choice(ids4, size=int(0.7 * len(ids4)), replace=False)
    in_ok = rng.choice(ids4, size=int(0.5 * len(ids4)), replace=False)
    pol = t.policy[EP_LXC_ID]
    add = np.zeros(1 + len(out_ok) + len(in_ok), POLICY_DT)
    add["identity"][0] = WORLD_ID
    add["egress"][0] = 1
    add["identity"][1:1 + len(out_ok)] = out_ok
    add["egress"][1:1 + len(out_ok)] = 1
    add["identity"][1 + len(out_ok):] = in_ok
    have = {(int(r["identity"]), int(r["dport"]), int(r["proto"]), int(r["egress"]))
            for r in pol}
    add = add[[(int(r["identity"]), 0, 0, int(r["egress"])) not in have for r in add]]
    t.policy[EP_LXC_ID] = np.concatenate([pol, add])
    return t, ipc4


def v4_mapped(v4):
    """::ffff:a.b.c.d of raw be32 IPv4 addresses -> (n, 16) u8"""
    a = np.zeros((len(v4), 16), np.uint8)
    a[:, 10:12] = 0xff
    a[:, 12:16] = np.asarray(v4, np.uint32).view(np.uint8).reshape(-1, 4)
    return a


def nat64_flows(rng, ipc4, n, sport_base):
    """n new IPv6 flows from EP_LXC_ID to v4-mapped peers inside IPv4 ipcache
    prefixes: TCP 60% (SYN), UDP 25%, ICMPv6 echo 15%"""
    peers = _addr_in_prefix_v4(rng, ipc4, rng.integers(0, len(ipc4), size=n))
    r = rng.random(n)
    proto = np.where(r < 0.6, IPPROTO_TCP,
                     np.where(r < 0.85, IPPROTO_UDP, IPPROTO_ICMPV6)).astype(np.uint8)
    h = Headers(6, np.tile(LXC_IPV6, (n, 1)), v4_mapped(peers),
                htons((sport_base + np.arange(n)) & 0xFFFF),
                htons(rng.choice(np.array([80, 443, 53, 8080]), size=n)),
                proto, np.zeros(n, np.uint8),
                rng.integers(100, 1500, size=n).astype(np.uint16), np.zeros(n, np.uint32))
    ic = proto == IPPROTO_ICMPV6
    h.sport[ic] = 128      # echo request
    h.dport[ic] = htons((np.arange(int(ic.sum())) + 1) & 0xFFFF).astype(np.uint16)
    h.tcpflags = np.where(proto == IPPROTO_TCP, 0x02, 0).astype(np.uint8)
    return h


def headers_nat64(t, ipc4, hist, n, seed=61):
    """An IPv6 egress stream of EP_LXC_ID full of NAT64 (bpf_lxc.c:353-360):
    later packets of the history's flows, new flows with several packets
    (SYN, ACK, data, FIN), ICMPv6 errors of every icmp6_to_icmp4 outcome,
    extension headers (DROP_INVALID_EXTHDR), CLUSTER-mapped peers and plain
    IPv6 traffic, interleaved"""
    rng = np.random.default_rng(seed + 500)
    parts, pos = [], []

    def add(h, p):
        parts.append(h)
        pos.append(p)
    est = take(hist, rng.integers(0, len(hist), size=int(n * 0.35)))
    est.tcpflags = np.where(est.proto == IPPROTO_TCP,
                            rng.choice(np.array([0x10, 0x18], np.uint8), size=len(est)), 0
                            ).astype(np.uint8)
    est.length = rng.integers(100, 1500, size=len(est)).astype(np.uint16)
    add(est, rng.random(len(est)))
    new = nat64_flows(rng, ipc4, int(n * 0.1), 40000)
    at = rng.random(len(new)) * 0.9
    add(new, at)
    for f, p_ in ((0x10, 0.8), (0x18, 0.5), (0x11, 0.3)):
        sel = np.flatnonzero(rng.random(len(new)) < p_)
        h = take(new, sel)
        h.tcpflags = np.where(h.proto == IPPROTO_TCP, f, 0).astype(np.uint8)
        if f == 0x11:
            h.flags = np.where(h.proto == IPPROTO_TCP, HF_TCP_CLOSE, 0).astype(np.uint8)
        at = at + rng.random(len(new)) * 0.03
        add(h, at[sel])
    k = int(n * 0.08)
    e = nat64_flows(rng, ipc4, k, 50000)
    tc = np.array([[1, 0], [1, 3], [1, 4], [1, 1], [1, 7], [2, 0], [3, 0], [3, 1],
                   [4, 0], [4, 1], [4, 2], [137, 0]], np.uint16)
    pick = tc[rng.integers(0, len(tc), size=k)]
    e.proto[:] = IPPROTO_ICMPV6
    e.sport[:] = (pick[:, 0] | pick[:, 1] << 8).astype(np.uint16)
    e.dport[:] = 0
    e.tcpflags = np.zeros(k, np.uint8)
    add(e, rng.random(k))
    x = nat64_flows(rng, ipc4, int(n * 0.03), 60000)
    x.flags[:] |= np.uint8(HF_EXTHDR)
    add(x, rng.random(len(x)))
    c = nat64_flows(rng, ipc4, int(n * 0.04), 61000)
    c.daddr[:, 12] = 10
    add(c, rng.random(len(c)))
    plain = gen_headers_v6(rng, int(n * 0.1), t.ipcache[t.ipcache["family"] == 2],
                           local_v6_addrs(t), local_frac=0.3, mark_host=0,
                           mark_proxy=0, src_fixed=LXC_IPV6, ext=0, exthdr_drop=0)
    add(plain, rng.random(len(plain)))
    h = concat(parts)
    h = take(h, np.argsort(np.concatenate(pos), kind="stable"))
    return h.slice(0, n)


def headers_nat46(t, ipc4, hist, hist_ok, n, seed=63):
    """An IPv4 ingress stream toward EP_LXC_ID's IPv4 address: replies from
    the peers of the history's NAT64 flows (hist_ok: the flows that were
    forwarded), ICMP errors about them (every icmp4_to_icmp6 case), and new
    IPv4 traffic; the replies of a flow several times, in order"""
    rng = np.random.default_rng(seed + 500)
    m = int(n * 0.6)
    pick = hist_ok[rng.integers(0, len(hist_ok), size=m)]
    src = take(hist, pick)
    peer = np.ascontiguousarray(src.daddr[:, 12:16]).view("<u4").ravel()
    icmp = src.proto == IPPROTO_ICMPV6
    rep = Headers(4, peer.copy(), np.full(m, LXC_IPV4, np.uint32),
                  np.where(icmp, 0, src.dport).astype(np.uint16),
                  np.where(icmp, src.dport, src.sport).astype(np.uint16),
                  np.where(icmp, IPPROTO_ICMP, src.proto).astype(np.uint8),
                  np.zeros(m, np.uint8), rng.integers(60, 1500, size=m).astype(np.uint16),
                  np.zeros(m, np.uint32))
    rep.tcpflags = np.where(rep.proto == IPPROTO_TCP,
                            rng.choice(np.array([0x12, 0x10, 0x18], np.uint8), size=m), 0
                            ).astype(np.uint8)
    fin = (rep.proto == IPPROTO_TCP) & (rng.random(m) < 0.05)
    rep.flags[fin] = HF_TCP_CLOSE
    rep.tcpflags[fin] = 0x11
    k = int(n * 0.12)
    ep_ = take(rep, rng.integers(0, m, size=k))
    tc = np.array([[3, 0], [3, 1], [3, 2], [3, 3], [3, 4], [3, 5], [3, 9], [3, 13],
                   [3, 14], [11, 0], [12, 0], [5, 0]], np.uint16)
    pick2 = tc[rng.integers(0, len(tc), size=k)]
    ep_.proto[:] = IPPROTO_ICMP
    ep_.sport[:] = (pick2[:, 0] | pick2[:, 1] << 8).astype(np.uint16)
    ep_.dport[:] = 0
    ep_.flags[:] = 0
    ep_.tcpflags = np.zeros(k, np.uint8)
    new = gen_headers_v4(rng, n - m - k, ipc4, local_v4_addrs(t)[:1], local_frac=1.0,
                         mark_host=0, mark_proxy=0, frag=0)
    h = concat([rep, ep_, new])
    return take(h, rng.permutation(len(h)))
