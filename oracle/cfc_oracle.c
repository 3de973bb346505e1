/*
 * cfc_oracle.c — CPU restatement of the reference verdict path.
 * TEST INFRASTRUCTURE ONLY (see cfc_oracle.h).
 *
 * Tables are kept the simple way: exact-match hash tables, and longest-prefix
 * match done as one hash table per prefix length probed from the longest
 * present length down — the same scheme as the reference's hashed-prefix
 * fallback LPM_LOOKUP_FN (bpf/lib/eps.h:88-108).  The kernel LPM trie the
 * reference uses (kernel/bpf/lpm_trie.c) returns the same longest match.
 */
#define _GNU_SOURCE
#include "cfc_oracle.h"

#include <stdlib.h>
#include <string.h>

/* bpf/node_config.h */
#define HOST_ID 1u
#define WORLD_ID 2u
#define CLUSTER_ID 3u
#define HEALTH_ID 4u
/* bpf/lib/common.h:237-269 */
#define DROP_INVALID_SIP -132
#define DROP_POLICY -133
#define DROP_CT_UNKNOWN_PROTO -137
#define DROP_MISSED_TAIL_CALL -140
#define DROP_FRAG_NOSUPPORT -157
#define DROP_NO_SERVICE -158
/* UAPI */
#define TC_ACT_OK 0
#define TC_ACT_SHOT 2
#define TC_ACT_REDIRECT 7
#define XDP_DROP 1
#define XDP_PASS 2
#define METRIC_INGRESS 1
#define METRIC_EGRESS 2
#define CT_EGRESS 0
#define CT_INGRESS 1
#define CT_SERVICE 2
#define HF_FRAG 1
#define HF_TCP_CLOSE 2
#define ENDPOINT_F_HOST 1u
#define MARK_MAGIC_HOST_MASK 0xF00u
#define MARK_MAGIC_PROXY_INGRESS 0xA00u
#define MARK_MAGIC_PROXY_EGRESS 0xB00u
#define MARK_MAGIC_HOST 0xC00u

/* ------------------------------------------------------------ hash table */
typedef struct {
    uint32_t ksz, cap, n;
    uint8_t *keys;
    uint32_t *vals;
    uint8_t *used;
} htab;

static uint64_t hbytes(const uint8_t *k, uint32_t n)
{
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < n; i++) {
        h ^= k[i];
        h *= 1099511628211ull;
    }
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return h;
}

static void ht_init(htab *h, uint32_t ksz)
{
    memset(h, 0, sizeof(*h));
    h->ksz = ksz;
}

static void ht_free(htab *h)
{
    free(h->keys);
    free(h->vals);
    free(h->used);
    memset(h, 0, sizeof(*h));
}

static void ht_put(htab *h, const uint8_t *k, uint32_t v);

static void ht_grow(htab *h)
{
    htab o = *h;
    h->cap = o.cap ? o.cap * 2 : 64;
    h->n = 0;
    h->keys = calloc((size_t)h->cap, h->ksz);
    h->vals = calloc((size_t)h->cap, sizeof(uint32_t));
    h->used = calloc((size_t)h->cap, 1);
    for (uint32_t i = 0; i < o.cap; i++)
        if (o.used[i])
            ht_put(h, o.keys + (size_t)i * o.ksz, o.vals[i]);
    free(o.keys);
    free(o.vals);
    free(o.used);
}

static int64_t ht_find(const htab *h, const uint8_t *k)
{
    if (!h->cap)
        return -1;
    uint32_t m = h->cap - 1, i = (uint32_t)hbytes(k, h->ksz) & m;
    while (h->used[i]) {
        if (!memcmp(h->keys + (size_t)i * h->ksz, k, h->ksz))
            return i;
        i = (i + 1) & m;
    }
    return -1;
}

static void ht_put(htab *h, const uint8_t *k, uint32_t v)
{
    int64_t s = ht_find(h, k);
    if (s >= 0) {
        h->vals[s] = v;
        return;
    }
    if ((h->n + 1) * 2 > h->cap)
        ht_grow(h);
    uint32_t m = h->cap - 1, i = (uint32_t)hbytes(k, h->ksz) & m;
    while (h->used[i])
        i = (i + 1) & m;
    h->used[i] = 1;
    memcpy(h->keys + (size_t)i * h->ksz, k, h->ksz);
    h->vals[i] = v;
    h->n++;
}

static int ht_get(const htab *h, const uint8_t *k, uint32_t *v)
{
    int64_t s = ht_find(h, k);
    if (s < 0)
        return 0;
    *v = h->vals[s];
    return 1;
}

/* ------------------------------------------------------------ LPM */
typedef struct {
    int alen;            /* address bytes: 4 or 16 */
    htab len[129];
    int lens[129];       /* present prefix lengths, descending */
    int nlens;
} lpm;

static void lpm_init(lpm *l, int alen)
{
    memset(l, 0, sizeof(*l));
    l->alen = alen;
    for (int i = 0; i <= alen * 8; i++)
        ht_init(&l->len[i], (uint32_t)alen);
}

static void lpm_free(lpm *l)
{
    for (int i = 0; i <= l->alen * 8; i++)
        ht_free(&l->len[i]);
}

/* ipv6_addr_clear_suffix / GET_PREFIX (bpf/lib/ipv6.h:136-150) */
static void mask_addr(uint8_t *out, const uint8_t *a, int alen, int plen)
{
    for (int i = 0; i < alen; i++) {
        int b = plen - 8 * i;
        uint8_t m = b >= 8 ? 0xFF : b <= 0 ? 0 : (uint8_t)(0xFF << (8 - b));
        out[i] = a[i] & m;
    }
}

static void lpm_add(lpm *l, int plen, const uint8_t *addr, uint32_t val)
{
    uint8_t k[16];
    mask_addr(k, addr, l->alen, plen);
    if (!l->len[plen].n) {
        int i = l->nlens++;
        while (i > 0 && l->lens[i - 1] < plen) {
            l->lens[i] = l->lens[i - 1];
            i--;
        }
        l->lens[i] = plen;
    }
    ht_put(&l->len[plen], k, val);
}

static int lpm_lookup(const lpm *l, const uint8_t *addr, uint32_t *val)
{
    uint8_t k[16];
    for (int i = 0; i < l->nlens; i++) {
        int p = l->lens[i];
        mask_addr(k, addr, l->alen, p);
        if (ht_get(&l->len[p], k, val))
            return 1;
    }
    return 0;
}

/* ------------------------------------------------------------ conntrack */
/* struct ct_entry (bpf/lib/common.h:380-406), 56 bytes */
struct ctent {
    uint64_t rx_packets, rx_bytes, tx_packets, tx_bytes;
    uint32_t lifetime;
    uint16_t bits;          /* rx_closing:1 tx_closing:1 nat46:1 lb_loopback:1
                               seen_non_syn:1 */
    uint16_t rev_nat_index, slave;
    uint8_t tx_flags_seen, rx_flags_seen;
    uint32_t src_sec_id, last_tx_report, last_rx_report;
};
_Static_assert(sizeof(struct ctent) == 56, "ct_entry is 56 bytes");
#define CTB_RX_CLOSING 1u
#define CTB_TX_CLOSING 2u
#define CTB_NAT46 4u
#define CTB_LB_LOOPBACK 8u
#define CTB_SEEN_NON_SYN 16u
/* conntrack.h:31-35, common.h:224, node_config.h:69 */
#define CT_LIFETIME_TCP 21600u
#define CT_LIFETIME_NONTCP 60u
#define CT_SYN_TIMEOUT 60u
#define CT_CLOSE_TIMEOUT 10u
#define CT_REPORT_INTERVAL 5u
#define TRACE_PAYLOAD_LEN 128u
#define MTU 1500u

/* CT map key as the oracle stores it: u16 owner (0 = the global maps
 * cilium_ct{4,_any4,6,_any6}_global, else lxc_id + 1 for the endpoint's
 * local maps, pkg/maps/ctmap/ctmap.go:59-69,403-425), u8 map kind
 * (0 = TCP map, 1 = ANY map: get_ct_map4/6, bpf_lxc.c:91-107), u8 family,
 * then struct ipv4_ct_tuple (14 B) / ipv6_ct_tuple (38 B)
 * (common.h:338-367) zero padded to 40. */
#define CTK 44
#define TUPLE_F_OUT 0
#define TUPLE_F_IN 1
#define TUPLE_F_RELATED 2
#define TUPLE_F_SERVICE 4
enum { CT_NEW = 0, CT_ESTABLISHED = 1, CT_REPLY = 2, CT_RELATED = 3 };
enum { ACTION_UNSPEC = 0, ACTION_CREATE = 1, ACTION_CLOSE = 2 };
/* per-header CT byte (cfc.h CFC_CT_*): two lookup stages, the second being
 * the destination endpoint's ingress policy after egress local delivery */
#define CTO_DONE1 0x04u
#define CTO_CREATE1 0x08u
#define CTO_DONE2 0x40u
#define CTO_CREATE2 0x80u

static void ct_key(uint8_t k[CTK], uint16_t owner, uint8_t kind, int alen,
                   const uint8_t *daddr, const uint8_t *saddr,
                   uint16_t dport, uint16_t sport, uint8_t nexthdr,
                   uint8_t flags)
{
    memset(k, 0, CTK);
    memcpy(k, &owner, 2);
    k[2] = kind;
    k[3] = (uint8_t)(alen == 4 ? 1 : 2);
    uint8_t *t = k + 4;
    memcpy(t, daddr, alen);
    memcpy(t + alen, saddr, alen);
    memcpy(t + 2 * alen, &dport, 2);
    memcpy(t + 2 * alen + 2, &sport, 2);
    t[2 * alen + 4] = nexthdr;
    t[2 * alen + 5] = flags;
}

/* The two keys ct_lookup4 / ct_lookup6 probe (conntrack.h:467-590,
 * :310-437).  k1: the tuple as loaded — addresses as in the packet, the L4
 * ports loaded into {dport, sport} (so swapped), flags TUPLE_F_OUT for
 * ingress / TUPLE_F_IN for egress; a hit is CT_REPLY (CT_RELATED with
 * TUPLE_F_RELATED).  k2: ipv{4,6}_ct_tuple_reverse(k1), a hit is
 * CT_ESTABLISHED, a miss CT_NEW and k2 is what ct_create{4,6} stores.
 * ICMP: ports zeroed; error types set TUPLE_F_RELATED; echo reply sets
 * tuple->dport = ECHO; echo request sets tuple->sport = its type.
 * Returns 0, or DROP_CT_UNKNOWN_PROTO for anything but TCP/UDP/ICMP. */
static int ct_keys(int alen, uint16_t owner, const uint8_t *sa,
                   const uint8_t *da, uint8_t proto, uint16_t sport,
                   uint16_t dport, int close, int dir, uint8_t k1[CTK],
                   uint8_t k2[CTK], int *action, uint16_t *td, uint16_t *ts)
{
    uint8_t fl = dir == CT_INGRESS ? TUPLE_F_OUT
                 : dir == CT_SERVICE ? TUPLE_F_SERVICE : TUPLE_F_IN;
    const uint8_t icmp = alen == 4 ? 1 : 58;
    *action = ACTION_UNSPEC;
    *td = *ts = 0;
    if (proto == icmp) {
        uint8_t type = (uint8_t)(sport & 0xFF);
        int related = alen == 4 ? (type == 3 || type == 11 || type == 12)
                                : (type >= 1 && type <= 4);
        uint8_t echo_reply = alen == 4 ? 0 : 129, echo = alen == 4 ? 8 : 128;
        if (related)
            fl |= TUPLE_F_RELATED;
        else if (type == echo_reply)
            *td = echo;
        else {
            if (type == echo)
                *ts = type;
            *action = ACTION_CREATE;
        }
    } else if (proto == 6) {
        *action = close ? ACTION_CLOSE : ACTION_CREATE;
        *td = sport;
        *ts = dport;
    } else if (proto == 17) {
        *action = ACTION_CREATE;
        *td = sport;
        *ts = dport;
    } else {
        return DROP_CT_UNKNOWN_PROTO;
    }
    const uint8_t kind = proto == 6 ? 0 : 1;
    ct_key(k1, owner, kind, alen, da, sa, *td, *ts, proto, fl);
    ct_key(k2, owner, kind, alen, sa, da, *ts, *td, proto, fl ^ TUPLE_F_IN);
    return 0;
}

static int64_t ct_find(const cfo_t *o, const uint8_t k[CTK]);

/* ------------------------------------------------------------ tables */
typedef struct {
    uint8_t key[8];      /* struct policy_key (common.h:180-186) raw bytes */
    uint16_t proxy_port; /* struct policy_entry.proxy_port, be16 raw */
    uint64_t packets, bytes;
} pentry;

typedef struct {
    htab idx;            /* key -> index into ents */
    pentry *ents;
    uint32_t n, cap;
} pmap;

typedef struct {
    uint32_t ifindex, flags;
    uint16_t lxc_id;
} epinfo;

/* struct lb4_service (common.h:433-439); the key struct lb4_key {address,
 * dport, slave} (:427-431) is the htab key */
typedef struct {
    uint32_t target;
    uint16_t port, count, rev_nat_index, weight;
} lb4svc;
/* struct lb6_service (common.h:414-420); the key struct lb6_key {address[16],
 * dport, slave} (:408-412, 20 bytes packed) is the htab key */
typedef struct {
    uint8_t target[16];
    uint16_t port, count, rev_nat_index, weight;
} lb6svc;

struct cfo {
    lpm ipc4, ipc6;
    htab lxc;            /* 20-byte endpoint_key -> index into eps */
    epinfo *eps;
    uint32_t neps, capeps;
    pmap *pol[65536];
    uint32_t seclabel[65536];
    uint8_t has_seclabel[65536];
    htab pf4_fix, pf6_fix; /* lpm_v{4,6}_key bytes (prefixlen + addr) */
    lpm pf4_dyn, pf6_dyn;
    uint64_t metrics[256][4][2];
    /* conntrack: every CT map in one table, keyed by (owner, map kind,
     * family, tuple) -> index into ct_ents */
    htab ct;
    struct ctent *ct_ents;
    uint8_t *ct_live;
    uint32_t ct_n, ct_cap, ct_added;
    uint32_t *notify_out; /* cfo_set_notify_out */
    uint8_t ct_local[65536];   /* endpoint has its own (local) CT maps */
    /* node_config.h constants the agent writes per node (daemon.go:916-934):
     * IPV4_CLUSTER_RANGE / _MASK (raw be32 as loaded), ROUTER_IP */
    uint32_t v4_cluster_range, v4_cluster_mask;
    uint8_t router_ip6[16];
    /* per-identity forward/drop counters (cfc.h cfc_identity_counters):
     * [dir 0 ingress / 1 egress][identity, >= 65536 in the last slot]
     * [fwd, drop][packets, bytes] */
    uint64_t *idc;
    uint32_t host_ifindex;     /* node_config.h HOST_IFINDEX */
    uint32_t now;              /* bpf_ktime_get_sec() of the batch (cfo_set_clock) */
    uint32_t *notify_mon;      /* cfo_set_notify_out: per-header monitor lengths */
    /* service load balancing (bpf/lib/lb.h): cilium_lb4_services and
     * cilium_lb4_reverse_nat (struct lb4_reverse_nat {address, port},
     * common.h:441-444, by rev_nat_index) */
    htab lb4;
    lb4svc *lb4v;
    uint32_t lb4_n, lb4_cap;
    uint32_t *rnat4_addr;
    uint16_t *rnat4_port;
    uint8_t *rnat4_ok;
    /* IPv6: cilium_lb6_services and cilium_lb6_reverse_nat (struct
     * lb6_reverse_nat {address[16], port}, common.h:422-425) */
    htab lb6;
    lb6svc *lb6v;
    uint32_t lb6_n, lb6_cap;
    uint8_t *rnat6_addr;       /* [65536][16] */
    uint16_t *rnat6_port;
    uint8_t *rnat6_ok;
    /* cfo_set_lb_io: skb->hash per header (NULL: cfo_flow_hash4/6), and the
     * packet's addresses after the program's rewrites: IPv4 3 u32 per header
     * (saddr, daddr, L4 word), IPv6 9 (saddr[4], daddr[4], L4 word) */
    const uint32_t *hash_in;
    uint32_t *pkt_out;
    /* each endpoint's own addresses (LXC_IPV4 / LXC_IP of its program,
     * lxc_config.h:24-25): NAT64's saddr, NAT46's daddr */
    uint32_t ep_v4[65536];
    uint8_t ep_v6[65536][16];
    uint8_t ep_has4[65536], ep_has6[65536];
    /* per header of the last classify: the NAT46 / NAT64 hop it took (the
     * CT stage of the other family, applied by ct_apply as stage 1) */
    struct hop *hop;
    size_t hop_cap;
};
#define ID_SLOTS 65537u

/* A header's NAT hop (LXC_NAT46, nat46.h): NAT64 — an IPv6 egress packet
 * to ::ffff:0:0/96 re-entering the IPv4 egress program translated
 * (tail_ipv6_to_ipv4, bpf_lxc.c:1070-1083); NAT46 — an IPv4 packet whose CT
 * entry says nat46 re-entering ipv6_policy translated (tail_ipv4_to_ipv6,
 * :1098-1110).  The hop's CT stage is stage 1 of the CT byte. */
#define HOP_NAT64 1
#define HOP_NAT46 2
struct hop {
    uint8_t kind, alen, proto, dir;
    uint16_t owner, sport, dport;
    uint8_t sa[16], da[16];
    int32_t dlen;   /* skb->len change: the IPv4 header is 20 bytes shorter */
    /* a NAT64 hop delivered locally (ipv4_local_delivery, l3.h:103-131):
     * the destination's ipv4_policy lookup is a third CT stage, in its CT
     * maps — its tuple and CT nibble (result | done | create) */
    uint8_t has2, ct2;
    uint16_t owner2, sport2, dport2;
    uint8_t sa2[4], da2[4];
};

static uint16_t ct_owner(const cfo_t *o, uint16_t lxc)
{
    return o->ct_local[lxc] ? (uint16_t)(lxc + 1) : 0;
}

static int64_t ct_find(const cfo_t *o, const uint8_t k[CTK])
{
    int64_t s = ht_find(&o->ct, k);
    if (s < 0)
        return -1;
    uint32_t idx = o->ct.vals[s];
    return o->ct_live[idx] ? (int64_t)idx : -1;
}

cfo_t *cfo_new(void)
{
    cfo_t *o = calloc(1, sizeof(*o));
    lpm_init(&o->ipc4, 4);
    lpm_init(&o->ipc6, 16);
    lpm_init(&o->pf4_dyn, 4);
    lpm_init(&o->pf6_dyn, 16);
    ht_init(&o->lxc, 20);
    ht_init(&o->pf4_fix, 8);
    ht_init(&o->pf6_fix, 20);
    ht_init(&o->ct, CTK);
    ht_init(&o->lb4, 8);
    ht_init(&o->lb6, 20);
    o->rnat6_addr = calloc(65536, 16);
    o->rnat6_port = calloc(65536, 2);
    o->rnat6_ok = calloc(65536, 1);
    o->rnat4_addr = calloc(65536, 4);
    o->rnat4_port = calloc(65536, 2);
    o->rnat4_ok = calloc(65536, 1);
    o->idc = calloc((size_t)2 * ID_SLOTS * 4, sizeof(uint64_t));
    /* bpf/node_config.h:30,42-43 */
    static const uint8_t router[16] = {0xbe, 0xef, 0, 0, 0, 0, 0, 0,
                                       0, 0, 0, 1, 0, 1, 0, 0};
    cfo_node_config(o, 0x100000u, 0xff0000u, router, 1);
    return o;
}

void cfo_node_config(cfo_t *o, uint32_t v4_cluster_range,
                     uint32_t v4_cluster_mask, const uint8_t router_ip6[16],
                     uint32_t host_ifindex)
{
    o->v4_cluster_range = v4_cluster_range;
    o->v4_cluster_mask = v4_cluster_mask;
    memcpy(o->router_ip6, router_ip6, 16);
    o->host_ifindex = host_ifindex;
}

void cfo_set_clock(cfo_t *o, uint32_t now) { o->now = now; }

void cfo_free(cfo_t *o)
{
    if (!o)
        return;
    lpm_free(&o->ipc4);
    lpm_free(&o->ipc6);
    lpm_free(&o->pf4_dyn);
    lpm_free(&o->pf6_dyn);
    ht_free(&o->lxc);
    ht_free(&o->pf4_fix);
    ht_free(&o->pf6_fix);
    ht_free(&o->ct);
    ht_free(&o->lb4);
    free(o->lb4v);
    ht_free(&o->lb6);
    free(o->lb6v);
    free(o->rnat6_addr);
    free(o->rnat6_port);
    free(o->rnat6_ok);
    free(o->rnat4_addr);
    free(o->rnat4_port);
    free(o->rnat4_ok);
    free(o->ct_ents);
    free(o->ct_live);
    free(o->idc);
    for (int i = 0; i < 65536; i++)
        if (o->pol[i]) {
            ht_free(&o->pol[i]->idx);
            free(o->pol[i]->ents);
            free(o->pol[i]);
        }
    free(o->eps);
    free(o->hop);
    free(o);
}

int cfo_ipcache_add(cfo_t *o, int family, int plen, const uint8_t addr[16],
                    uint32_t label)
{
    if (family == 1 && plen >= 0 && plen <= 32)
        lpm_add(&o->ipc4, plen, addr, label);
    else if (family == 2 && plen >= 0 && plen <= 128)
        lpm_add(&o->ipc6, plen, addr, label);
    else
        return -22;
    return 0;
}

/* ipcache_lookup4/6 (eps.h:56-80) on n addresses */
void cfo_ipcache_lookup(cfo_t *o, int family, size_t n, const uint8_t *addrs,
                        uint32_t *label, uint8_t *hit)
{
    const lpm *l = family == 1 ? &o->ipc4 : &o->ipc6;
    const size_t al = family == 1 ? 4 : 16;
    for (size_t i = 0; i < n; i++) {
        uint32_t v = 0;
        hit[i] = (uint8_t)lpm_lookup(l, addrs + al * i, &v);
        label[i] = hit[i] ? v : 0;
    }
}

static void ep_key(uint8_t k[20], int family, const uint8_t *addr)
{
    memset(k, 0, 20);
    memcpy(k, addr, family == 1 ? 4 : 16);
    k[16] = (uint8_t)family;
}

int cfo_endpoint_add(cfo_t *o, int family, const uint8_t addr[16],
                     uint32_t ifindex, uint16_t lxc_id, uint32_t flags)
{
    uint8_t k[20];
    ep_key(k, family, addr);
    if (o->neps == o->capeps) {
        o->capeps = o->capeps ? o->capeps * 2 : 16;
        o->eps = realloc(o->eps, o->capeps * sizeof(epinfo));
    }
    o->eps[o->neps] = (epinfo){ifindex, flags, lxc_id};
    ht_put(&o->lxc, k, o->neps++);
    /* LXC_IPV4 / LXC_IP of the endpoint (the NAT46 / NAT64 addresses): the
     * lowest address of the family among its cilium_lxc entries (an
     * endpoint normally has one per family; the engine picks the same) */
    if (!(flags & ENDPOINT_F_HOST)) {
        if (family == 1 && (!o->ep_has4[lxc_id] || memcmp(addr, &o->ep_v4[lxc_id], 4) < 0)) {
            memcpy(&o->ep_v4[lxc_id], addr, 4);
            o->ep_has4[lxc_id] = 1;
        } else if (family == 2 &&
                   (!o->ep_has6[lxc_id] || memcmp(addr, o->ep_v6[lxc_id], 16) < 0)) {
            memcpy(o->ep_v6[lxc_id], addr, 16);
            o->ep_has6[lxc_id] = 1;
        }
    }
    return 0;
}

int cfo_seclabel_set(cfo_t *o, uint16_t lxc_id, uint32_t seclabel)
{
    o->seclabel[lxc_id] = seclabel;
    o->has_seclabel[lxc_id] = 1;
    return 0;
}

static void pkey(uint8_t k[8], uint32_t id, uint16_t dport, uint8_t proto,
                 uint8_t egress)
{
    memcpy(k, &id, 4);
    memcpy(k + 4, &dport, 2);
    k[6] = proto;
    k[7] = egress;
}

int cfo_policy_add(cfo_t *o, uint16_t lxc_id, uint32_t identity,
                   uint16_t dport_be, uint8_t proto, uint8_t egress,
                   uint16_t proxy_port_be)
{
    pmap *m = o->pol[lxc_id];
    if (!m) {
        m = o->pol[lxc_id] = calloc(1, sizeof(pmap));
        ht_init(&m->idx, 8);
    }
    uint8_t k[8];
    pkey(k, identity, dport_be, proto, egress);
    uint32_t i;
    if (!ht_get(&m->idx, k, &i)) {
        if (m->n == m->cap) {
            m->cap = m->cap ? m->cap * 2 : 64;
            m->ents = realloc(m->ents, m->cap * sizeof(pentry));
        }
        i = m->n++;
        ht_put(&m->idx, k, i);
    }
    memcpy(m->ents[i].key, k, 8);
    m->ents[i].proxy_port = proxy_port_be;
    m->ents[i].packets = m->ents[i].bytes = 0;
    return 0;
}

int cfo_prefilter_add(cfo_t *o, int family, int plen, const uint8_t addr[16],
                      int dyn)
{
    int alen = family == 1 ? 4 : 16;
    if (dyn) {
        lpm_add(family == 1 ? &o->pf4_dyn : &o->pf6_dyn, plen, addr, 1);
    } else {
        uint8_t k[20];
        uint32_t pl = (uint32_t)plen;
        memcpy(k, &pl, 4);
        memcpy(k + 4, addr, alen);
        ht_put(family == 1 ? &o->pf4_fix : &o->pf6_fix, k, 1);
    }
    return 0;
}

/* cilium_lb4_services: key struct lb4_key (8 bytes: address, dport be16,
 * slave), value struct lb4_service (12 bytes) — lb.h:70-76 */
int cfo_lb4_service_add(cfo_t *o, const uint8_t key[8], const uint8_t val[12])
{
    uint32_t v;
    if (!ht_get(&o->lb4, key, &v)) {
        if (o->lb4_n == o->lb4_cap) {
            o->lb4_cap = o->lb4_cap ? 2 * o->lb4_cap : 64;
            o->lb4v = realloc(o->lb4v, o->lb4_cap * sizeof(lb4svc));
        }
        v = o->lb4_n++;
        ht_put(&o->lb4, key, v);
    }
    lb4svc *e = &o->lb4v[v];
    memcpy(&e->target, val, 4);
    memcpy(&e->port, val + 4, 2);
    memcpy(&e->count, val + 6, 2);
    memcpy(&e->rev_nat_index, val + 8, 2);
    memcpy(&e->weight, val + 10, 2);
    return 0;
}

/* cilium_lb4_reverse_nat: key rev_nat_index, value struct lb4_reverse_nat
 * (6 bytes: address, port be16) — lb.h:62-68 */
int cfo_lb4_revnat_add(cfo_t *o, uint16_t index, const uint8_t val[6])
{
    memcpy(&o->rnat4_addr[index], val, 4);
    memcpy(&o->rnat4_port[index], val + 4, 2);
    o->rnat4_ok[index] = 1;
    return 0;
}

/* cilium_lb6_services: key struct lb6_key (20 bytes: address, dport be16,
 * slave), value struct lb6_service (24 bytes) — lb.h:46-53 */
int cfo_lb6_service_add(cfo_t *o, const uint8_t key[20], const uint8_t val[24])
{
    uint32_t v;
    if (!ht_get(&o->lb6, key, &v)) {
        if (o->lb6_n == o->lb6_cap) {
            o->lb6_cap = o->lb6_cap ? 2 * o->lb6_cap : 64;
            o->lb6v = realloc(o->lb6v, o->lb6_cap * sizeof(lb6svc));
        }
        v = o->lb6_n++;
        ht_put(&o->lb6, key, v);
    }
    lb6svc *e = &o->lb6v[v];
    memcpy(e->target, val, 16);
    memcpy(&e->port, val + 16, 2);
    memcpy(&e->count, val + 18, 2);
    memcpy(&e->rev_nat_index, val + 20, 2);
    memcpy(&e->weight, val + 22, 2);
    return 0;
}

/* cilium_lb6_reverse_nat: key rev_nat_index, value struct lb6_reverse_nat
 * (18 bytes: address, port be16) — lb.h:38-45 */
int cfo_lb6_revnat_add(cfo_t *o, uint16_t index, const uint8_t val[18])
{
    memcpy(o->rnat6_addr + 16 * (size_t)index, val, 16);
    memcpy(&o->rnat6_port[index], val + 16, 2);
    o->rnat6_ok[index] = 1;
    return 0;
}

void cfo_set_lb_io(cfo_t *o, const uint32_t *hash, uint32_t *pkt)
{
    o->hash_in = hash;
    o->pkt_out = pkt;
}

static uint32_t fmix32(uint32_t h)
{
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

/* the engine's stand-in for the kernel's skb hash when the batch carries
 * none (cfc.h CFC_FLOW_HASH, oracle.py flow_hash): symmetric in the
 * 5-tuple, over the packet as it entered the program */
uint32_t cfo_flow_hash4(uint32_t sa, uint32_t da, uint16_t sport, uint16_t dport,
                        uint8_t proto)
{
    const uint32_t lo = sa < da ? sa : da, hi = sa < da ? da : sa;
    const uint32_t a = sport, b = dport;
    const uint32_t pw = (a < b ? a : b) | (a < b ? b : a) << 16;
    return fmix32(lo * 0x9E3779B1u + hi * 0x85EBCA77u + pw * 0xC2B2AE3Du + proto);
}

/* the same over IPv6 addresses, each folded to a word as notify.hip fold6
 * (raw words loaded little-endian) */
static uint32_t fold6(const uint8_t *a)
{
    uint32_t w[4];
    memcpy(w, a, 16);
    uint32_t h = fmix32(w[3]);
    h = fmix32(w[2] ^ h);
    h = fmix32(w[1] ^ h);
    return fmix32(w[0] ^ h);
}
uint32_t cfo_flow_hash6(const uint8_t sa[16], const uint8_t da[16], uint16_t sport,
                        uint16_t dport, uint8_t proto)
{
    return cfo_flow_hash4(fold6(sa), fold6(da), sport, dport, proto);
}

/* ------------------------------------------------------------ datapath */
static inline void add64(uint64_t *p, uint64_t v)
{
    __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
}

/* update_metrics (bpf/lib/metrics.h:43-61); reason = -DROP_* or 0 */
static void metric(cfo_t *o, int reason, int dir, uint32_t len)
{
    uint8_t r = (uint8_t)(-reason);
    add64(&o->metrics[r][dir][0], 1);
    add64(&o->metrics[r][dir][1], len);
}

/* one policy verdict (a __policy_can_access call, policy.h:46-110) of
 * identity `ident` in direction dir (0 ingress: ipv{4,6}_policy's source
 * identity; 1 egress: handle_ipv4_from_lxc's destination identity): a drop
 * when the verdict path drops the packet for it (DROP_POLICY), else a
 * forward */
static void id_event(cfo_t *o, int dir, uint32_t ident, int drop, uint32_t len)
{
    uint32_t s = ident < ID_SLOTS - 1 ? ident : ID_SLOTS - 1;
    uint64_t *p = o->idc + (((size_t)dir * ID_SLOTS + s) * 2 + (drop ? 1 : 0)) * 2;
    add64(p, 1);
    add64(p + 1, len);
}

static const epinfo *lxc_lookup(const cfo_t *o, int family,
                                const uint8_t *addr)
{
    uint8_t k[20];
    uint32_t i;
    ep_key(k, family, addr);
    return ht_get(&o->lxc, k, &i) ? &o->eps[i] : NULL;
}

/* map_lookup_elem() calls the reference executes for the current header
 * (SURVEY.md §8d "L"): prefilter, endpoint, ipcache and policy lookups. */
static _Thread_local uint32_t tl_lookups;

static pentry *pol_lookup(pmap *m, uint32_t id, uint16_t dport, uint8_t proto,
                          uint8_t egress)
{
    tl_lookups++;
    if (!m)
        return NULL;
    uint8_t k[8];
    uint32_t i;
    pkey(k, id, dport, proto, egress);
    return ht_get(&m->idx, k, &i) ? &m->ents[i] : NULL;
}

static void hit(pentry *e, uint32_t len)
{
    add64(&e->packets, 1);
    add64(&e->bytes, len);
}

/* __policy_can_access (bpf/lib/policy.h:46-110).  cb[CB_POLICY] is always 0
 * here: policy_clear_mark() runs first on every path we model
 * (bpf_lxc.c:916, :626). */
static int policy_can_access(pmap *m, uint32_t identity, uint16_t dport,
                             uint8_t proto, int dir, int frag, uint32_t len)
{
    uint8_t egress = !dir;
    pentry *e;
    if (!frag) {
        e = pol_lookup(m, identity, dport, proto, egress);
        if (e) {
            hit(e, len);
            return e->proxy_port;
        }
    }
    e = pol_lookup(m, identity, 0, 0, egress);
    if (e) {
        hit(e, len);
        return TC_ACT_OK;
    }
    if (!frag) {
        e = pol_lookup(m, 0, dport, proto, egress);
        if (e) {
            hit(e, len);
            return e->proxy_port;
        }
    }
    return frag ? DROP_FRAG_NOSUPPORT : DROP_POLICY;
}

/* nt: which send_drop_notify reported a drop (drop.h:94-109), as
 * site << 16 | EVENT_SOURCE; 0 = none.  Sites: 1 bpf_netdev's
 * send_drop_notify_error (bpf_netdev.c:463,502), 2 the sending endpoint's
 * (SECLABEL, dstID, 0, 0) (bpf_lxc.c:432,700), 3 the destination's
 * tail_ipv{4,6}_policy (src_label, SECLABEL, LXC_ID, ifindex)
 * (bpf_lxc.c:891,1024). */
typedef struct {
    int32_t action, verdict;
    uint32_t identity;
    uint32_t nt;
} res_t;
#define NT_NETDEV 1u
#define NT_EGRESS 2u
#define NT_POLICY 3u
/* bit 24: the event followed a NAT46 / NAT64 hop, its length is the
 * translated packet's (IPv4 header 20 bytes shorter than IPv6) */
#define NT_NATLEN 0x01000000u
/* The monitor event of a header (cfc.h CFC_NT_*): bits 0-15 EVENT_SOURCE,
 * bits 16-19 the kind — drop sites 1-3 above, or a trace_notify at
 * observation point kind - 4 (TRACE_TO_LXC 4, TO_PROXY 5, TO_HOST 6,
 * TO_STACK 7; trace.h:37-48) — and for traces bits 20-21 the reason (the CT
 * result, trace.h:51-56) and bits 22-23 the monitor length: 1 =
 * TRACE_PAYLOAD_LEN, 2 = MTU, 3 = 1 (an active flow's report).  With MONITOR_AGGREGATION 5 (node_config.h:68)
 * the FROM_* points and every trace whose monitor length is 0 are not sent
 * (trace.h:119-132); no header has more than one event. */
#define NT_TRACE 4u
enum { OBS_TO_LXC = 0, OBS_TO_PROXY = 1, OBS_TO_HOST = 2, OBS_TO_STACK = 3 };

static uint32_t trace_word(uint32_t obs, uint16_t source, int reason, uint32_t mon)
{
    /* (monitor length 0, not sent: class 0 — the site stays in the word) */
    return (NT_TRACE + obs) << 16 | source | (uint32_t)reason << 20 |
           (mon == 0 ? 0u : mon == MTU ? 2u : mon == 1 ? 3u : 1u) << 22;
}

/* sites 1-2 follow from the mode; lxc_ingress sets site 3 itself */
static uint32_t notify_site(int mode, uint16_t ep_lxc, const res_t *r)
{
    if (r->verdict == -1 || r->verdict == -2)
        return 0; /* XDP prefilter drop / VERDICT_PUNT */
    if (r->verdict >= 0 || r->nt)
        return r->nt; /* a trace (or nothing), or the policy drop site */
    return mode == CFO_MODE_EGRESS ? NT_EGRESS << 16 | ep_lxc : NT_NETDEV << 16;
}


/* ipv4_policy (bpf_lxc.c:898-1015) + tail_ipv4_policy (:1017-1028) for
 * endpoint ep, called after local delivery with cb[CB_SRC_LABEL]=src; with
 * v6 set, ipv6_policy (:753-882) + tail_ipv6_policy (:884-895), which differ
 * only in the CT port derivation and pass is_fragment = false. */
/* CT byte of the current header (CTO_*) */
static _Thread_local uint8_t tl_ct;
static _Thread_local uint8_t tl_ct3;   /* a NAT64 hop's third stage (struct hop ct2) */
/* the current header's TCP flag byte (byte 13) and the monitor length each
 * CT stage's lookup returned (0 / TRACE_PAYLOAD_LEN / MTU) */
static _Thread_local uint8_t tl_tcpfl;
static _Thread_local uint32_t tl_mon[3];
/* skb->cb[CB_NAT46_STATE] (common.h:316-325): NAT46_CLEAR, NAT64 (set by
 * tail_ipv6_to_ipv4), NAT46 (set by __ct_lookup on an entry with nat46);
 * and the NAT hop the current header took */
#define NAT64 1
#define NAT46 2
static _Thread_local int tl_nat;
static _Thread_local struct hop tl_hop;

/* __ct_update_timeout (conntrack.h:125-185): the lifetime, and whether this
 * packet is reported (the flow's report interval passed, or it carries TCP
 * flags the direction has not seen) */
static uint32_t ct_upd(struct ctent *e, uint32_t now, uint32_t lifetime, int dir,
                       uint8_t flags)
{
    e->lifetime = now + lifetime;
    uint8_t *acc = dir == CT_INGRESS ? &e->rx_flags_seen : &e->tx_flags_seen;
    uint32_t *last = dir == CT_INGRESS ? &e->last_rx_report : &e->last_tx_report;
    const uint8_t seen = (uint8_t)(flags | *acc);
    if (*last + CT_REPORT_INTERVAL < now || *acc != seen) {
        *last = now;
        *acc = seen;
        return TRACE_PAYLOAD_LEN;
    }
    return 0;
}

/* ct_update_timeout (:191-205); syn is bit 0 of TCP byte 12, which every
 * bitfield of union tcp_flags aliases (:92-104).  It is declared bool, so
 * the monitor length it hands __ct_lookup is 1, not TRACE_PAYLOAD_LEN: a
 * reported packet of an active flow captures one byte. */
static uint32_t ct_upd_timeout(struct ctent *e, uint32_t now, int is_tcp, int dir,
                               int syn, uint8_t flags)
{
    uint32_t lifetime = CT_LIFETIME_NONTCP;
    if (is_tcp) {
        if (!syn)
            e->bits |= CTB_SEEN_NON_SYN;
        lifetime = (e->bits & CTB_SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
    }
    return ct_upd(e, now, lifetime, dir, flags) != 0;
}

static int ct_alive(const struct ctent *e)
{
    return !(e->bits & CTB_RX_CLOSING) || !(e->bits & CTB_TX_CLOSING);
}

/* What __ct_lookup (:221-285) does to a hit entry (timeouts, report
 * timestamps, seen flags, closing bits; the accounting is counted apart),
 * returning *monitor */
static uint32_t ct_hit_entry(struct ctent *e, uint32_t now, int action, int dir,
                             int is_tcp, int syn, uint8_t flags)
{
    uint32_t m = 0;
    if (ct_alive(e))
        m = ct_upd_timeout(e, now, is_tcp, dir, syn, flags);
    if (action == ACTION_CREATE) {
        if (e->bits & (CTB_RX_CLOSING | CTB_TX_CLOSING)) {
            e->bits &= (uint16_t)~(CTB_RX_CLOSING | CTB_TX_CLOSING);
            m = ct_upd_timeout(e, now, is_tcp, dir, syn, flags);
        }
    } else if (action == ACTION_CLOSE) {
        e->bits |= dir == CT_INGRESS ? CTB_RX_CLOSING : CTB_TX_CLOSING;
        m = TRACE_PAYLOAD_LEN;
        if (!ct_alive(e))
            ct_upd(e, now, CT_CLOSE_TIMEOUT, dir, flags);
    }
    return m;
}

/* ct_state as ct_create{4,6} reads it (common.h:452-461) */
typedef struct {
    uint16_t rev_nat, slave;
    int loopback;
    uint32_t addr, svc_addr;
    int nat46;     /* ct_create4 under NAT64: entry.nat46 (conntrack.h:714-716) */
} ctstate_t;
static int ct_create_entries(const cfo_t *o, const uint8_t k2[CTK], int alen, int dir,
                             uint32_t len, uint32_t src_sec_id, const ctstate_t *st,
                             uint8_t keys[3][CTK], struct ctent ents[3]);

/* The entries the egress stage of the current header created (ct_create4:
 * main, reverse-NAT and ICMP entries): the destination endpoint's lookup
 * after local delivery runs on the same skb, after those writes — a service
 * looped back into the sender finds its own reverse-NAT entry
 * (CT_ESTABLISHED) there. */
typedef struct {
    int n;
    uint8_t key[3][CTK];
    struct ctent ent[3];
} fresh_t;
static _Thread_local fresh_t tl_fresh;

static int64_t fresh_find(const uint8_t k[CTK])
{
    for (int j = 0; j < tl_fresh.n; j++)
        if (!memcmp(tl_fresh.key[j], k, CTK))
            return j;
    return -1;
}

/* ct_lookup{4,6} against the tables as they were when the batch started
 * (and, for the destination's lookup after local delivery, the entries the
 * egress stage of the same header created, tl_fresh): sets *res, the policy
 * port (tuple->dport after the lookup: the packet's source port for
 * CT_REPLY, its destination port otherwise), the entry hit (*hent, or NULL)
 * and, when k2out is given, the tuple ct_create would store (k2). */
static int ct_lookup(cfo_t *o, int alen, uint16_t owner, const uint8_t *sa,
                     const uint8_t *da, uint8_t proto, uint16_t sport,
                     uint16_t dport, int close, int dir, int stage, int *res,
                     uint16_t *pdport, const struct ctent **hent, uint8_t *k2out)
{
    uint8_t k1[CTK], k2[CTK];
    int action;
    uint16_t td, ts;
    int ret = ct_keys(alen, owner, sa, da, proto, sport, dport, close, dir,
                      k1, k2, &action, &td, &ts);
    if (ret < 0)
        return ret;
    if (k2out)
        memcpy(k2out, k2, CTK);
    /* one or two map lookups in the reference (k1, then k2 on a miss),
     * counted in L whether or not the maps hold entries: ct_lookup4/6 runs
     * them on every tc-path packet (conntrack.h:587-640) */
    tl_lookups++;
    /* *monitor (conntrack.h:221-285, 587-589) against the entry as
     * committed: the batch's own updates are applied afterwards (ct_apply) */
    const struct ctent *ent = NULL;
    /* (stage 2: a NAT64 hop's local delivery, after its IPv4 egress stage) */
    int64_t f = stage >= 1 ? fresh_find(k1) : -1, e;
    if (f >= 0 || (e = ct_find(o, k1)) >= 0) {
        ent = f >= 0 ? &tl_fresh.ent[f] : &o->ct_ents[e];
        *res = (k1[4 + 2 * alen + 5] & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
        *pdport = td;
    } else {
        tl_lookups++;
        f = stage >= 1 ? fresh_find(k2) : -1;
        if (f >= 0 || (e = ct_find(o, k2)) >= 0)
            ent = f >= 0 ? &tl_fresh.ent[f] : &o->ct_ents[e];
        *res = ent ? CT_ESTABLISHED : CT_NEW;
        *pdport = ts;
    }
    if (hent)
        *hent = ent;
    /* __ct_lookup (conntrack.h:241-244): an entry with nat46 asks for the
     * NAT46 translation; ct_lookup6 clears the state after its forward
     * lookup (:429-431) */
    if (ent && (ent->bits & CTB_NAT46) && !tl_nat)
        tl_nat = NAT46;
    if (alen == 16 && *res < CT_REPLY)
        tl_nat = 0;
    uint32_t mon = TRACE_PAYLOAD_LEN;
    if (ent) {
        struct ctent copy = *ent;
        mon = ct_hit_entry(&copy, o->now, action, dir, proto == 6, close,
                           proto == 6 ? tl_tcpfl : 0);
    }
    if (*pdport == 0x3500)   /* conn_is_dns: tuple->dport == htons(53) */
        mon = MTU;
    tl_mon[stage] = mon;
    if (stage == 2)
        tl_ct3 = (uint8_t)(*res | 4);
    else
        tl_ct |= (uint8_t)((*res | 4) << (4 * stage));
    return 0;
}

/* ------------------------------------------------------------ load balancer */
/* IPV4_LOOPBACK (node_config.h:45), raw be32 as stored */
#define IPV4_LOOPBACK 0x1ffff50au

/* the packet's addresses as the program leaves them (cfo_set_lb_io), and
 * skb->hash, per header */
typedef struct {
    uint32_t sa, da;
    uint16_t sport, dport;   /* raw be16, as the L4 header holds them */
} pkt4_t;
static _Thread_local pkt4_t tl_pkt;
static _Thread_local uint32_t tl_hash;

/* one cilium_lb4_services lookup */
static const lb4svc *lb4_get(cfo_t *o, uint32_t addr, uint16_t dport, uint16_t slave)
{
    uint8_t k[8];
    uint32_t v;
    memcpy(k, &addr, 4);
    memcpy(k + 4, &dport, 2);
    memcpy(k + 6, &slave, 2);
    tl_lookups++;
    return ht_get(&o->lb4, k, &v) ? &o->lb4v[v] : NULL;
}

/* lb4_lookup_service (lb.h:604-635): with LB_L4 the key as given while its
 * dport is set, and on a miss the dport is cleared in the caller's key;
 * then (LB_L3) the key with dport 0.  An entry counts only with count != 0. */
static const lb4svc *lb4_lookup_service(cfo_t *o, uint32_t addr, uint16_t *dport,
                                        uint16_t slave)
{
    const lb4svc *v;
    if (*dport) {
        v = lb4_get(o, addr, *dport, slave);
        if (v && v->count)
            return v;
        *dport = 0;
    }
    v = lb4_get(o, addr, 0, slave);
    return v && v->count ? v : NULL;
}

/* What handle_ipv4_from_lxc's service step (bpf_lxc.c:476-492) did to one
 * header: lb4_extract_key, lb4_lookup_service, lb4_local (lb.h:590-776). */
typedef struct {
    int svc;                 /* a service matched */
    int drop;                /* DROP_NO_SERVICE, or 0 */
    uint32_t t_da;           /* tuple->daddr for everything after the step */
    int svc_res;             /* the CT_SERVICE lookup's result */
    int64_t svc_hit;         /* its entry, or -1 */
    int reslave;             /* ct_update4_slave ran (backend gone) */
    uint8_t k_svc[CTK];      /* the CT_SERVICE tuple */
    /* ct_state_new as lb4_local leaves it for ct_create4; slave0: the
     * selection the CT_SERVICE entry is created with */
    uint16_t slave, rev_nat, slave0;
    int loopback;
    uint32_t addr, svc_addr;
} lbx_t;

static void lb4_egress(cfo_t *o, uint16_t owner, uint32_t sa, uint32_t da,
                       uint8_t proto, int close, lbx_t *x)
{
    memset(x, 0, sizeof(*x));
    x->t_da = da;
    x->svc_hit = -1;
    /* lb4_extract_key: key.address = daddr; LB_L4: the L4 dport for TCP and
     * UDP, none for ICMP, and any other protocol skips the service step
     * (DROP_UNKNOWN_L4 -> skip_service_lookup) */
    if (proto != 6 && proto != 17 && proto != 1)
        return;
    uint16_t kd = proto == 1 ? 0 : tl_pkt.dport;
    const lb4svc *svc = lb4_lookup_service(o, da, &kd, 0);
    if (!svc)
        return;
    x->svc = 1;
    /* lb4_local: ct_lookup4(CT_SERVICE) — the tuple as loaded, flags
     * TUPLE_F_SERVICE, one lookup (no reverse, conntrack.h:580); a hit is
     * CT_REPLY (CT_RELATED for ICMP errors) and fills ct_state from the
     * entry (:235-239) */
    uint8_t k2[CTK];
    int action;
    uint16_t td, ts;
    if (ct_keys(4, owner, (const uint8_t *)&sa, (const uint8_t *)&da, proto,
                tl_pkt.sport, tl_pkt.dport, close, CT_SERVICE, x->k_svc, k2,
                &action, &td, &ts) < 0)
        return;
    tl_lookups++;
    x->svc_hit = ct_find(o, x->k_svc);
    if (x->svc_hit >= 0) {
        const struct ctent *e = &o->ct_ents[x->svc_hit];
        x->svc_res = (x->k_svc[4 + 13] & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
        x->rev_nat = e->rev_nat_index;
        x->loopback = (e->bits & CTB_LB_LOOPBACK) != 0;
        x->slave = e->slave;
    } else {
        /* lb4_select_slave (lb.h:158-190): hash % count + 1 */
        x->svc_res = CT_NEW;
        x->slave = (uint16_t)(tl_hash % svc->count + 1);
    }
    x->slave0 = x->slave;
    /* lb4_lookup_slave, then the fall-back to the service itself with the
     * key as it stands (slave set) and a new selection */
    const lb4svc *b = lb4_get(o, da, kd, x->slave);
    if (!b) {
        b = lb4_lookup_service(o, da, &kd, x->slave);
        if (!b) {
            x->drop = DROP_NO_SERVICE;
            return;
        }
        x->slave = (uint16_t)(tl_hash % b->count + 1);
        x->reslave = 1;
    }
    x->rev_nat = b->rev_nat_index;
    x->addr = b->target;
    uint32_t new_sa = 0;
    if (sa == b->target) {   /* !DISABLE_LOOPBACK_LB (lb.h:753-767) */
        new_sa = IPV4_LOOPBACK;
        x->loopback = 1;
        x->addr = new_sa;
        x->svc_addr = sa;
    }
    if (!x->loopback)
        x->t_da = b->target;
    /* lb4_xlate: daddr, the loopback saddr, the L4 dport */
    tl_pkt.da = b->target;
    if (new_sa)
        tl_pkt.sa = new_sa;
    if (b->port && kd != b->port && (proto == 6 || proto == 17))
        tl_pkt.dport = b->port;
}

/* lb4_rev_nat (lb.h:485-588) on the packet for a CT hit with
 * rev_nat_index: source address (and port) from cilium_lb4_reverse_nat; a
 * loopback entry also moves the old source into the destination */
static void lb4_rev_nat(cfo_t *o, const struct ctent *e, uint8_t proto)
{
    tl_lookups++;
    const uint16_t i = e->rev_nat_index;
    if (!o->rnat4_ok[i])
        return;
    const uint16_t port = o->rnat4_port[i];
    if (port && (proto == 6 || proto == 17) && port != tl_pkt.sport)
        tl_pkt.sport = port;   /* reverse_map_l4_port */
    const uint32_t old_sip = tl_pkt.sa;
    if (e->bits & CTB_LB_LOOPBACK)
        tl_pkt.da = old_sip;
    tl_pkt.sa = o->rnat4_addr[i];
}

/* IPv6: the packet as the programs leave it (cfo_set_lb_io) */
typedef struct {
    uint8_t sa[16], da[16];
    uint16_t sport, dport;   /* raw be16, as the L4 header holds them */
} pkt6_t;
static _Thread_local pkt6_t tl_pkt6;

/* one cilium_lb6_services lookup */
static const lb6svc *lb6_get(cfo_t *o, const uint8_t addr[16], uint16_t dport,
                             uint16_t slave)
{
    uint8_t k[20];
    uint32_t v;
    memcpy(k, addr, 16);
    memcpy(k + 16, &dport, 2);
    memcpy(k + 18, &slave, 2);
    tl_lookups++;
    return ht_get(&o->lb6, k, &v) ? &o->lb6v[v] : NULL;
}

/* lb6_lookup_service (lb.h:352-381): as lb4_lookup_service */
static const lb6svc *lb6_lookup_service(cfo_t *o, const uint8_t addr[16],
                                        uint16_t *dport, uint16_t slave)
{
    const lb6svc *v;
    if (*dport) {
        v = lb6_get(o, addr, *dport, slave);
        if (v && v->count)
            return v;
        *dport = 0;
    }
    v = lb6_get(o, addr, 0, slave);
    return v && v->count ? v : NULL;
}

/* What ipv6_l3_from_lxc's service step (bpf_lxc.c:149-167) did to one
 * header: lb6_extract_key (lb.h:336-350), lb6_lookup_service, lb6_local
 * (:427-481).  No loopback translation and no reverse-NAT CT entry for
 * IPv6 (ct_create6, conntrack.h:615-662, writes the flow's entry and its
 * ICMPv6 entry only). */
typedef struct {
    int svc, drop;
    uint8_t t_da[16];        /* tuple->daddr (orig_dip) after the step */
    int64_t svc_hit;         /* the CT_SERVICE entry, or -1 */
    int reslave;
    uint8_t k_svc[CTK];
    uint16_t slave, rev_nat, slave0;
} lbx6_t;

static void lb6_egress(cfo_t *o, uint16_t owner, const uint8_t *sa, const uint8_t *da,
                       uint8_t proto, int close, lbx6_t *x)
{
    memset(x, 0, sizeof(*x));
    memcpy(x->t_da, da, 16);
    x->svc_hit = -1;
    /* lb6_extract_key: key.address = tuple->daddr; extract_l4_port: TCP
     * and UDP the dport, ICMPv6 none, anything else DROP_UNKNOWN_L4 ->
     * skip_service_lookup */
    if (proto != 6 && proto != 17 && proto != 58)
        return;
    if (!o->lb6_n)
        return;
    uint16_t kd = proto == 58 ? 0 : tl_pkt6.dport;
    const lb6svc *svc = lb6_lookup_service(o, da, &kd, 0);
    if (!svc)
        return;
    x->svc = 1;
    /* lb6_local: ct_lookup6(CT_SERVICE) — one lookup of the tuple as
     * loaded with TUPLE_F_SERVICE (conntrack.h:414-424); a hit fills
     * ct_state from the entry */
    uint8_t k2[CTK];
    int action;
    uint16_t td, ts;
    if (ct_keys(16, owner, sa, da, proto, tl_pkt6.sport, tl_pkt6.dport, close, CT_SERVICE,
                x->k_svc, k2, &action, &td, &ts) < 0)
        return;
    tl_lookups++;
    x->svc_hit = ct_find(o, x->k_svc);
    if (x->svc_hit >= 0) {
        x->slave = o->ct_ents[x->svc_hit].slave;
    } else {
        /* lb6_select_slave (lb.h:124-152): hash % count + 1 */
        x->slave = (uint16_t)(tl_hash % svc->count + 1);
    }
    x->slave0 = x->slave;
    /* lb6_lookup_slave, then the fall-back to the service with the key as
     * it stands (slave set) and a new selection (ct_update6_slave) */
    const lb6svc *b = lb6_get(o, da, kd, x->slave);
    if (!b) {
        b = lb6_lookup_service(o, da, &kd, x->slave);
        if (!b) {
            x->drop = DROP_NO_SERVICE;
            return;
        }
        x->slave = (uint16_t)(tl_hash % b->count + 1);
        x->reslave = 1;
    }
    x->rev_nat = b->rev_nat_index;
    memcpy(x->t_da, b->target, 16);
    /* lb6_xlate: daddr, then the L4 dport (the tuple's ports are reloaded
     * from the packet by the next ct_lookup6) */
    memcpy(tl_pkt6.da, b->target, 16);
    if (b->port && kd != b->port && (proto == 6 || proto == 17))
        tl_pkt6.dport = b->port;
}

/* lb6_rev_nat (lb.h:306-319) with flags 0: the packet's source address
 * (and port: reverse_map_l4_port) from cilium_lb6_reverse_nat[index] */
static void lb6_rev_nat(cfo_t *o, uint16_t index, uint8_t proto)
{
    tl_lookups++;
    if (!o->rnat6_ok[index])
        return;
    const uint16_t port = o->rnat6_port[index];
    if (port && (proto == 6 || proto == 17) && port != tl_pkt6.sport)
        tl_pkt6.sport = port;
    memcpy(tl_pkt6.sa, o->rnat6_addr + 16 * (size_t)index, 16);
}

/* ipv4_policy (bpf_lxc.c:898-1015) + tail_ipv4_policy (:1017-1028) for
 * endpoint ep, called after local delivery with cb[CB_SRC_LABEL]=src; with
 * alen 16, ipv6_policy (:753-882) + tail_ipv6_policy (:884-895), which
 * differ only in the CT tuple and pass is_fragment = false.  stage is 0 for
 * an ingress batch, 1 after egress local delivery. */
/* ---- NAT46 / NAT64 (LXC_NAT46: lxc_config.h:28 ENABLE_NAT46 with IPv4 and
 * CONNTRACK, nat46.h:30-32).  Header ports of ICMP hold {type, code} in the
 * sport word; the translations rewrite them. */
#define DROP_INVALID -134
#define DROP_INVALID_EXTHDR -156
#define IPPROTO_ICMP 1
#define IPPROTO_ICMPV6 58
#define HF_EXTHDR 4
#define DROP_UNKNOWN_ICMP_CODE -143
#define DROP_UNKNOWN_ICMP_TYPE -144
#define DROP_UNKNOWN_ICMP6_CODE -145
#define DROP_UNKNOWN_ICMP6_TYPE -146
/* NAT46_PREFIX (node_config.h:40): the translated source's first 96 bits */
static const uint8_t nat46_prefix[12] = {0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0x0a, 0};

/* icmp4_to_icmp6 (nat46.h:60-141) on {type, code}.  Its callers use the
 * return value as a checksum difference and never test it (nat46.h:303,
 * :384): an "error" only leaves the ICMP header untranslated — no drop. */
static int icmp4_to_icmp6(uint16_t *w)
{
    const uint8_t type = (uint8_t)(*w & 0xFF), code = (uint8_t)(*w >> 8);
    uint8_t t6 = 0, c6 = 0;
    switch (type) {
    case 8: t6 = 128; break;                        /* ECHO -> ECHO_REQUEST */
    case 0: t6 = 129; break;                        /* ECHOREPLY */
    case 3:                                         /* DEST_UNREACH */
        t6 = 1;
        switch (code) {
        case 0: case 1: c6 = 0; break;              /* NOROUTE */
        case 2: t6 = 4; c6 = 1; break;              /* PARAMPROB / UNK_NEXTHDR */
        case 3: c6 = 4; break;                      /* PORT_UNREACH */
        case 4: t6 = 2; c6 = 0; break;              /* PKT_TOOBIG */
        case 5: c6 = 0; break;
        case 6: case 7: case 8: case 11: case 12: c6 = 0; break;
        case 9: case 10: case 13: c6 = 1; break;    /* ADM_PROHIBITED */
        default: return DROP_UNKNOWN_ICMP_CODE;
        }
        break;
    case 11: t6 = 3; break;                         /* TIME_EXCEEDED (code 0) */
    case 12: t6 = 4; break;                         /* PARAMETERPROB */
    default: return DROP_UNKNOWN_ICMP_TYPE;
    }
    *w = (uint16_t)(t6 | c6 << 8);
    return 0;
}

/* icmp6_to_icmp4 (nat46.h:143-220), fall-throughs included: a destination
 * unreachable with a known code ends as ICMP_FRAG_NEEDED (no break after
 * its inner switch), a parameter problem always as an unknown type */
static int icmp6_to_icmp4(uint16_t *w)
{
    const uint8_t type = (uint8_t)(*w & 0xFF), code = (uint8_t)(*w >> 8);
    uint8_t t4 = 0, c4 = 0;
    switch (type) {
    case 128: t4 = 8; break;
    case 129: t4 = 0; break;
    case 1:
        if (code != 0 && code != 2 && code != 3 && code != 1 && code != 4)
            return DROP_UNKNOWN_ICMP6_CODE;
        /* fall through */
    case 2: t4 = 3; c4 = 4; break;                  /* DEST_UNREACH / FRAG_NEEDED */
    case 3: t4 = 11; c4 = code; break;              /* TIME_EXCEED */
    case 4:
        if (code != 0 && code != 1)
            return DROP_UNKNOWN_ICMP6_CODE;
        return DROP_UNKNOWN_ICMP6_TYPE;
    default:
        return DROP_UNKNOWN_ICMP6_TYPE;
    }
    *w = (uint16_t)(t4 | c4 << 8);
    return 0;
}

static res_t lxc_ingress(cfo_t *o, const epinfo *ep, uint32_t src, int alen,
                         const uint8_t *sa, const uint8_t *da, uint8_t proto,
                         uint16_t sport, uint16_t dport, int frag, int close,
                         uint32_t len, int skip_proxy, int dir_missed,
                         int stage);

/* ipv4_policy's NAT46 tail call (bpf_lxc.c:939-944): tail_ipv4_to_ipv6
 * (:1098-1110) — ipv4_to_ipv6 (nat46.h:236-328): saddr NAT46_PREFIX/96 +
 * the IPv4 source, daddr the endpoint's LXC_IP, ICMP as ICMPv6 — then
 * tail_ipv6_policy on the translated packet with the source identity of
 * the IPv4 path (cb[CB_SRC_LABEL]); its CT lookup is stage 1 behind
 * from-netdev, stage 2 (tl_ct3, struct hop ct2, has2 = 2) behind an IPv4
 * egress batch's local delivery (ipv4_local_delivery, l3.h:103-131, whose
 * ipv4_policy lookup is stage 1) */
static res_t nat46_ingress(cfo_t *o, const epinfo *ep, uint32_t src, uint32_t sa4,
                           uint8_t proto, uint16_t sport, uint16_t dport, int close,
                           uint32_t len, int skip_proxy, int stage)
{
    uint16_t sp = sport;
    const uint8_t p6 = proto == IPPROTO_ICMP ? IPPROTO_ICMPV6 : proto;
    if (proto == IPPROTO_ICMP)   /* (unchecked: see icmp4_to_icmp6) */
        (void)icmp4_to_icmp6(&sp);
    uint8_t sa6[16], da6[16];
    memcpy(sa6, nat46_prefix, 12);
    memcpy(sa6 + 12, &sa4, 4);
    memcpy(da6, o->ep_v6[ep->lxc_id], 16);
    tl_hop = (struct hop){HOP_NAT46, 16, p6, CT_INGRESS, ct_owner(o, ep->lxc_id), sp, dport,
                          {0}, {0}, 20, 0, 0, 0, 0, 0, {0}, {0}};
    tl_hop.has2 = stage == 2 ? 2 : 0;
    memcpy(tl_hop.sa, sa6, 16);
    memcpy(tl_hop.da, da6, 16);
    memcpy(tl_pkt6.sa, sa6, 16);
    memcpy(tl_pkt6.da, da6, 16);
    tl_pkt6.sport = sp;
    tl_pkt6.dport = dport;
    return lxc_ingress(o, ep, src, 16, sa6, da6, p6, sp, dport, 0, close, len + 20,
                       skip_proxy, METRIC_INGRESS, stage);
}

static res_t lxc_ingress(cfo_t *o, const epinfo *ep, uint32_t src, int alen,
                         const uint8_t *sa, const uint8_t *da, uint8_t proto,
                         uint16_t sport, uint16_t dport, int frag, int close,
                         uint32_t len, int skip_proxy, int dir_missed,
                         int stage)
{
    res_t r = {TC_ACT_SHOT, 0, src, 0};
    if (!o->pol[ep->lxc_id]) {
        /* no endpoint program behind cilium_policy[lxc_id]: the tail call
         * in ipv4_local_delivery (l3.h:130) falls through and the caller
         * drops with DROP_MISSED_TAIL_CALL */
        r.verdict = DROP_MISSED_TAIL_CALL;
        metric(o, DROP_MISSED_TAIL_CALL, dir_missed, len);
        return r;
    }
    uint16_t pdport;
    int res;
    const struct ctent *hit;
    /* ipv6_policy (:785-801): the tuple keeps daddr, the packet's daddr
     * loses the low 16 bits of its last word (the rev_nat_index a create
     * stores) */
    uint8_t da0[16];
    if (alen == 16) {
        memcpy(da0, da, 16);
        da = da0;
        uint16_t rv;
        memcpy(&rv, tl_pkt6.da + 12, 2);
        if (rv)
            memset(tl_pkt6.da + 12, 0, 2);
    }
    int ret = ct_lookup(o, alen, ct_owner(o, ep->lxc_id), sa, da, proto, sport,
                        dport, close, CT_INGRESS, stage, &res, &pdport, &hit, NULL);
    if (ret < 0) {
        r.verdict = ret;
        r.nt = NT_POLICY << 16 | ep->lxc_id;
        metric(o, ret, METRIC_INGRESS, len);
        return r;
    }
    if (alen == 4 && tl_nat == NAT46 && o->ep_has6[ep->lxc_id]) {
        uint32_t sa4;
        memcpy(&sa4, sa, 4);
        /* (stage 1 is an IPv4 egress batch's local delivery: the hop is a
         * third stage; behind from-netdev, and behind a NAT64 hop's local
         * delivery as before, it takes stage 1) */
        return nat46_ingress(o, ep, src, sa4, proto, sport, dport, close, len, skip_proxy,
                             stage == 1 ? 2 : 1);
    }
    /* (:808-815) any hit whose entry carries a rev_nat_index: the packet's
     * source from cilium_lb6_reverse_nat, when it holds the index */
    if (alen == 16 && hit && hit->rev_nat_index)
        lb6_rev_nat(o, hit->rev_nat_index, proto);
    /* bpf_lxc.c:946-955: a reply of a load-balanced flow gets its source
     * translated back (packet only: the verdict does not depend on it) */
    if (alen == 4 && res == CT_REPLY && hit->rev_nat_index &&
        !(hit->bits & CTB_LB_LOOPBACK))
        lb4_rev_nat(o, hit, proto);
    int verdict = policy_can_access(o->pol[ep->lxc_id], src, pdport, proto,
                                    CT_INGRESS, frag, len);
    id_event(o, 0, src, res != CT_REPLY && res != CT_RELATED && verdict < 0, len);
    /* replies and related packets skip the policy verdict (:963-970); a
     * denied CT_ESTABLISHED flow loses its entry (ct_delete4) */
    if (res != CT_REPLY && res != CT_RELATED && verdict < 0) {
        r.verdict = DROP_POLICY;
        r.nt = NT_POLICY << 16 | ep->lxc_id;
        metric(o, DROP_POLICY, METRIC_INGRESS, len);
        return r;
    }
    if (skip_proxy)
        verdict = 0;
    if (res == CT_NEW) {   /* ct_create4 */
        if (stage == 2)
            tl_ct3 |= CTO_CREATE1;
        else
            tl_ct |= (uint8_t)(CTO_CREATE1 << (4 * stage));
    }
    if (verdict > 0 && (res == CT_NEW || res == CT_ESTABLISHED)) {
        /* redirect_to_proxy: cb[CB_IFINDEX] = HOST_IFINDEX; TRACE_TO_PROXY
         * from ipv4_redirect_to_host_port (lxc.h:117) */
        r.action = TC_ACT_REDIRECT;
        r.verdict = verdict;
        r.nt = trace_word(OBS_TO_PROXY, ep->lxc_id, res, tl_mon[stage]);
        return r;
    }
    metric(o, 0, METRIC_INGRESS, len); /* send_trace_notify(TRACE_TO_LXC) */
    r.action = ep->ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
    r.verdict = 0;
    r.nt = trace_word(OBS_TO_LXC, ep->lxc_id, res, tl_mon[stage]);   /* :1006 */
    return r;
}

/* handle_identity_from_host (bpf_netdev.c:128-153) */
static uint32_t identity_from_mark(uint32_t mark, int *skip_proxy)
{
    uint32_t magic = mark & MARK_MAGIC_HOST_MASK;
    *skip_proxy = 0;
    if (magic == MARK_MAGIC_PROXY_INGRESS || magic == MARK_MAGIC_PROXY_EGRESS) {
        *skip_proxy = magic == MARK_MAGIC_PROXY_INGRESS;
        return ((mark & 0xFF) << 16) | (mark >> 16);
    }
    return magic == MARK_MAGIC_HOST ? HOST_ID : WORLD_ID;
}

/* from_netdev (FROM_HOST) -> handle_ipv4 (bpf_netdev.c:128-153, 357-453) */
static res_t netdev_ingress_v4(cfo_t *o, uint32_t saddr, uint32_t daddr,
                               uint8_t proto, uint16_t sport, uint16_t dport,
                               uint8_t hflags, uint32_t len, uint32_t mark)
{
    int skip_proxy;
    uint32_t identity = identity_from_mark(mark, &skip_proxy);
    if (identity < HEALTH_ID) { /* identity_is_reserved, policy.h:41-44 */
        uint32_t label;
        tl_lookups++;
        if (lpm_lookup(&o->ipc4, (const uint8_t *)&saddr, &label) && label &&
            label != CLUSTER_ID && label != HOST_ID)
            identity = label;
    }
    res_t r = {TC_ACT_OK, 0, identity, 0};
    tl_lookups++;
    const epinfo *ep = lxc_lookup(o, 1, (const uint8_t *)&daddr);
    if (!ep || (ep->flags & ENDPOINT_F_HOST))
        return r; /* to the stack (tunnel endpoints out of scope) */
    return lxc_ingress(o, ep, identity, 4, (const uint8_t *)&saddr,
                       (const uint8_t *)&daddr, proto, sport, dport,
                       hflags & HF_FRAG, hflags & HF_TCP_CLOSE, len,
                       skip_proxy, METRIC_INGRESS, 0);
}

/* handle_ipv4_from_lxc (bpf_lxc.c:440-692) for endpoint lxc */
static res_t lxc_egress_v4(cfo_t *o, uint16_t lxc, uint32_t saddr,
                           uint32_t daddr, uint8_t proto, uint16_t sport,
                           uint16_t dport, uint8_t hflags, uint32_t len, int st0)
{
    (void)sport;
    (void)dport;   /* the packet's ports are tl_pkt's */
    res_t r = {TC_ACT_SHOT, 0, 0, 0};
    const epinfo *self = lxc_lookup(o, 1, (const uint8_t *)&saddr);
    if (!self || self->lxc_id != lxc) { /* is_valid_lxc_src_ipv4, lxc.h:55 */
        r.verdict = DROP_INVALID_SIP;
        metric(o, DROP_INVALID_SIP, METRIC_EGRESS, len);
        return r;
    }
    /* the service step (:476-492); the tuple's daddr may change */
    lbx_t x;
    lb4_egress(o, ct_owner(o, lxc), saddr, daddr, proto, hflags & HF_TCP_CLOSE, &x);
    if (x.drop) {
        r.verdict = x.drop;
        metric(o, x.drop, METRIC_EGRESS, len);
        return r;
    }
    const uint32_t tda = x.t_da;   /* orig_dip */
    const uint8_t *sa = (const uint8_t *)&saddr, *da = (const uint8_t *)&tda;
    uint16_t pdport;
    int res;
    const struct ctent *hit;
    uint8_t k2[CTK];
    int ret = ct_lookup(o, 4, ct_owner(o, lxc), sa, da, proto, tl_pkt.sport,
                        tl_pkt.dport, hflags & HF_TCP_CLOSE, CT_EGRESS, st0, &res,
                        &pdport, &hit, k2);
    if (ret < 0) {
        r.verdict = ret;
        metric(o, ret, METRIC_EGRESS, len);
        return r;
    }
    uint32_t label = 0, dst;
    tl_lookups++;
    if (lpm_lookup(&o->ipc4, da, &label) && label)
        dst = label;
    else if ((tda & o->v4_cluster_mask) == o->v4_cluster_range)
        dst = CLUSTER_ID;
    else
        dst = WORLD_ID;
    r.identity = dst;
    int verdict = policy_can_access(o->pol[lxc], dst, pdport, proto,
                                    CT_EGRESS, 0, len);
    id_event(o, 1, dst, res != CT_REPLY && res != CT_RELATED && verdict < 0, len);
    if (res != CT_REPLY && res != CT_RELATED && verdict < 0) { /* :538-545 */
        r.verdict = DROP_POLICY;
        metric(o, DROP_POLICY, METRIC_EGRESS, len);
        return r;
    }
    if (res == CT_NEW) {                            /* ct_create4, :547-559 */
        tl_ct |= (uint8_t)(CTO_CREATE1 << (4 * st0));
        ctstate_t cs = {0, 0, 0, 0, 0, 0};
        if (x.svc)
            cs = (ctstate_t){x.rev_nat, x.slave, x.loopback, x.addr, x.svc_addr, 0};
        cs.nat46 = tl_nat == NAT64;
        tl_fresh.n = ct_create_entries(o, k2, 4, CT_EGRESS, len, o->seclabel[lxc], &cs,
                                       tl_fresh.key, tl_fresh.ent);
    } else if (res >= CT_REPLY && hit->rev_nat_index) {
        lb4_rev_nat(o, hit, proto);                 /* :565-576 */
    }
    if (verdict > 0) { /* proxy: redirect(HOST_IFINDEX), TRACE_TO_PROXY */
        r.action = TC_ACT_REDIRECT;
        r.verdict = verdict;
        r.nt = trace_word(OBS_TO_PROXY, lxc, res, tl_mon[st0]);
        return r;
    }
    /* delivery by the packet's destination (lookup_ip4_endpoint, :617) */
    const uint8_t *pda = (const uint8_t *)&tl_pkt.da;
    tl_lookups++;
    const epinfo *ep = lxc_lookup(o, 1, pda);
    if (ep) {
        if (ep->flags & ENDPOINT_F_HOST) { /* to_host: TRACE_TO_HOST, :668 */
            metric(o, 0, METRIC_EGRESS, len);
            r.action = TC_ACT_REDIRECT;
            r.nt = trace_word(OBS_TO_HOST, lxc, res, tl_mon[st0]);
            return r;
        }
        /* ipv4_local_delivery (l3.h:103-131): egress forward metric, then
         * the destination's policy program with src = SECLABEL, on the
         * packet as it now is */
        metric(o, 0, METRIC_EGRESS, len);
        const uint32_t psa = tl_pkt.sa, pd = tl_pkt.da;
        const uint16_t psp = tl_pkt.sport, pdp = tl_pkt.dport;
        /* (after a NAT64 hop the destination's lookup is a third CT stage:
         * recorded with the hop, applied after its IPv4 egress stage) */
        res_t d = lxc_ingress(o, ep, o->seclabel[lxc], 4, (const uint8_t *)&psa,
                              (const uint8_t *)&pd, proto, psp, pdp,
                              hflags & HF_FRAG, hflags & HF_TCP_CLOSE,
                              len, 0, METRIC_EGRESS, st0 + 1);
        if (st0 == 1 && tl_hop.kind == HOP_NAT64 && (tl_ct3 & 4)) {
            tl_hop.has2 = 1;
            tl_hop.owner2 = ct_owner(o, ep->lxc_id);
            tl_hop.sport2 = psp;
            tl_hop.dport2 = pdp;
            memcpy(tl_hop.sa2, &psa, 4);
            memcpy(tl_hop.da2, &pd, 4);
        }
        d.identity = dst;
        return d;
    }
    metric(o, 0, METRIC_EGRESS, len); /* pass_to_stack: TRACE_TO_STACK */
    r.action = TC_ACT_OK;
    r.nt = trace_word(OBS_TO_STACK, lxc, res, tl_mon[st0]);   /* :687 */
    return r;
}

/* ipv6_l3_from_lxc's NAT64 tail call (bpf_lxc.c:353-360, a destination
 * outside the cluster in ::ffff:0:0/96, ipv6.h:279-282): tail_ipv6_to_ipv4
 * (:1070-1083) — ipv6_to_ipv4 (nat46.h:336-420): saddr the endpoint's
 * LXC_IPV4, daddr the last 32 bits, ICMPv6 as ICMP, extension headers
 * dropped — then handle_ipv4_from_lxc with cb[CB_NAT46_STATE] = NAT64 (its
 * creates carry nat46); its CT lookup is stage 1 */
static res_t nat64_egress(cfo_t *o, uint16_t lxc, const uint8_t *da6, uint8_t proto,
                          uint8_t flags, uint32_t len)
{
    res_t r = {TC_ACT_SHOT, 0, 0, 0};
    uint16_t sp = tl_pkt6.sport;
    const uint16_t dp = tl_pkt6.dport;
    const uint8_t p4 = proto == IPPROTO_ICMPV6 ? IPPROTO_ICMP : proto;
    const int ret = (flags & HF_EXTHDR) ? DROP_INVALID_EXTHDR : 0;
    if (ret || !o->ep_has4[lxc]) {   /* send_drop_notify(skb, SECLABEL, 0, ..) */
        r.verdict = ret ? ret : DROP_INVALID;
        metric(o, r.verdict, METRIC_EGRESS, len);
        return r;
    }
    if (proto == IPPROTO_ICMPV6)   /* (unchecked: see icmp4_to_icmp6) */
        (void)icmp6_to_icmp4(&sp);
    const uint32_t sa4 = o->ep_v4[lxc];
    uint32_t da4;
    memcpy(&da4, da6 + 12, 4);
    tl_nat = NAT64;
    tl_hop = (struct hop){HOP_NAT64, 4, p4, CT_EGRESS, ct_owner(o, lxc), sp, dp, {0}, {0}, -20,
                          0, 0, 0, 0, 0, {0}, {0}};
    memcpy(tl_hop.sa, &sa4, 4);
    memcpy(tl_hop.da, &da4, 4);
    tl_pkt = (pkt4_t){sa4, da4, sp, dp};
    return lxc_egress_v4(o, lxc, sa4, da4, p4, sp, dp, flags, len - 20, 1);
}

/* check_v4 (bpf_xdp.c:97-121) */
static int xdp_v4(cfo_t *o, uint32_t saddr, uint32_t daddr)
{
    uint32_t v;
    /* the dyn (LPM) lookup only exists when CIDR4_LPM_PREFILTER is compiled
     * in; production keeps it off (prefilter.go:282-289): count it only
     * when that map holds entries */
    if (o->pf4_dyn.nlens)
        tl_lookups++;
    if (lpm_lookup(&o->pf4_dyn, (const uint8_t *)&saddr, &v))
        return XDP_DROP;
    uint8_t k[8];
    uint32_t pl = 32;
    memcpy(k, &pl, 4);
    memcpy(k + 4, &saddr, 4);
    tl_lookups++;
    if (ht_get(&o->pf4_fix, k, &v))
        return XDP_DROP;
    tl_lookups++;
    return lxc_lookup(o, 1, (const uint8_t *)&daddr) ? XDP_PASS : XDP_DROP;
}

/* the per-header NAT hop records of a classify of n headers */
static void hop_reserve(cfo_t *o, size_t n)
{
    if (n > o->hop_cap) {
        free(o->hop);
        o->hop_cap = n;
        o->hop = calloc(n, sizeof(struct hop));
    }
}

void cfo_classify_v4(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint32_t *saddr, const uint32_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint32_t *mark,
                     const uint8_t *tcpflags, int32_t *action, int32_t *verdict,
                     uint32_t *identity, uint8_t *lookups, uint8_t *ct,
                     int nthreads)
{
    hop_reserve(o, n);
    if (nthreads <= 0)
        nthreads = 1;
#pragma omp parallel for schedule(static, 4096) num_threads(nthreads)
    for (size_t i = 0; i < n; i++) {
        res_t r;
        tl_lookups = 0;
        tl_ct = 0;
        tl_ct3 = 0;
        tl_tcpfl = tcpflags ? tcpflags[i] : 0;
        tl_mon[0] = tl_mon[1] = tl_mon[2] = 0;
        tl_fresh.n = 0;
        tl_nat = 0;
        tl_hop.kind = 0;
        tl_hop.has2 = 0;
        tl_pkt.sa = saddr[i];
        tl_pkt.da = daddr[i];
        tl_pkt.sport = sport[i];
        tl_pkt.dport = dport[i];
        tl_hash = o->hash_in ? o->hash_in[i]
                             : cfo_flow_hash4(saddr[i], daddr[i], sport[i], dport[i],
                                              proto[i]);
        if (o->pkt_out) {   /* (XDP verdicts leave the packet as it is) */
            o->pkt_out[3 * i] = saddr[i];
            o->pkt_out[3 * i + 1] = daddr[i];
            o->pkt_out[3 * i + 2] = sport[i] | (uint32_t)dport[i] << 16;
        }
        if (mode == CFO_MODE_XDP || mode == CFO_MODE_FULL) {
            int x = xdp_v4(o, saddr[i], daddr[i]);
            if (mode == CFO_MODE_XDP || x == XDP_DROP) {
                action[i] = x;
                verdict[i] = x == XDP_PASS ? 0 : -1;
                identity[i] = 0;
                if (lookups)
                    lookups[i] = (uint8_t)tl_lookups;
                if (ct)
                    ct[i] = 0;
                if (o->notify_out)
                    o->notify_out[i] = 0;
                if (o->notify_mon)
                    o->notify_mon[i] = 0;
                o->hop[i].kind = 0;
                continue;
            }
        }
        if (mode == CFO_MODE_EGRESS)
            r = lxc_egress_v4(o, ep_lxc, saddr[i], daddr[i], proto[i],
                              sport[i], dport[i], flags[i], len[i], 0);
        else
            r = netdev_ingress_v4(o, saddr[i], daddr[i], proto[i], sport[i],
                                  dport[i], flags[i], len[i],
                                  mark ? mark[i] : 0);
        action[i] = r.action;
        verdict[i] = r.verdict;
        identity[i] = r.identity;
        if (lookups)
            lookups[i] = (uint8_t)tl_lookups;
        if (ct)
            ct[i] = tl_ct;
        if (o->notify_out) {
            const uint32_t w = notify_site(mode, ep_lxc, &r);
            /* (an event after a NAT hop: skb->len of the translated packet) */
            o->notify_out[i] = w && tl_hop.kind ? w | NT_NATLEN : w;
        }
        if (o->notify_mon)   /* both stages' monitor lengths (ct_apply) */
            o->notify_mon[i] = tl_mon[0] | tl_mon[1] << 16;
        tl_hop.ct2 = tl_hop.has2 ? tl_ct3 : 0;
        o->hop[i] = tl_hop;
        if (o->pkt_out) {
            o->pkt_out[3 * i] = tl_pkt.sa;
            o->pkt_out[3 * i + 1] = tl_pkt.da;
            o->pkt_out[3 * i + 2] = tl_pkt.sport | (uint32_t)tl_pkt.dport << 16;
        }
    }
}

/* ------------------------------------------------------------ IPv6 */
#define NEXTHDR_FRAGMENT 44
#define NEXTHDR_NONE 59
#define VERDICT_PUNT -2

/* ipv6_hdrlen (ipv6.h:61-98): the header's proto is the next header the
 * extension-header walk stops at; NONE and FRAGMENT end in a drop. */
static int exthdr_drop(uint8_t proto)
{
    return proto == NEXTHDR_NONE ? DROP_INVALID_EXTHDR
           : proto == NEXTHDR_FRAGMENT ? DROP_FRAG_NOSUPPORT : 0;
}

/* icmp6_handle (icmp6.h:390-412) answers neighbour solicitations and echo
 * requests to the router itself; those headers are reported as punted.  It
 * reads the type right after the fixed header, so behind extension headers
 * it sees the next-header byte and never triggers. */
static int icmp6_punt(const cfo_t *o, uint8_t proto, uint8_t flags,
                      uint16_t sport, const uint8_t *daddr)
{
    if (proto != IPPROTO_ICMPV6 || (flags & HF_EXTHDR))
        return 0;
    uint8_t type = (uint8_t)(sport & 0xFF);
    return type == 135 || (type == 128 && !memcmp(daddr, o->router_ip6, 16));
}

/* from_netdev (FROM_HOST) -> handle_ipv6 (bpf_netdev.c:172-275, 494-503) */
static res_t netdev_ingress_v6(cfo_t *o, const uint8_t *saddr,
                               const uint8_t *daddr, uint8_t proto,
                               uint16_t sport, uint16_t dport, uint8_t flags,
                               uint32_t len, uint32_t mark)
{
    int skip_proxy;
    uint32_t identity = identity_from_mark(mark, &skip_proxy);
    res_t r = {TC_ACT_SHOT, 0, 0, 0};
    int ret = exthdr_drop(proto);
    if (ret) { /* send_drop_notify_error(skb, ret, TC_ACT_SHOT, INGRESS) */
        r.verdict = ret;
        metric(o, ret, METRIC_INGRESS, len);
        return r;
    }
    if (icmp6_punt(o, proto, flags, sport, daddr)) {
        r.action = TC_ACT_OK;
        r.verdict = VERDICT_PUNT;
        return r;
    }
    if (identity < HEALTH_ID) { /* :203-213, no HOST_ID exclusion for v6 */
        uint32_t label;
        tl_lookups++;
        if (lpm_lookup(&o->ipc6, saddr, &label) && label && label != CLUSTER_ID)
            identity = label;
    }
    r.action = TC_ACT_OK;
    r.identity = identity;
    tl_lookups++;
    const epinfo *ep = lxc_lookup(o, 2, daddr);
    if (!ep || (ep->flags & ENDPOINT_F_HOST))
        return r;
    return lxc_ingress(o, ep, identity, 16, saddr, daddr, proto, sport, dport,
                       0, flags & HF_TCP_CLOSE, len, skip_proxy,
                       METRIC_INGRESS, 0);
}

/* from-container -> handle_ipv6 -> ipv6_l3_from_lxc (bpf_lxc.c:112-436) */
static res_t lxc_egress_v6(cfo_t *o, uint16_t lxc, const uint8_t *saddr,
                           const uint8_t *daddr, uint8_t proto, uint16_t sport,
                           uint16_t dport, uint8_t flags, uint32_t len)
{
    res_t r = {TC_ACT_SHOT, 0, 0, 0};
    if (icmp6_punt(o, proto, flags, sport, daddr)) { /* :411-419 */
        r.action = TC_ACT_OK;
        r.verdict = VERDICT_PUNT;
        return r;
    }
    const epinfo *self = lxc_lookup(o, 2, saddr);
    if (!self || self->lxc_id != lxc) { /* is_valid_lxc_src_ip, lxc.h:46 */
        r.verdict = DROP_INVALID_SIP;
        metric(o, DROP_INVALID_SIP, METRIC_EGRESS, len);
        return r;
    }
    (void)sport;
    (void)dport;   /* the packet's ports are tl_pkt6's */
    int ret = exthdr_drop(proto);
    uint16_t pdport;
    int res;
    const struct ctent *hit = NULL;
    /* the service step (:149-167); the tuple's daddr may change */
    lbx6_t x;
    memset(&x, 0, sizeof(x));
    memcpy(x.t_da, daddr, 16);
    if (!ret) {
        lb6_egress(o, ct_owner(o, lxc), saddr, daddr, proto, flags & HF_TCP_CLOSE, &x);
        ret = x.drop;
    }
    const uint8_t *tda = x.t_da;   /* orig_dip */
    uint8_t k2[CTK];
    if (!ret)
        ret = ct_lookup(o, 16, ct_owner(o, lxc), saddr, tda, proto, tl_pkt6.sport,
                        tl_pkt6.dport, flags & HF_TCP_CLOSE, CT_EGRESS, 0, &res,
                        &pdport, &hit, k2);
    if (ret) {
        r.verdict = ret;
        metric(o, ret, METRIC_EGRESS, len);
        return r;
    }
    uint32_t label = 0, dst;
    tl_lookups++;
    if (lpm_lookup(&o->ipc6, tda, &label) && label)
        dst = label;
    else if (!memcmp(tl_pkt6.da, o->router_ip6, 8)) /* ipv6_match_prefix_64 */
        dst = CLUSTER_ID;
    else
        dst = WORLD_ID;
    r.identity = dst;
    int verdict = policy_can_access(o->pol[lxc], dst, pdport, proto,
                                    CT_EGRESS, 0, len);
    id_event(o, 1, dst, res != CT_REPLY && res != CT_RELATED && verdict < 0, len);
    if (res != CT_REPLY && res != CT_RELATED && verdict < 0) { /* :228-235 */
        r.verdict = DROP_POLICY;
        metric(o, DROP_POLICY, METRIC_EGRESS, len);
        return r;
    }
    /* after ct_create6 the v6 egress path sets monitor = TRACE_PAYLOAD_LEN
     * (bpf_lxc.c:248), so a new DNS flow is not captured at MTU */
    const uint32_t mon = res == CT_NEW ? TRACE_PAYLOAD_LEN : tl_mon[0];
    if (res == CT_NEW) {
        tl_ct |= CTO_CREATE1;                       /* ct_create6, :237-249 */
        /* (the destination's lookup after local delivery sees them: an
         * endpoint's traffic to itself, whose tuple and its reverse
         * coincide, finds its own entry, CT_REPLY) */
        ctstate_t cs = {0, 0, 0, 0, 0, 0};
        if (x.svc)
            cs = (ctstate_t){x.rev_nat, x.slave, 0, 0, 0, 0};
        tl_fresh.n = ct_create_entries(o, k2, 16, CT_EGRESS, len, o->seclabel[lxc], &cs,
                                       tl_fresh.key, tl_fresh.ent);
    } else if (res >= CT_REPLY && hit->rev_nat_index)
        lb6_rev_nat(o, hit->rev_nat_index, proto);  /* :255-266 */
    if (verdict > 0) {
        r.action = TC_ACT_REDIRECT;
        r.verdict = verdict;
        r.nt = trace_word(OBS_TO_PROXY, lxc, res, mon);
        return r;
    }
    /* delivery by the packet's destination (lookup_ip6_endpoint, :305) */
    tl_lookups++;
    const epinfo *ep = lxc_lookup(o, 2, tl_pkt6.da);
    /* LXC_NAT46: a peer outside the cluster in ::ffff:0:0/96 (:353-360) */
    static const uint8_t mapped[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};
    if (!ep && dst != CLUSTER_ID && !memcmp(tl_pkt6.da, mapped, 12))
        return nat64_egress(o, lxc, tl_pkt6.da, proto, flags, len);
    metric(o, 0, METRIC_EGRESS, len); /* to_host / local / to_stack */
    if (ep) {
        if (ep->flags & ENDPOINT_F_HOST) {   /* TRACE_TO_HOST, :373 */
            r.action = TC_ACT_REDIRECT;
            r.nt = trace_word(OBS_TO_HOST, lxc, res, mon);
            return r;
        }
        /* ipv6_local_delivery: the destination's ipv6_policy on the packet
         * as it now is */
        uint8_t psa[16], pda[16];
        memcpy(psa, tl_pkt6.sa, 16);
        memcpy(pda, tl_pkt6.da, 16);
        res_t d = lxc_ingress(o, ep, o->seclabel[lxc], 16, psa, pda, proto,
                              tl_pkt6.sport, tl_pkt6.dport, 0, flags & HF_TCP_CLOSE, len, 0,
                              METRIC_EGRESS, 1);
        d.identity = dst;
        return d;
    }
    r.action = TC_ACT_OK;
    r.nt = trace_word(OBS_TO_STACK, lxc, res, mon);   /* :390 */
    return r;
}

/* check_v6 (bpf_xdp.c:132-156) */
static int xdp_v6(cfo_t *o, const uint8_t *saddr, const uint8_t *daddr)
{
    uint32_t v;
    if (o->pf6_dyn.nlens)
        tl_lookups++;
    if (lpm_lookup(&o->pf6_dyn, saddr, &v))
        return XDP_DROP;
    uint8_t k[20];
    uint32_t pl = 128;
    memcpy(k, &pl, 4);
    memcpy(k + 4, saddr, 16);
    tl_lookups++;
    if (ht_get(&o->pf6_fix, k, &v))
        return XDP_DROP;
    tl_lookups++;
    return lxc_lookup(o, 2, daddr) ? XDP_PASS : XDP_DROP;
}

void cfo_classify_v6(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint8_t *saddr, const uint8_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint32_t *mark,
                     const uint8_t *tcpflags, int32_t *action, int32_t *verdict,
                     uint32_t *identity, uint8_t *lookups, uint8_t *ct,
                     int nthreads)
{
    hop_reserve(o, n);
    if (nthreads <= 0)
        nthreads = 1;
#pragma omp parallel for schedule(static, 4096) num_threads(nthreads)
    for (size_t i = 0; i < n; i++) {
        res_t r;
        const uint8_t *sa = saddr + 16 * i, *da = daddr + 16 * i;
        tl_lookups = 0;
        tl_ct = 0;
        tl_ct3 = 0;
        tl_tcpfl = tcpflags ? tcpflags[i] : 0;
        tl_mon[0] = tl_mon[1] = tl_mon[2] = 0;
        tl_fresh.n = 0;
        tl_nat = 0;
        tl_hop.kind = 0;
        tl_hop.has2 = 0;
        memcpy(tl_pkt6.sa, sa, 16);
        memcpy(tl_pkt6.da, da, 16);
        tl_pkt6.sport = sport[i];
        tl_pkt6.dport = dport[i];
        tl_hash = o->hash_in ? o->hash_in[i]
                             : cfo_flow_hash6(sa, da, sport[i], dport[i], proto[i]);
        if (o->pkt_out) {   /* (XDP verdicts leave the packet as it is) */
            memcpy(o->pkt_out + 9 * i, sa, 16);
            memcpy(o->pkt_out + 9 * i + 4, da, 16);
            o->pkt_out[9 * i + 8] = sport[i] | (uint32_t)dport[i] << 16;
        }
        if (mode == CFO_MODE_XDP || mode == CFO_MODE_FULL) {
            int x = xdp_v6(o, sa, da);
            if (mode == CFO_MODE_XDP || x == XDP_DROP) {
                action[i] = x;
                verdict[i] = x == XDP_PASS ? 0 : -1;
                identity[i] = 0;
                if (lookups)
                    lookups[i] = (uint8_t)tl_lookups;
                if (ct)
                    ct[i] = 0;
                if (o->notify_out)
                    o->notify_out[i] = 0;
                if (o->notify_mon)
                    o->notify_mon[i] = 0;
                o->hop[i].kind = 0;
                continue;
            }
        }
        if (mode == CFO_MODE_EGRESS)
            r = lxc_egress_v6(o, ep_lxc, sa, da, proto[i], sport[i], dport[i],
                              flags[i], len[i]);
        else
            r = netdev_ingress_v6(o, sa, da, proto[i], sport[i], dport[i],
                                  flags[i], len[i], mark ? mark[i] : 0);
        action[i] = r.action;
        verdict[i] = r.verdict;
        identity[i] = r.identity;
        if (lookups)
            lookups[i] = (uint8_t)tl_lookups;
        if (ct)
            ct[i] = tl_ct;
        if (o->notify_out) {
            const uint32_t w = notify_site(mode, ep_lxc, &r);
            /* (an event after a NAT hop: skb->len of the translated packet) */
            o->notify_out[i] = w && tl_hop.kind ? w | NT_NATLEN : w;
        }
        if (o->notify_mon)   /* both stages' monitor lengths (ct_apply) */
            o->notify_mon[i] = tl_mon[0] | tl_mon[1] << 16;
        tl_hop.ct2 = tl_hop.has2 ? tl_ct3 : 0;
        o->hop[i] = tl_hop;
        if (o->pkt_out) {
            memcpy(o->pkt_out + 9 * i, tl_pkt6.sa, 16);
            memcpy(o->pkt_out + 9 * i + 4, tl_pkt6.da, 16);
            o->pkt_out[9 * i + 8] = tl_pkt6.sport | (uint32_t)tl_pkt6.dport << 16;
        }
    }
}

void cfo_set_notify_out(cfo_t *o, uint32_t *words, uint32_t *mon)
{
    o->notify_out = words;
    o->notify_mon = mon;
}

int cfo_policy_create(cfo_t *o, uint16_t lxc_id)
{
    if (!o->pol[lxc_id]) {
        o->pol[lxc_id] = calloc(1, sizeof(pmap));
        ht_init(&o->pol[lxc_id]->idx, 8);
    }
    return 0;
}

static int cmp_rows7(const void *a, const void *b)
{
    const uint64_t *x = a, *y = b;
    for (int i = 0; i < 7; i++)
        if (x[i] != y[i])
            return x[i] < y[i] ? -1 : 1;
    return 0;
}

size_t cfo_policy_dump(cfo_t *o, uint16_t lxc_id, uint64_t *rows, size_t cap)
{
    pmap *m = o->pol[lxc_id];
    if (!m)
        return 0;
    if (rows && cap >= m->n) {
        for (uint32_t i = 0; i < m->n; i++) {
            pentry *e = &m->ents[i];
            uint32_t id;
            uint16_t dp;
            memcpy(&id, e->key, 4);
            memcpy(&dp, e->key + 4, 2);
            uint64_t *r = rows + 7 * (size_t)i;
            r[0] = id;
            r[1] = dp;
            r[2] = e->key[6];
            r[3] = e->key[7];
            r[4] = e->proxy_port;
            r[5] = e->packets;
            r[6] = e->bytes;
        }
        qsort(rows, m->n, 7 * sizeof(uint64_t), cmp_rows7);
    }
    return m->n;
}

size_t cfo_metrics_dump(cfo_t *o, uint64_t *rows, size_t cap)
{
    size_t n = 0;
    for (int r = 0; r < 256; r++)
        for (int d = 0; d < 4; d++)
            if (o->metrics[r][d][0]) {
                if (rows && n < cap) {
                    rows[4 * n] = (uint64_t)r;
                    rows[4 * n + 1] = (uint64_t)d;
                    rows[4 * n + 2] = o->metrics[r][d][0];
                    rows[4 * n + 3] = o->metrics[r][d][1];
                }
                n++;
            }
    return n;
}

size_t cfo_identity_dump(cfo_t *o, uint64_t *rows, size_t cap)
{
    size_t n = 0;
    for (uint32_t id = 0; id < ID_SLOTS; id++)
        for (uint32_t dir = 0; dir < 2; dir++) {
            const uint64_t *v = o->idc + ((size_t)dir * ID_SLOTS + id) * 4;
            if (!(v[0] | v[1] | v[2] | v[3]))
                continue;
            if (rows && n < cap) {
                uint64_t *r = rows + 6 * n;
                r[0] = id == ID_SLOTS - 1 ? 0xFFFFFFFFu : id;
                r[1] = dir + 1;
                memcpy(r + 2, v, 32);
            }
            n++;
        }
    return n;
}

void cfo_counters_reset(cfo_t *o)
{
    memset(o->idc, 0, (size_t)2 * ID_SLOTS * 4 * sizeof(uint64_t));
    memset(o->metrics, 0, sizeof(o->metrics));
    for (int i = 0; i < 65536; i++)
        if (o->pol[i])
            for (uint32_t j = 0; j < o->pol[i]->n; j++)
                o->pol[i]->ents[j].packets = o->pol[i]->ents[j].bytes = 0;
}

/* ------------------------------------------------------------ CT maps */
static void ct_put(cfo_t *o, const uint8_t k[CTK], const struct ctent *e)
{
    int64_t s = ht_find(&o->ct, k);
    uint32_t idx;
    if (s >= 0) {
        idx = o->ct.vals[s];
    } else {
        if (o->ct_n == o->ct_cap) {
            o->ct_cap = o->ct_cap ? 2 * o->ct_cap : 1024;
            o->ct_ents = realloc(o->ct_ents, o->ct_cap * sizeof(struct ctent));
            o->ct_live = realloc(o->ct_live, o->ct_cap);
        }
        idx = o->ct_n++;
        ht_put(&o->ct, k, idx);
    }
    o->ct_ents[idx] = *e;
    o->ct_live[idx] = 1;
}

int cfo_ct_add(cfo_t *o, int family, int lxc, int any_map,
               const uint8_t *tuple, const uint8_t entry[56])
{
    int alen = family == 1 ? 4 : 16;
    uint8_t k[CTK];
    uint16_t owner = 0;
    if (lxc >= 0) {
        o->ct_local[lxc & 0xFFFF] = 1;
        owner = (uint16_t)((lxc & 0xFFFF) + 1);
    }
    memset(k, 0, CTK);
    memcpy(k, &owner, 2);
    k[2] = (uint8_t)(any_map ? 1 : 0);
    k[3] = (uint8_t)family;
    memcpy(k + 4, tuple, 2 * (size_t)alen + 6);
    struct ctent e;
    memcpy(&e, entry, sizeof(e));
    ct_put(o, k, &e);
    o->ct_added++;
    return 0;
}

/* n packed synth.CT_DT records (family u8, lxc i32, any u8, tuple[38],
 * entry[56]; 100 bytes each) */
int cfo_ct_add_n(cfo_t *o, size_t n, const uint8_t *rec)
{
    for (size_t i = 0; i < n; i++) {
        const uint8_t *r = rec + 100 * i;
        int32_t lxc;
        memcpy(&lxc, r + 1, 4);
        int rc = cfo_ct_add(o, r[0], lxc, r[5], r + 6, r + 44);
        if (rc)
            return rc;
    }
    return 0;
}

/* A hit's entry update (__ct_lookup, conntrack.h:221-285) applied in header
 * order, plus CONNTRACK_ACCOUNTING (lxc_config.h:50, :247-257) for a hit
 * the batch's lookup did not see (len 0: counted in pass 1).  Returns the
 * monitor length the reference's lookup would have produced. */
static uint32_t ct_hit_update(cfo_t *o, struct ctent *e, int action, int dir,
                              int is_tcp, int syn, uint8_t flags, uint32_t len)
{
    if (len && dir == CT_INGRESS) {
        e->rx_packets++;
        e->rx_bytes += len;
    } else if (len) {
        e->tx_packets++;
        e->tx_bytes += len;
    }
    return ct_hit_entry(e, o->now, action, dir, is_tcp, syn, flags);
}

/* ct_create4 / ct_create6 (conntrack.h:615-662, :691-772): the k2 entry,
 * then — when the load balancer left ct_state->addr set (lb4_local) — the
 * entry reverse NAT needs (daddr / saddr replaced by addr; a loopback flow's
 * reply tuple with TUPLE_F_IN and svc_addr), then the ICMP entry that
 * relates errors to it, written into the same map.  ct_update_timeout runs
 * with seen_flags.syn = is_tcp — bit 0 of the union, so lower_bits stays 0
 * and a TCP entry keeps seen_non_syn clear (CT_SYN_TIMEOUT); CT_SERVICE
 * entries take the tx side like egress ones.  ipv6_policy derives
 * ct_state_new.rev_nat_index from the low 16 bits of daddr.s6_addr32[3]
 * (bpf_lxc.c:787-788), so IPv6 ingress entries carry it. */
static int ct_create_entries(const cfo_t *o, const uint8_t k2[CTK], int alen, int dir,
                             uint32_t len, uint32_t src_sec_id, const ctstate_t *st,
                             uint8_t keys[3][CTK], struct ctent ents[3])
{
    int n = 0;
    struct ctent e;
    memset(&e, 0, sizeof(e));
    e.rev_nat_index = st->rev_nat;
    e.slave = st->slave;
    if (st->loopback)
        e.bits |= CTB_LB_LOOPBACK;
    if (st->nat46)
        e.bits |= CTB_NAT46;
    const uint8_t *t = k2 + 4;
    const int is_tcp = t[2 * alen + 4] == 6;
    ct_upd_timeout(&e, o->now, is_tcp, dir, is_tcp, 0);
    if (dir == CT_INGRESS) {
        e.rx_packets = 1;
        e.rx_bytes = len;
    } else {
        e.tx_packets = 1;
        e.tx_bytes = len;
    }
    e.src_sec_id = src_sec_id;
    memcpy(keys[n], k2, CTK);
    ents[n++] = e;
    if (st->addr && alen == 4) {
        memcpy(keys[n], k2, CTK);
        uint8_t *x = keys[n] + 4;
        memcpy(dir == CT_INGRESS ? x + 4 : x, &st->addr, 4);
        if (st->loopback) {
            x[13] = TUPLE_F_IN;
            memcpy(dir == CT_INGRESS ? x : x + 4, &st->svc_addr, 4);
        }
        ents[n++] = e;
    }
    uint16_t owner;
    memcpy(&owner, k2, 2);
    ct_key(keys[n], owner, k2[2], alen, t, t + alen, 0, 0, alen == 4 ? 1 : 58,
           (uint8_t)(t[2 * alen + 5] | TUPLE_F_RELATED));
    e.bits |= CTB_SEEN_NON_SYN;   /* "For ICMP, there is no SYN" */
    ents[n++] = e;
    return n;
}

static void ct_create(cfo_t *o, const uint8_t k2[CTK], int alen, int dir,
                      uint32_t len, uint32_t src_sec_id, const ctstate_t *st)
{
    uint8_t keys[3][CTK];
    struct ctent ents[3];
    const int n = ct_create_entries(o, k2, alen, dir, len, src_sec_id, st, keys, ents);
    for (int j = 0; j < n; j++)
        ct_put(o, keys[j], &ents[j]);
}

/* The CT stage of a header's NAT hop (stage 1, the other family's maps:
 * the IPv4 egress lookup after NAT64, ipv6_policy's after NAT46), as
 * ct_apply does for a header's own stages; a NAT64 create carries nat46
 * (conntrack.h:714-716), an IPv6 ingress create its rev_nat_index
 * (bpf_lxc.c:787-788). */
static void apply_hop(cfo_t *o, int pass, size_t i, const struct hop *hp, uint8_t cs,
                      int32_t verdict, uint32_t len, int syn, uint8_t tfl, uint32_t sec,
                      uint8_t *fresh, int svc_only)
{
    (void)i;   /* fresh: this stage's "hit an entry the batch created" flag */
    const int alen = hp->alen, dir = hp->dir, is_tcp = hp->proto == 6;
    uint8_t k1[CTK], k2[CTK];
    int action;
    uint16_t td, ts;
    /* a NAT64 hop's IPv4 egress program runs its service step first
     * (lb4_local, bpf_lxc.c:476-492, on the translated packet, tl_hash as the
     * classify saw it): the hop's CT stage looks up (saddr, the service
     * step's daddr), its create carries lb4_local's ct_state, and the
     * CT_SERVICE entry is hit or created (ct_update4_slave) here too */
    lbx_t x;
    memset(&x, 0, sizeof(x));
    uint8_t tda[16];
    memcpy(tda, hp->da, 16);
    uint16_t tsp = hp->sport, tdp = hp->dport;
    int lbv = 0;
    if (hp->kind == HOP_NAT64 && dir == CT_EGRESS && alen == 4 && o->lb4_n) {
        uint32_t sa4, da4;
        memcpy(&sa4, hp->sa, 4);
        memcpy(&da4, hp->da, 4);
        tl_pkt = (pkt4_t){sa4, da4, hp->sport, hp->dport};
        lb4_egress(o, hp->owner, sa4, da4, hp->proto, syn, &x);
        lbv = x.svc && !x.drop;
        if (lbv) {
            memcpy(tda, &x.t_da, 4);
            tsp = tl_pkt.sport;
            tdp = tl_pkt.dport;
        }
        if (pass == 2 && x.svc) {
            uint8_t kk2[CTK];
            int act;
            uint16_t a_, b_;
            (void)ct_keys(4, hp->owner, hp->sa, hp->da, hp->proto, hp->sport, hp->dport, syn,
                          CT_SERVICE, x.k_svc, kk2, &act, &a_, &b_);
            const uint8_t sfl = is_tcp ? tfl : 0;
            if (x.svc_hit >= 0) {   /* __ct_lookup on the service entry */
                ct_hit_update(o, &o->ct_ents[x.svc_hit], act, CT_SERVICE, is_tcp, syn, sfl,
                              len);
                if (x.reslave && !x.drop)   /* ct_update4_slave */
                    o->ct_ents[x.svc_hit].slave = x.slave;
            } else {
                ctstate_t cs0 = {0, x.slave0, 0, 0, 0, 0};
                ct_create(o, x.k_svc, 4, CT_SERVICE, len, 0, &cs0);
                if (x.reslave && !x.drop) {
                    int64_t ne = ct_find(o, x.k_svc);
                    if (ne >= 0)
                        o->ct_ents[ne].slave = x.slave;
                }
            }
        }
    }
    if (svc_only)   /* (lb4_local found no backend: DROP_NO_SERVICE, no CT stage) */
        return;
    if (ct_keys(alen, hp->owner, hp->sa, tda, hp->proto, tsp, tdp, syn, dir,
                k1, k2, &action, &td, &ts) < 0)
        return;
    const int b = cs & 3;
    const int64_t e1 = ct_find(o, k1), e2 = ct_find(o, k2);
    const uint8_t fl = is_tcp ? tfl : 0;
    if (pass == 1) {   /* CONNTRACK_ACCOUNTING of the lookup's hit */
        const int64_t e = b >= CT_REPLY ? e1 : b == CT_ESTABLISHED ? e2 : -1;
        if (e < 0 && b != CT_NEW)
            *fresh = 1;
        if (e >= 0) {
            struct ctent *x = &o->ct_ents[e];
            if (dir == CT_INGRESS) {
                x->rx_packets++;
                x->rx_bytes += len;
            } else {
                x->tx_packets++;
                x->tx_bytes += len;
            }
        }
        return;
    }
    const uint32_t cnt = *fresh ? len : 0;
    if (b == CT_REPLY || b == CT_RELATED) {
        if (e1 >= 0)
            ct_hit_update(o, &o->ct_ents[e1], action, dir, is_tcp, syn, fl, cnt);
    } else if (b == CT_ESTABLISHED) {
        if (e2 >= 0) {
            ct_hit_update(o, &o->ct_ents[e2], action, dir, is_tcp, syn, fl, cnt);
            /* ct_delete at the stage that drops: the hop's, unless a NAT64
             * hop's local delivery follows it (the destination's) */
            if (verdict == DROP_POLICY && (!hp->has2 || hp->dir == CT_INGRESS))
                o->ct_live[e2] = 0;
        }
    } else if (cs & CTO_CREATE1) {
        if (e2 >= 0) {
            ct_hit_update(o, &o->ct_ents[e2], action, dir, is_tcp, syn, fl, len);
        } else {
            ctstate_t st = {alen == 16 && dir == CT_INGRESS
                                ? (uint16_t)(hp->da[12] | hp->da[13] << 8) : 0,
                            0, 0, 0, 0, hp->kind == HOP_NAT64 && dir == CT_EGRESS};
            if (lbv)   /* ct_state_new from lb4_local */
                st = (ctstate_t){x.rev_nat, x.slave, x.loopback, x.addr, x.svc_addr, 1};
            ct_create(o, k2, alen, dir, len, sec, &st);
        }
    }
}

/* Fold one classified batch into the CT maps, in header order, as the
 * engine does between batches: the CT result (and the monitor length) of
 * every lookup stage was taken against the maps as they were when the
 * batch started (ct[], mon[]), and the entry updates of the hits, the
 * creates (ct_create), deletes (ct_delete on a denied CT_ESTABLISHED flow)
 * and closing-bit / timeout updates are applied here, at the batch's clock.
 * A flow created twice in one batch is created once (the reference sees its
 * second packet as CT_ESTABLISHED).  hazard[i] (optional) = 1 when the
 * reference, running the batch one packet at a time, would have seen a
 * different CT result or monitor length for header i because of an earlier
 * header of the same batch — streams used for golden vectors drop those
 * headers. */
static void ct_apply(cfo_t *o, int alen, int mode, uint16_t ep_lxc, size_t n,
                     const uint8_t *saddr, const uint8_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint8_t *tcpflags,
                     const uint32_t *identity, const int32_t *verdict,
                     const uint8_t *ct, const uint32_t *mon, uint8_t *hazard)
{
    /* pass 1 counts every hit of the batch on the entry it hit (the maps as
     * committed); pass 2 applies the writes in header order.  The reference
     * interleaves the two per packet; they differ only when a write in the
     * batch (delete, or the ICMP entry a create overwrites) lands on an entry
     * another header of the same batch hits — a hazard (below). */
    uint32_t *hit_idx = hazard ? calloc(o->ct_n + 1, sizeof(uint32_t)) : NULL;
    /* per (header, stage): the lookup hit an entry the maps did not hold when
     * the batch started (one the header's own egress stage created): pass 2
     * counts it, the device did not */
    uint8_t *fresh = calloc(2 * n + 1, 1);
    uint8_t *fresh3 = calloc(n + 1, 1);   /* (a NAT64 hop's third stage) */
    for (int pass = 1; pass <= 2; pass++)
    for (size_t i = 0; i < n; i++) {
        if (hazard && pass == 1)
            hazard[i] = 0;
        const uint8_t c = ct[i];
        /* (lb4_local / lb6_local created its CT_SERVICE entry before it
         * found no backend) */
        const int no_svc = mode == CFO_MODE_EGRESS && verdict[i] == DROP_NO_SERVICE;
        if (!(c & (CTO_DONE1 | CTO_DONE2)) && !no_svc)
            continue;
        const uint8_t *sa = saddr + (size_t)alen * i;
        const uint8_t *da = daddr + (size_t)alen * i;
        const int last = (c & CTO_DONE2) ? 1 : 0;
        const int is_tcp = proto[i] == 6;
        const int syn = (flags[i] & HF_TCP_CLOSE) != 0;
        const uint8_t fl = is_tcp && tcpflags ? tcpflags[i] : 0;
        /* IPv4 egress: the service step again, on the maps as they now are
         * (its CT_SERVICE entry: created, or hit and updated), and the tuple
         * and packet it leaves for the stages */
        lbx_t x;
        lbx6_t x6;
        int lbv = 0;
        uint32_t tda4 = 0, psa4 = 0, pda4 = 0;
        uint8_t tda6[16], psa6[16], pda6[16];
        uint16_t psp = sport[i], pdp = dport[i];
        if (alen == 4) {
            memcpy(&tl_pkt.sa, sa, 4);
            memcpy(&tl_pkt.da, da, 4);
            tl_pkt.sport = sport[i];
            tl_pkt.dport = dport[i];
            tl_hash = o->hash_in ? o->hash_in[i]
                                 : cfo_flow_hash4(tl_pkt.sa, tl_pkt.da, sport[i],
                                                  dport[i], proto[i]);
            tda4 = tl_pkt.da;
            if (mode == CFO_MODE_EGRESS && ((c & CTO_DONE1) || no_svc)) {
                lb4_egress(o, ct_owner(o, ep_lxc), tl_pkt.sa, tl_pkt.da, proto[i],
                           syn, &x);
                lbv = x.svc;
                tda4 = x.t_da;
                if (pass == 2 && lbv) {
                    uint8_t kk2[CTK];
                    int act;
                    uint16_t a_, b_;
                    (void)ct_keys(4, ct_owner(o, ep_lxc), sa, da, proto[i], sport[i],
                                  dport[i], syn, CT_SERVICE, x.k_svc, kk2, &act, &a_, &b_);
                    if (x.svc_hit >= 0) {   /* __ct_lookup on the service entry */
                        ct_hit_update(o, &o->ct_ents[x.svc_hit], act, CT_SERVICE, is_tcp,
                                      syn, fl, len[i]);
                        if (x.reslave)    /* ct_update4_slave */
                            o->ct_ents[x.svc_hit].slave = x.slave;
                    } else {
                        ctstate_t cs = {0, x.slave0, 0, 0, 0, 0};
                        ct_create(o, x.k_svc, 4, CT_SERVICE, len[i], 0, &cs);
                        if (x.reslave) {
                            int64_t ne = ct_find(o, x.k_svc);
                            if (ne >= 0)
                                o->ct_ents[ne].slave = x.slave;
                        }
                    }
                }
            }
            psa4 = tl_pkt.sa;
            pda4 = tl_pkt.da;
            psp = tl_pkt.sport;
            pdp = tl_pkt.dport;
        } else {
            /* IPv6 egress: the same for lb6_local (no loopback, no
             * reverse-NAT entry) */
            memcpy(tl_pkt6.sa, sa, 16);
            memcpy(tl_pkt6.da, da, 16);
            tl_pkt6.sport = sport[i];
            tl_pkt6.dport = dport[i];
            tl_hash = o->hash_in ? o->hash_in[i]
                                 : cfo_flow_hash6(sa, da, sport[i], dport[i], proto[i]);
            memcpy(tda6, da, 16);
            if (mode == CFO_MODE_EGRESS && ((c & CTO_DONE1) || no_svc)) {
                lb6_egress(o, ct_owner(o, ep_lxc), sa, da, proto[i], syn, &x6);
                lbv = x6.svc;
                memcpy(tda6, x6.t_da, 16);
                if (pass == 2 && lbv) {
                    uint8_t kk2[CTK];
                    int act;
                    uint16_t a_, b_;
                    (void)ct_keys(16, ct_owner(o, ep_lxc), sa, da, proto[i], sport[i],
                                  dport[i], syn, CT_SERVICE, x6.k_svc, kk2, &act, &a_, &b_);
                    if (x6.svc_hit >= 0) {
                        ct_hit_update(o, &o->ct_ents[x6.svc_hit], act, CT_SERVICE, is_tcp,
                                      syn, fl, len[i]);
                        if (x6.reslave)   /* ct_update6_slave */
                            o->ct_ents[x6.svc_hit].slave = x6.slave;
                    } else {
                        ctstate_t cs = {0, x6.slave0, 0, 0, 0, 0};
                        ct_create(o, x6.k_svc, 16, CT_SERVICE, len[i], 0, &cs);
                        if (x6.reslave) {
                            int64_t ne = ct_find(o, x6.k_svc);
                            if (ne >= 0)
                                o->ct_ents[ne].slave = x6.slave;
                        }
                    }
                }
            }
            memcpy(psa6, tl_pkt6.sa, 16);
            memcpy(pda6, tl_pkt6.da, 16);
            psp = tl_pkt6.sport;
            pdp = tl_pkt6.dport;
        }
        const epinfo *dst = lxc_lookup(o, alen == 4 ? 1 : 2,
                                       alen == 4 ? (const uint8_t *)&pda4 : pda6);
        for (int s = 0; s < 2; s++) {
            if (s == 1)   /* (a reverse NAT may have moved it) */
                dst = lxc_lookup(o, alen == 4 ? 1 : 2,
                                 alen == 4 ? (const uint8_t *)&pda4 : pda6);
            const uint8_t cs = (uint8_t)(c >> (4 * s));
            if (s == 1 && !(cs & CTO_DONE1) && verdict[i] == DROP_NO_SERVICE && o->hop &&
                i < o->hop_cap && o->hop[i].kind == HOP_NAT64) {
                /* a NAT64 hop whose service step found no backend: its
                 * CT_SERVICE entry was created (or hit) before the drop */
                const struct hop *hp = &o->hop[i];
                apply_hop(o, pass, i, hp, cs, verdict[i],
                          (uint32_t)((int32_t)len[i] + hp->dlen),
                          (flags[i] & HF_TCP_CLOSE) != 0, fl, 0, fresh + 2 * i + 1, 1);
                continue;
            }
            if (!(cs & CTO_DONE1))
                continue;
            if (s == 1 && o->hop && i < o->hop_cap && o->hop[i].kind == HOP_NAT46 &&
                o->hop[i].has2 == 2) {
                /* NAT46 behind an egress batch's local delivery: the hop's
                 * IPv6 stage is a third one (its keys are IPv6, the
                 * destination's ipv4_policy stage below IPv4, so their order
                 * within the header does not matter) */
                const struct hop *hp = &o->hop[i];
                if (hp->ct2 & CTO_DONE1)
                    apply_hop(o, pass, i, hp, hp->ct2, verdict[i],
                              (uint32_t)((int32_t)len[i] + hp->dlen),
                              (flags[i] & HF_TCP_CLOSE) != 0, fl, o->seclabel[ep_lxc],
                              fresh3 + i, 0);
            } else if (s == 1 && o->hop && i < o->hop_cap && o->hop[i].kind) {
                const struct hop *hp = &o->hop[i];
                const uint32_t hl = (uint32_t)((int32_t)len[i] + hp->dlen);
                const uint32_t sec = mode == CFO_MODE_EGRESS ? o->seclabel[ep_lxc] : identity[i];
                apply_hop(o, pass, i, hp, cs, verdict[i], hl, (flags[i] & HF_TCP_CLOSE) != 0,
                          fl, sec, fresh + 2 * i + 1, 0);
                if (hp->has2 && (hp->ct2 & CTO_DONE1)) {
                    /* a NAT64 hop's local delivery: the destination's
                     * ipv4_policy lookup, after the hop's egress stage */
                    struct hop h2 = *hp;
                    h2.dir = CT_INGRESS;
                    h2.owner = hp->owner2;
                    h2.sport = hp->sport2;
                    h2.dport = hp->dport2;
                    memcpy(h2.sa, hp->sa2, 4);
                    memcpy(h2.da, hp->da2, 4);
                    apply_hop(o, pass, i, &h2, hp->ct2, verdict[i], hl,
                              (flags[i] & HF_TCP_CLOSE) != 0, fl, sec, fresh3 + i, 0);
                }
                continue;
            }
            const int egress_stage = mode == CFO_MODE_EGRESS && s == 0;
            const int dir = egress_stage ? CT_EGRESS : CT_INGRESS;
            const uint16_t owner = egress_stage ? ct_owner(o, ep_lxc)
                                   : dst ? ct_owner(o, dst->lxc_id) : 0;
            const uint32_t sec = mode == CFO_MODE_EGRESS ? o->seclabel[ep_lxc]
                                                         : identity[i];
            uint8_t k1[CTK], k2[CTK];
            int action;
            uint16_t td, ts;
            /* IPv4: stage 0 of an egress batch looks up (saddr, the service
             * step's daddr); every other stage the packet as it now is */
            const uint8_t *ksa = sa, *kda = da;
            uint16_t ksp = sport[i], kdp = dport[i];
            if (alen == 4) {
                ksa = egress_stage ? sa : (const uint8_t *)&psa4;
                kda = egress_stage ? (const uint8_t *)&tda4 : (const uint8_t *)&pda4;
                ksp = egress_stage ? tl_pkt.sport : psp;
                kdp = egress_stage ? tl_pkt.dport : pdp;
            } else {
                ksa = egress_stage ? sa : psa6;
                kda = egress_stage ? tda6 : pda6;
                ksp = egress_stage ? tl_pkt6.sport : psp;
                kdp = egress_stage ? tl_pkt6.dport : pdp;
            }
            if (ct_keys(alen, owner, ksa, kda, proto[i], ksp, kdp,
                        syn, dir, k1, k2, &action, &td, &ts) < 0)
                continue;
            const int b = cs & 3;
            const int64_t e1 = ct_find(o, k1), e2 = ct_find(o, k2);
            /* an egress reply's reverse NAT (bpf_lxc.c:565-576) moves the
             * packet the destination's stage sees */
            if (alen == 4 && egress_stage && b >= CT_REPLY && e1 >= 0 &&
                o->ct_ents[e1].rev_nat_index) {
                lb4_rev_nat(o, &o->ct_ents[e1], proto[i]);
                psa4 = tl_pkt.sa;
                pda4 = tl_pkt.da;
                psp = tl_pkt.sport;
                pdp = tl_pkt.dport;
            }
            if (alen == 16 && egress_stage && b >= CT_REPLY && e1 >= 0 &&
                o->ct_ents[e1].rev_nat_index) {
                lb6_rev_nat(o, o->ct_ents[e1].rev_nat_index, proto[i]);
                memcpy(psa6, tl_pkt6.sa, 16);
                psp = tl_pkt6.sport;
            }
            if (pass == 1) {   /* CONNTRACK_ACCOUNTING of the lookup hits */
                const int64_t e = b >= CT_REPLY ? e1 : b == CT_ESTABLISHED ? e2 : -1;
                if (e < 0 && b != CT_NEW)
                    fresh[2 * i + s] = 1;
                if (e >= 0) {
                    struct ctent *x = &o->ct_ents[e];
                    if (dir == CT_INGRESS) {
                        x->rx_packets++;
                        x->rx_bytes += len[i];
                    } else {
                        x->tx_packets++;
                        x->tx_bytes += len[i];
                    }
                    if (hit_idx)
                        hit_idx[e] = (uint32_t)i + 1;   /* last hitting header */
                }
                continue;
            }
            const int created = (cs & CTO_CREATE1) != 0;
            const int dropped = s == last && verdict[i] == DROP_POLICY;
            const int rel = (k1[4 + 2 * alen + 5] & TUPLE_F_RELATED) != 0;
            const int q = e1 >= 0 ? (rel ? CT_RELATED : CT_REPLY)
                          : e2 >= 0 ? CT_ESTABLISHED : CT_NEW;
            /* (a flow created earlier in the batch: the reference's second
             * packet is CT_ESTABLISHED, the batch's CT_NEW — the same
             * verdict and entry, but ipv6_policy reverse-NATs an IPv6 hit
             * whose entry's rev_nat_index cilium_lb6_reverse_nat holds,
             * bpf_lxc.c:808-815, so there the packets differ) */
            const int rn6 = alen == 16 && dir == CT_INGRESS && e2 >= 0 &&
                            o->rnat6_ok[o->ct_ents[e2].rev_nat_index];
            if (hazard && q != b && !(b == CT_NEW && q == CT_ESTABLISHED && created && !rn6))
                hazard[i] = 1;
            /* the monitor length a packet-at-a-time lookup would return */
            uint32_t m = TRACE_PAYLOAD_LEN;
            const uint32_t cnt = fresh[2 * i + s] ? len[i] : 0;
            if (b == CT_REPLY || b == CT_RELATED) {
                if (e1 >= 0)
                    m = ct_hit_update(o, &o->ct_ents[e1], action, dir, is_tcp, syn, fl, cnt);
            } else if (b == CT_ESTABLISHED) {
                if (e2 >= 0) {
                    m = ct_hit_update(o, &o->ct_ents[e2], action, dir, is_tcp, syn, fl, cnt);
                    if (dropped) {
                        if (hit_idx && hit_idx[e2] > i + 1)
                            hazard[hit_idx[e2] - 1] = 1;  /* hit after delete */
                        o->ct_live[e2] = 0;
                    }
                }
            } else if (created) {
                if (e2 >= 0) {
                    m = ct_hit_update(o, &o->ct_ents[e2], action, dir, is_tcp, syn, fl,
                                      len[i]);
                } else {
                    if (hit_idx) {   /* the ICMP entry it overwrites */
                        uint8_t ki[CTK];
                        uint16_t ow;
                        memcpy(&ow, k2, 2);
                        ct_key(ki, ow, k2[2], alen, k2 + 4, k2 + 4 + alen, 0, 0,
                               alen == 4 ? 1 : 58,
                               (uint8_t)(k2[4 + 2 * alen + 5] | TUPLE_F_RELATED));
                        int64_t ei = ct_find(o, ki);
                        if (ei >= 0 && (size_t)ei < o->ct_n && hit_idx[ei])
                            hazard[i] = 1;
                    }
                    ctstate_t cs = {alen == 16 && dir == CT_INGRESS
                                        ? (uint16_t)(kda[12] | kda[13] << 8) : 0,
                                    0, 0, 0, 0, 0};
                    if (egress_stage && lbv && alen == 4)   /* ct_state_new from lb4_local */
                        cs = (ctstate_t){x.rev_nat, x.slave, x.loopback, x.addr,
                                         x.svc_addr, 0};
                    if (egress_stage && lbv && alen == 16)  /* ... from lb6_local */
                        cs = (ctstate_t){x6.rev_nat, x6.slave, 0, 0, 0, 0};
                    ct_create(o, k2, alen, dir, len[i], sec, &cs);
                }
            }
            const uint16_t pdport = q >= CT_REPLY ? td : ts;
            if (pdport == 0x3500)
                m = MTU;
            if (hazard && mon && m != ((mon[i] >> (16 * s)) & 0xFFFF))
                hazard[i] = 1;
        }
    }
    free(hit_idx);
    free(fresh);
    free(fresh3);
}

void cfo_ct_apply_v4(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint32_t *saddr, const uint32_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint8_t *tcpflags,
                     const uint32_t *identity, const int32_t *verdict,
                     const uint8_t *ct, const uint32_t *mon, uint8_t *hazard)
{
    ct_apply(o, 4, mode, ep_lxc, n, (const uint8_t *)saddr,
             (const uint8_t *)daddr, sport, dport, proto, flags, len, tcpflags,
             identity, verdict, ct, mon, hazard);
}

void cfo_ct_apply_v6(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint8_t *saddr, const uint8_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint8_t *tcpflags,
                     const uint32_t *identity, const int32_t *verdict,
                     const uint8_t *ct, const uint32_t *mon, uint8_t *hazard)
{
    ct_apply(o, 16, mode, ep_lxc, n, saddr, daddr, sport, dport, proto, flags,
             len, tcpflags, identity, verdict, ct, mon, hazard);
}

static int cmp_ctrow(const void *a, const void *b)
{
    return memcmp(a, b, CTK);
}

/* an address in a GCFilter IP set: records of 17 bytes {family 1|2,
 * address[16]} (IPv4: the first 4 bytes) */
static int gc_ip_in(const uint8_t *set, size_t n, int fam, const uint8_t *a)
{
    const size_t al = fam == 1 ? 4 : 16;
    for (size_t i = 0; i < n; i++)
        if (set[17 * i] == fam && !memcmp(set + 17 * i + 1, a, al))
            return 1;
    return 0;
}

/* ctmap.GC (pkg/maps/ctmap/ctmap.go:339-350) on the maps selected by
 * family (0 any, 1, 2), owner (-1 any, 0 global, lxc_id + 1) and kind
 * (-1 any, 0 TCP, 1 ANY): doFiltering (:303-325) on every live entry —
 * RemoveExpired: lifetime < time; ValidIPs (n_valid != SIZE_MAX): neither
 * tuple address in the set; MatchIPs (n_match != SIZE_MAX): either is.
 * Returns the entries deleted. */
size_t cfo_ct_gc(cfo_t *o, int family, int owner, int kind, int remove_expired,
                 uint32_t time, const uint8_t *valid, size_t n_valid,
                 const uint8_t *match, size_t n_match)
{
    size_t del = 0;
    for (uint32_t s = 0; s < o->ct.cap; s++) {
        if (!o->ct.used[s])
            continue;
        const uint32_t idx = o->ct.vals[s];
        if (!o->ct_live[idx])
            continue;
        const uint8_t *k = o->ct.keys + (size_t)s * CTK;
        uint16_t ow;
        memcpy(&ow, k, 2);
        if ((family && k[3] != family) || (owner >= 0 && ow != owner) ||
            (kind >= 0 && k[2] != kind))
            continue;
        const int fam = k[3], al = fam == 1 ? 4 : 16;
        const uint8_t *da = k + 4, *sa = k + 4 + al;
        int d = remove_expired && o->ct_ents[idx].lifetime < time;
        if (!d && n_valid != (size_t)-1)
            d = !gc_ip_in(valid, n_valid, fam, da) && !gc_ip_in(valid, n_valid, fam, sa);
        if (!d && n_match != (size_t)-1)
            d = gc_ip_in(match, n_match, fam, da) || gc_ip_in(match, n_match, fam, sa);
        if (d) {
            o->ct_live[idx] = 0;
            del++;
        }
    }
    return del;
}

size_t cfo_ct_dump(cfo_t *o, uint8_t *rows, size_t cap)
{
    size_t n = 0;
    for (uint32_t s = 0; s < o->ct.cap; s++) {
        if (!o->ct.used[s])
            continue;
        uint32_t idx = o->ct.vals[s];
        if (!o->ct_live[idx])
            continue;
        if (rows && n < cap) {
            uint8_t *r = rows + CFO_CT_ROW * n;
            memset(r, 0, CFO_CT_ROW);
            memcpy(r, o->ct.keys + (size_t)s * CTK, CTK);
            memcpy(r + CTK, &o->ct_ents[idx], sizeof(struct ctent));
        }
        n++;
    }
    if (rows && n <= cap)
        qsort(rows, n, CFO_CT_ROW, cmp_ctrow);
    return n;
}

/* The reference's own semantics, in C (TEST INFRASTRUCTURE): the headers one
 * at a time, each classified against the CT maps as the headers before it
 * left them and folded into them before the next — what the kernel does
 * packet by packet (conntrack.h:221-285 lookups, :615-772 creates, the
 * ct_delete of a denied established flow), at bpf_ktime_get_sec() = clock[i]
 * (clock NULL: the clock as set).  Outputs as cfo_classify_* (+ the CT byte
 * and the monitor event site word of every header). */
void cfo_run_seq(cfo_t *o, int family, int mode, uint16_t ep_lxc, size_t n,
                 const uint8_t *saddr, const uint8_t *daddr, const uint16_t *sport,
                 const uint16_t *dport, const uint8_t *proto, const uint8_t *flags,
                 const uint16_t *len, const uint32_t *mark, const uint8_t *tcpflags,
                 const uint32_t *clock, int32_t *action, int32_t *verdict,
                 uint32_t *identity, uint8_t *ct, uint32_t *words)
{
    const size_t al = family == 4 ? 4 : 16, pw = family == 4 ? 3 : 9;
    const uint32_t *hash0 = o->hash_in;
    uint32_t *pkt0 = o->pkt_out;
    uint32_t *nt0 = o->notify_out, *mon0 = o->notify_mon;
    uint32_t mon1 = 0;
    for (size_t i = 0; i < n; i++) {
        if (clock)
            o->now = clock[i];
        o->hash_in = hash0 ? hash0 + i : NULL;
        o->pkt_out = pkt0 ? pkt0 + pw * i : NULL;
        o->notify_out = words ? words + i : NULL;
        o->notify_mon = &mon1;
        uint8_t c = 0;
        const uint8_t *sa = saddr + al * i, *da = daddr + al * i;
        if (family == 4)
            cfo_classify_v4(o, mode, ep_lxc, 1, (const uint32_t *)sa, (const uint32_t *)da,
                            sport + i, dport + i, proto + i, flags + i, len + i,
                            mark ? mark + i : NULL, tcpflags ? tcpflags + i : NULL,
                            action + i, verdict + i, identity + i, NULL, &c, 1);
        else
            cfo_classify_v6(o, mode, ep_lxc, 1, sa, da, sport + i, dport + i, proto + i,
                            flags + i, len + i, mark ? mark + i : NULL,
                            tcpflags ? tcpflags + i : NULL, action + i, verdict + i,
                            identity + i, NULL, &c, 1);
        o->pkt_out = NULL;
        o->notify_out = NULL;
        o->notify_mon = NULL;
        ct_apply(o, (int)al, mode, ep_lxc, 1, sa, da, sport + i, dport + i, proto + i,
                 flags + i, len + i, tcpflags ? tcpflags + i : NULL,
                 (const uint32_t *)identity + i, verdict + i, &c, NULL, NULL);
        if (ct)
            ct[i] = c;
    }
    o->hash_in = hash0;
    o->pkt_out = pkt0;
    o->notify_out = nt0;
    o->notify_mon = mon0;
}
