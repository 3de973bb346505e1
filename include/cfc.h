/*
 * cfc.h — C ABI of the MI355X flow-classification engine (libcfc.so).
 *
 * This is the drop-in boundary for Cilium's datapath verdict path.  The
 * map-population half mirrors pkg/bpf's fd-based BPF map API one call for
 * one call, with the reference's key/value byte layouts, so pkg/maps/
 * {policymap,ipcache,lxcmap,cidrmap,metricsmap} and pkg/policy/prefilter.go
 * work unchanged on top of a thin cgo shim.  The datapath
 * half replaces the per-packet BPF programs (bpf_xdp.c, bpf_netdev.c,
 * bpf_lxc.c) by one batched call over SoA header arrays resident in HBM.
 *
 * Conventions
 *  - every function returns 0 or a negative errno (-ENOENT, -EEXIST,
 *    -E2BIG, -ENOSPC, -EINVAL, -ENOMEM, -EBADF, -ENODEV); nothing aborts.
 *  - key/value buffers are caller-owned and copied (pkg/bpf/bpf.go:153-252).
 *  - all mutators and cfc_classify are thread-safe; a table change becomes
 *    visible to the next cfc_classify (auto-commit) or at cfc_commit().
 *    Work already queued on a stream keeps reading the previous epoch.
 *  - addresses/ports are raw network-order bytes loaded little-endian
 *    ("be32"/"be16" raw), identities are host-order u32.
 */
#ifndef CFC_H
#define CFC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CFC_ABI_VERSION 13

typedef struct cfc_ctx cfc_ctx;

/* ------------------------------------------------------------------ context */
/* One context per GPU (device ordinal).  Tables are replicated per context.
 * device = CFC_DEVICE_NONE opens a host-only context: the map API works
 * (control-plane tooling, tests without a GPU); cfc_commit, cfc_classify_*
 * and the counter calls return -ENODEV.  There is no CPU datapath. */
#define CFC_DEVICE_NONE (-1)
int cfc_open(int device, cfc_ctx **out);
void cfc_close(cfc_ctx *ctx);
int cfc_abi_version(void);

/* ------------------------------------------------------------- BPF map API */
/* Map types use the kernel's numbering (pkg/bpf/bpf.go:39-59). */
#define CFC_MAP_TYPE_HASH 1
#define CFC_MAP_TYPE_PERCPU_HASH 5
#define CFC_MAP_TYPE_LRU_HASH 9
#define CFC_MAP_TYPE_LPM_TRIE 11

/* Update flags (pkg/bpf/bpf.go BPF_ANY/BPF_NOEXIST/BPF_EXIST). */
#define CFC_ANY 0
#define CFC_NOEXIST 1
#define CFC_EXIST 2

/*
 * Replaces bpf.OpenOrCreateMap(path, mapType, keySize, valueSize,
 * maxEntries, flags) (pkg/bpf/bpf.go:371) and bpf.CreateMap (:108).
 * The basename of `path` selects the datapath role, as the pin path does in
 * the reference:
 *   cilium_ipcache          LPM_TRIE key 24 (struct ipcache_key) value 8
 *   cilium_lxc              HASH key 20 (struct endpoint_key) value 48
 *   cilium_policy_<id>      HASH key 8 (struct policy_key) value 24; the
 *                           policy of endpoint LXC_ID <id> (decimal)
 *   cilium_metrics          PERCPU_HASH key 8 value 16 (one "CPU": the GPU)
 *   cilium_cidr_v4_fix|v4_dyn|v6_fix|v6_dyn   prefilter (pkg/maps/cidrmap)
 *                           HASH or LPM_TRIE, key 4+addr bytes, value 1
 *   cilium_lb4_services     HASH key 8 (struct lb4_key {address, dport,
 *                           slave}) value 12 (struct lb4_service {target,
 *                           port, count, rev_nat_index, weight}); the
 *                           master slot (slave 0) carries count, slots
 *                           1..count the backends (pkg/maps/lbmap)
 *   cilium_lb4_reverse_nat  HASH key 2 (rev_nat_index) value 6 (struct
 *                           lb4_reverse_nat {address, port})
 * Any other name is a plain map with no datapath role.  Opening an existing
 * path with the same geometry returns a new handle to it (*created = 0);
 * a geometry mismatch returns -EINVAL (pkg/bpf/bpf.go:306 objCheck).
 */
int cfc_map_open(cfc_ctx *ctx, const char *path, uint32_t map_type,
                 uint32_t key_size, uint32_t value_size,
                 uint32_t max_entries, uint32_t flags, int *fd,
                 int *created);
/* bpf.ObjClose (pkg/bpf/bpf.go:299).  The map itself persists (pinned). */
int cfc_map_close(cfc_ctx *ctx, int fd);
/* bpf.UpdateElement (pkg/bpf/bpf.go:153) */
int cfc_map_update(cfc_ctx *ctx, int fd, const void *key, const void *value,
                   uint64_t flags);
/* BPF_MAP_UPDATE_BATCH: `count` packed keys and values, applied in order;
 * stops at the first error and returns it (bulk loads, e.g. a restored
 * conntrack table). */
int cfc_map_update_batch(cfc_ctx *ctx, int fd, const void *keys,
                         const void *values, uint64_t count, uint64_t flags);
/* bpf.LookupElement (pkg/bpf/bpf.go:177).  LPM maps do longest-prefix
 * match like the kernel trie.  Policy-map values carry the packet/byte
 * counters as of the last cfc_counters_sync(). */
int cfc_map_lookup(cfc_ctx *ctx, int fd, const void *key, void *value);
/* bpf.DeleteElement (pkg/bpf/bpf.go:214) */
int cfc_map_delete(cfc_ctx *ctx, int fd, const void *key);
/* bpf.GetNextKey (pkg/bpf/bpf.go:225); key == NULL (or absent) -> first. */
int cfc_map_get_next_key(cfc_ctx *ctx, int fd, const void *key,
                         void *next_key);
/* BPF_MAP_LOOKUP_BATCH over the whole map (what DumpWithCallback,
 * pkg/bpf/map.go:479, does one GetNextKey/Lookup pair at a time, and what
 * ctmap GC walks, ctmap.go:272): keys[0 .. min(*n, cap)) and their values
 * (value_size bytes, per-CPU maps rounded as cfc_map_lookup), in iteration
 * order; *n = the number of entries. */
int cfc_map_dump(cfc_ctx *ctx, int fd, void *keys, void *values, uint64_t cap,
                 uint64_t *n);
/* Number of per-CPU value slots of PERCPU maps (always 1). */
int cfc_num_possible_cpus(void);

/* Per-endpoint datapath constants that the reference compiles into each
 * endpoint program from lxc_config.h (written by pkg/endpoint/bpf.go:86-190):
 * SECLABEL, the endpoint's security identity used as the source identity
 * of its egress traffic. */
int cfc_endpoint_config(cfc_ctx *ctx, uint16_t lxc_id, uint32_t seclabel);

/* Per-node datapath constants the agent writes into node_config.h
 * (daemon/daemon.go:916-934 writeNetdevHeader / compileBase):
 *   ipv4_cluster_range / ipv4_cluster_mask  IPV4_CLUSTER_RANGE / _MASK, as
 *       the %#x of byteorder.HostSliceToNetwork(...) — i.e. the raw
 *       network-order address bytes loaded little-endian, the form
 *       handle_ipv4_from_lxc compares orig_dip against (bpf_lxc.c:523);
 *   router_ip6  ROUTER_IP, the node's IPv6 router address (the /64 that
 *       makes an egress destination CLUSTER_ID, bpf_lxc.c:214, and the
 *       echo-request target icmp6_handle answers, icmp6.h:390-412).
 * A new context starts with the values of the reference's
 * bpf/node_config.h (0x100000 / 0xff0000, beef::1:0:1:0:0).  Takes effect
 * for every classify call made after it returns. */
typedef struct {
    uint32_t ipv4_cluster_range;
    uint32_t ipv4_cluster_mask;
    uint8_t router_ip6[16];
    uint32_t host_ifindex;    /* HOST_IFINDEX (trace records of proxy and
                                 host deliveries); node_config.h: 1 */
} cfc_node_config;
int cfc_set_node_config(cfc_ctx *ctx, const cfc_node_config *cfg);
int cfc_get_node_config(cfc_ctx *ctx, cfc_node_config *cfg);

/* The datapath clock, bpf_ktime_get_sec(): seconds of CLOCK_MONOTONIC (or
 * any clock the agent's CT garbage collector reads the same way,
 * pkg/maps/ctmap/ctmap.go:272).  It stamps the CT entries' lifetimes and
 * report times and decides which packets of an active flow are traced
 * (conntrack.h:125-205, CT_REPORT_INTERVAL 5 s) for every classify and
 * CT-apply call made after it returns.  A new context starts at 0. */
int cfc_set_clock(cfc_ctx *ctx, uint32_t now_sec);

/* Publish the maps' changes to the device (the first classify after a
 * change commits by itself).  The device tables form five groups —
 * ipcache IPv4, ipcache IPv6, prefilter, endpoints + policymaps, conntrack —
 * and a commit re-flattens only the groups whose maps changed.  A value
 * overwritten in place (an existing IPv6 ipcache prefix's identity, an
 * existing policy entry's proxy port) is patched into the live tables
 * instead, as a BPF map update is visible to the next packet.  The new
 * tables are uploaded on `stream` (hipStream_t, NULL = default stream);
 * launches already queued on other streams keep the tables they were
 * launched with, which stay allocated until those streams pass the commit
 * (no device-wide drain). */
int cfc_commit(cfc_ctx *ctx, void *stream);

/* ----------------------------------------------------------------- options */
/* CFC_OPT_LPM4: device layout of the IPv4 ipcache, applied at the next
 * commit.  AUTO (default) and TRIE use the compact multibit layout — a /16
 * directory, 8-bit chunks and short per-node prefix lists, a few MiB and
 * L2-resident; DIR-24-8 is the classic 64 MiB table (Infinity-Cache
 * resident), also used when the compact layout's offsets would overflow.
 * Lookups give the same result in every layout.
 * CFC_OPT_TIMING: 1 = record HIP events around the kernels of every
 * cfc_classify_* call (read back with cfc_timing_collect).
 * CFC_OPT_CT_APPLY: where cfc_ct_apply_v4 runs: DEVICE (default) applies the
 * batch's CT writes to the device CT table in place and keeps the host's
 * view of the CT maps lazily (synchronised when a CT map is next read or
 * written through this API, or at cfc_counters_sync); HOST walks the batch
 * on the host.  Both give the same maps.
 * CFC_OPT_CT_EVICT: 1 (default) = a batch whose creates would take an IPv4
 * CT map past its max_entries stays on the device: the map's entries
 * closest to expiry that the batch's lookups did not hit are deleted first
 * (as a GC would; the reference's LRU hash evicts its least recently used
 * entries instead, in an order the kernel's per-CPU lists decide); 0 = such
 * a batch takes the host walk, whose maps evict in LRU order. */
#define CFC_OPT_LPM4 1
#define CFC_LPM4_AUTO 0
#define CFC_LPM4_DIR24_8 1
#define CFC_LPM4_TRIE 2
#define CFC_OPT_TIMING 2
#define CFC_OPT_CT_APPLY 3
#define CFC_CT_APPLY_DEVICE 0
#define CFC_CT_APPLY_HOST 1
#define CFC_OPT_CT_EVICT 4
int cfc_set_option(cfc_ctx *ctx, int option, int64_t value);

/* ---------------------------------------------------------------- datapath */
/* Which reference program chain a batch runs through. */
#define CFC_MODE_INGRESS 0 /* bpf_netdev from-netdev (FROM_HOST) -> local
                              delivery -> bpf_lxc ipv4_policy */
#define CFC_MODE_EGRESS 1  /* bpf_lxc from-container of endpoint ep_lxc */
#define CFC_MODE_XDP 2     /* bpf_xdp prefilter only */
#define CFC_MODE_FULL 3    /* XDP prefilter, then INGRESS for XDP_PASS */

/* header meta word bits (cfc_hdr_v4.meta) */
#define CFC_HF_FRAG 0x100u      /* ipv4_is_fragment() (ipv4.h:50-61) */
#define CFC_HF_TCP_CLOSE 0x200u /* what ct_lookup reads as RST|FIN
                                   (conntrack.h:533): union tcp_flags keeps
                                   each bitfield as its own union member, so
                                   all of them are bit 0 of TCP byte 12 */

/* Device-resident SoA batch of IPv4 headers; all pointers are device
 * pointers with n elements.  `ports` is the first 32-bit word of the L4
 * header exactly as ct_lookup4 loads it (sport be16 in bits 0-15, dport be16
 * in bits 16-31; for ICMP: type | code << 8 | csum << 16).  `meta` packs
 * proto (bits 0-7), CFC_HF_* flags (bits 8-15) and skb->len (bits 16-31):
 * the batch format carries packets of at most 65535 bytes; a larger (GSO)
 * skb cannot be expressed and must be classified on the slow path.
 * `mark` (skb->mark, FROM_HOST identity) may be NULL = 0.  `tcp_flags`
 * (may be NULL = 0) is TCP header byte 13 of each header (FIN SYN RST PSH
 * ACK ...): ct_lookup accumulates it into the CT entry's seen flags and
 * traces a packet whose flags the flow had not seen (conntrack.h:137-185);
 * the close bit in meta is byte 12's bit 0, which union tcp_flags reads as
 * rst/fin/syn alike. */
typedef struct {
    const uint32_t *saddr;
    const uint32_t *daddr;
    const uint32_t *ports;
    const uint32_t *meta;
    const uint32_t *mark;
    const uint8_t *tcp_flags;   /* may be NULL = 0 */
    uint64_t n;
    /* skb->hash of each header (the kernel's flow hash, what
     * lb4_select_slave reduces modulo a service's backend count, lb.h:158-190,
     * and what the monitor records carry).  NULL = CFC_FLOW_HASH (below). */
    const uint32_t *hash;
} cfc_hdr_v4;
/* The engine's stand-in for skb->hash when a batch carries none: symmetric
 * in the 5-tuple, h = fmix32(min(sa,da) * 0x9E3779B1 + max(sa,da) *
 * 0x85EBCA77 + (min(sp,dp) | max(sp,dp) << 16) * 0xC2B2AE3D + proto) over
 * the header as it arrived (fmix32: murmur3's finalizer). */

/* Device-resident SoA batch of IPv6 headers.  saddr/daddr: n addresses of
 * 16 network-order bytes each (16-byte aligned).  ports, meta and mark as in
 * cfc_hdr_v4, where meta's proto is the next header ipv6_hdrlen() stops at
 * (ipv6.h:61-98; 44 FRAGMENT and 59 NONE end in drops) and CFC_HF_EXTHDR
 * says extension headers precede it; CFC_HF_FRAG is ignored (ipv6_policy
 * passes is_fragment = false). */
#define CFC_HF_EXTHDR 0x400u
typedef struct {
    const uint8_t *saddr;
    const uint8_t *daddr;
    const uint32_t *ports;
    const uint32_t *meta;
    const uint32_t *mark;
    const uint8_t *tcp_flags;
    uint64_t n;
    /* skb->hash of each header (lb6_select_slave, lb.h:124-152, and the
     * monitor records), or NULL = CFC_FLOW_HASH over the addresses folded to
     * a word each (fold(a) = fmix32(w0 ^ fmix32(w1 ^ fmix32(w2 ^ fmix32(w3)))),
     * w = the address's raw words) */
    const uint32_t *hash;
} cfc_hdr_v6;

/* Outputs (device pointers, n elements; action may be NULL).
 *  verdict : bpf/lib/policy.h convention — <0 drop reason (DROP_*, or
 *            CFC_DROP_PREFILTER for an XDP prefilter drop), 0 forwarded,
 *            >0 proxy port (policy_entry.proxy_port, be16 raw).
 *  identity: INGRESS/FULL: source security identity the policy used;
 *            EGRESS: destination identity; XDP: 0.
 *  action  : return code of the last reference program that ran
 *            (TC_ACT_OK 0 / TC_ACT_SHOT 2 / TC_ACT_REDIRECT 7, or XDP_DROP 1 /
 *            XDP_PASS 2 in XDP mode and for prefilter drops in FULL mode). */
#define CFC_DROP_PREFILTER (-1)
/* IPv6 only: an ICMPv6 neighbour solicitation, or an echo request to the
 * router address, that the reference answers itself (icmp6_handle,
 * icmp6.h:390-412) instead of classifying; action TC_ACT_OK. */
#define CFC_VERDICT_PUNT (-2)
/*  ct      : (may be NULL) the CT byte of each header — what the reference's
 *            ct_lookup4/6 returned, against the CT maps as committed when
 *            the batch started: bits 0-1 CT_NEW 0 / ESTABLISHED 1 / REPLY 2 /
 *            RELATED 3, bit 2 looked up, bit 3 a new flow the reference
 *            would ct_create; bits 4-7 the same for the destination
 *            endpoint's ingress lookup after egress local delivery, or for
 *            the other family's lookup after a NAT hop (LXC_NAT46,
 *            lxc_config.h:28 / nat46.h:30-32: an IPv6 egress header to a
 *            v4-mapped peer outside the cluster re-runs as IPv4 through the
 *            endpoint's IPv4 egress path, bpf_lxc.c:353-360, 1070-1083; an
 *            IPv4 ingress header whose CT entry carries nat46 re-runs as IPv6
 *            through ipv6_policy, bpf_lxc.c:939-944, 1098-1110 — its verdict,
 *            identity, action and event are the hop's).  Feed it to
 *            cfc_ct_apply_v4/v6 of the same batch (cfc_classify's outputs
 *            untouched in between) to fold creates, deletes and closing flags
 *            into the CT maps, the hop's into the other family's. */
#define CFC_CT_RES_MASK 0x3u
#define CFC_CT_DONE 0x4u
#define CFC_CT_CREATE 0x8u
/*  notify  : (may be NULL) the monitor event the reference sent on its perf
 *            ring cilium_events for the header — at most one per header:
 *            0 none, else EVENT_SOURCE (the LXC_ID of the program that sent
 *            it, 0 for bpf_netdev) | kind << 16 with kind
 *              CFC_NT_NETDEV  drop: bpf_netdev's send_drop_notify_error
 *                             (bpf_netdev.c:463,502; no identities)
 *              CFC_NT_EGRESS  drop: the sending endpoint's send_drop_notify
 *                             (SECLABEL, dstID, 0, 0) (bpf_lxc.c:432,700)
 *              CFC_NT_POLICY  drop: the destination's tail_ipv{4,6}_policy
 *                             (src_label, SECLABEL, LXC_ID, ifindex)
 *                             (bpf_lxc.c:891,1024)
 *              CFC_NT_TRACE + obs   send_trace_notify at observation point
 *                             obs (TRACE_TO_LXC 0, TO_PROXY 1, TO_HOST 2,
 *                             TO_STACK 3; trace.h:37-48, call sites
 *                             bpf_lxc.c:373,390,668,687,873,1006, lxc.h:117,
 *                             169), with the CT result as reason in bits
 *                             20-21 and the monitor length in bits 22-23
 *                             (1 TRACE_PAYLOAD_LEN, 2 MTU, 3 one byte: an
 *                             active flow's periodic report, ct_update_timeout
 *                             returns bool, conntrack.h:191; 0: not sent — a
 *                             flow inside its report interval under
 *                             MONITOR_AGGREGATION 5, trace.h:119-132; the
 *                             site stays in the word so cfc_ct_apply can
 *                             re-decide the length in packet order).
 *            No event: a 0 word — forwarded packets the reference does not
 *            trace (to the stack from bpf_netdev; FROM_* points), XDP
 *            prefilter drops (bpf_xdp.c notifies nothing), punts — or a trace
 *            word of length class 0.
 *            cfc_drop_notify_v4/v6 turn the drops into records,
 *            cfc_monitor_events_v4/v6 every event. */
#define CFC_NT_NETDEV 1u
#define CFC_NT_EGRESS 2u
#define CFC_NT_POLICY 3u
#define CFC_NT_TRACE 4u
/* bit 24 of a nonzero word: the event was sent after a NAT hop (LXC_NAT46,
 * below) — the record's skb->len is the translated packet's (an IPv6
 * header's batch: 20 bytes less; an IPv4 one's: 20 more), its tuple the
 * header's own */
#define CFC_NT_NATLEN 0x01000000u
typedef struct {
    int32_t *verdict;
    uint32_t *identity;
    uint8_t *action;
    uint8_t *ct;
    uint32_t *notify;
    /* (may be NULL) the packet's L3/L4 addresses as the programs left
     * them: saddr, daddr and the first L4 word after service translation
     * (lb4_local / lb4_xlate: a service address and port replaced by the
     * backend's, a looped-back flow's source by IPV4_LOOPBACK) and reverse
     * NAT of load-balanced replies (lb4_rev_nat: the backend's source back
     * to the service address and port).  Headers the programs did not
     * rewrite keep their input.  (A proxy redirect's new port is the
     * verdict.)  cfc_classify_v6: pkt_saddr / pkt_daddr are n 16-byte rows
     * (16-byte aligned) — lb6_local / lb6_xlate, lb6_rev_nat of egress
     * replies, and ipv6_policy's rewrites (bpf_lxc.c:785-815: the last
     * word's low 16 bits of daddr cleared, the source of every hit whose
     * entry's rev_nat_index cilium_lb6_reverse_nat holds reverse-NATed). */
    uint32_t *pkt_saddr;
    uint32_t *pkt_daddr;
    uint32_t *pkt_ports;
} cfc_out;

/* Classify a batch (asynchronous on `stream`).  Policy-entry and metrics
 * counters accumulate on the device until cfc_counters_sync().
 * An EGRESS batch with out->ct whose headers talk to the sending endpoint's
 * own address (or to a service that loops back into it) is cut where a
 * header's lookup key may have been written by an earlier header of the
 * batch (conntrack.h:487-494, 725-748): the segments before the last are
 * classified and folded into CT here, in order (synchronising `stream`),
 * and the cfc_ct_apply_* of the same batch folds the last
 * (cfc_stats.ct_self_segments). */
int cfc_classify_v4(cfc_ctx *ctx, const cfc_hdr_v4 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream);
/* The IPv6 chain: bpf_netdev.c handle_ipv6 (:172-275) -> bpf_lxc.c
 * ipv6_policy (:753-895); egress ipv6_l3_from_lxc (:112-436); XDP check_v6
 * (bpf_xdp.c:132-156).  Same outputs and counters as cfc_classify_v4. */
int cfc_classify_v6(cfc_ctx *ctx, const cfc_hdr_v6 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream);

/* --------------------------------------------------------------- conntrack */
/* CT maps are opened through cfc_map_open with the pkg/maps/ctmap names
 * (ctmap.go:59-69): cilium_ct4_global, cilium_ct_any4_global,
 * cilium_ct6_global, cilium_ct_any6_global, or an endpoint's local maps
 * cilium_ct4_<lxc_id>, cilium_ct_any4_<lxc_id>, ... (LRU_HASH or HASH, key
 * struct ipv4_ct_tuple 14 B / ipv6_ct_tuple 38 B, value struct ct_entry
 * 56 B).  An endpoint with local maps uses them, every other the global
 * ones.  Every classify looks them up (ct_lookup4/6: reply / related
 * packets skip the policy verdict, the policy port of a reply is its source
 * port) and counts hits into the entries' rx/tx packets and bytes
 * (CONNTRACK_ACCOUNTING), visible after cfc_counters_sync().
 *
 * cfc_ct_apply_v4/v6 folds one classified batch (its headers and outputs,
 * out->ct set) into the CT maps in header order, as the reference does per
 * packet: ct_create4/6 for new flows (the flow entry and its ICMP "related"
 * entry), ct_delete for established flows the policy now denies, the
 * closing flags of RST/FIN (CFC_HF_TCP_CLOSE) and re-opening.  A flow seen
 * twice in one batch is created once and counted on its second packet.
 * The classify launch looked every header up against the maps as committed
 * before the batch; the apply first rewrites the CT bytes (and, with
 * out->notify, the trace words' reason and monitor length) into what the
 * reference's packet-at-a-time run gives — a later packet of a flow the
 * batch created is ESTABLISHED, a packet after a delete is NEW — and then
 * applies the writes.  A batch with a NAT hop (cfc_classify kept its hop
 * batch) folds the hop's stage into the other family's maps too.
 * Runs on the device (CFC_OPT_CT_APPLY) unless host-side CT map changes
 * wait for a commit, or an IPv6 (or, with CFC_OPT_CT_EVICT 0, an IPv4) CT
 * map could pass its max_entries: then on the host.  A table that would
 * pass 3/4 load is rebuilt larger.
 * Synchronises `stream`. */
int cfc_ct_apply_v4(cfc_ctx *ctx, const cfc_hdr_v4 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream);
int cfc_ct_apply_v6(cfc_ctx *ctx, const cfc_hdr_v6 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream);

/* Conntrack garbage collection: ctmap.GC(m, filter) (pkg/maps/ctmap/
 * ctmap.go:339-350) with doFiltering (:303-325) on one CT map (`fd`), or on
 * every CT map (fd = -1: what EnableConntrackGC's loop covers,
 * pkg/endpointmanager/conntrack.go:96-125, every
 * conntrack-garbage-collector-interval, 60 s by default,
 * daemon/main.go:367).  struct GCFilter (ctmap.go:163-182): */
#define CFC_GC_REMOVE_EXPIRED 1u   /* RemoveExpired: delete lifetime < time */
#define CFC_GC_VALID_IPS 2u        /* ValidIPs set: delete when neither tuple
                                      address is in valid_ips (empty set: all) */
#define CFC_GC_MATCH_IPS 4u        /* MatchIPs set: delete when either is in
                                      match_ips */
typedef struct {
    uint8_t family;                /* 4 or 6 */
    uint8_t pad[3];
    uint8_t addr[16];              /* network order; IPv4: the first 4 bytes */
} cfc_ip;
typedef struct {
    uint32_t flags;                /* CFC_GC_* */
    uint32_t time;                 /* Time, bpf_ktime_get_sec() seconds
                                      (ctmap.GC fills it from bpf.GetMtime) */
    const cfc_ip *valid_ips;
    uint32_t n_valid;
    uint32_t pad0;
    const cfc_ip *match_ips;
    uint32_t n_match;
    uint32_t pad1;
} cfc_ct_gc_filter;
/* gcStats (ctmap.go doGC4/doGC6): entries deleted and left in the selected
 * maps; where the work happened */
typedef struct {
    uint64_t deleted;
    uint64_t alive;
    uint64_t device_deleted;       /* IPv4 entries in the device table */
    uint64_t log_deleted;          /* ICMP entries of device creates in TCP
                                      maps not yet in the host mirror (one
                                      per pending write: a key written twice
                                      before the host took it counts twice) */
    uint64_t host_deleted;         /* entries only the host holds (IPv6, and
                                      IPv4 TCP maps' ICMP entries) */
    uint64_t slots_freed;          /* device slots returned to free (the rest
                                      of the deletes stay tombstones) */
} cfc_ct_gc_stats;
/* The IPv4 part runs on the device (one pass over the CT table: deleted
 * entries become tombstones at once, a cluster's trailing tombstones become
 * free slots; the host mirror takes the deletes lazily, like the applies'
 * changes).  Commits pending host-side map changes first.  Synchronises
 * `stream`. */
int cfc_ct_gc(cfc_ctx *ctx, int fd, const cfc_ct_gc_filter *filter,
              cfc_ct_gc_stats *stats, void *stream);

/* ------------------------------------------------------ drop notifications */
/* struct drop_notify (bpf/lib/drop.h:40-48, NOTIFY_COMMON_HDR common.h:217)
 * as __send_drop_notify (drop.h:50-78) fills it for the perf ring
 * cilium_events, which pkg/monitor decodes (datapath_drop.go:28-40
 * DropNotify: the same fields, little-endian, 32 bytes).
 * The captured payload that follows it on the ring (len_cap bytes of the
 * packet) is not part of a header batch; hdr_index locates the header. */
#define CFC_NOTIFY_DROP 1          /* CILIUM_NOTIFY_DROP (common.h:211) */
#define CFC_TRACE_PAYLOAD_LEN 128  /* TRACE_PAYLOAD_LEN (common.h:224) */
typedef struct {
    uint8_t type;        /* CFC_NOTIFY_DROP */
    uint8_t subtype;     /* -reason (DROP_* magnitude) */
    uint16_t source;     /* EVENT_SOURCE: LXC_ID of the endpoint program, 0
                            for bpf_netdev */
    uint32_t hash;       /* symmetric 5-tuple flow hash: the reference's
                            get_hash_recalc() is the kernel's skb hash under
                            a boot-random key */
    uint32_t len_orig;   /* skb->len */
    uint32_t len_cap;    /* min(CFC_TRACE_PAYLOAD_LEN, len_orig) */
    uint32_t src_label;  /* cb[1] >> 16: 16 bits of the source identity */
    uint32_t dst_label;  /* cb[1] & 0xFFFF */
    uint32_t dst_id;     /* cb[3] */
    uint32_t ifindex;    /* cb[4] */
} cfc_drop_notify;

/* The drop notifications of one classified batch (in: the headers, out: its
 * outputs with out->notify set), in header order, into device memory
 * (`records` 16-byte aligned, else -EINVAL):
 * records[0 .. min(total, cap)) and, if hdr_index != NULL, the header index
 * of each.  *count (device u64) receives the total; drops past cap are not
 * recorded (a full perf ring loses samples the same way).  mode and ep_lxc
 * as given to the classify call.  The records' endpoint fields (SECLABEL,
 * ifindex) come from the endpoint table committed at the time of this call:
 * call it before a commit that changes cilium_lxc or an endpoint's config.
 * Asynchronous on `stream`. */
int cfc_drop_notify_v4(cfc_ctx *ctx, const cfc_hdr_v4 *in, const cfc_out *out,
                       int mode, uint16_t ep_lxc, cfc_drop_notify *records,
                       uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                       void *stream);
int cfc_drop_notify_v6(cfc_ctx *ctx, const cfc_hdr_v6 *in, const cfc_out *out,
                       int mode, uint16_t ep_lxc, cfc_drop_notify *records,
                       uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                       void *stream);

/* struct trace_notify (bpf/lib/trace.h:71-81) as send_trace_notify
 * (:97-155) fills it; pkg/monitor decodes it (datapath_trace.go:28-40
 * TraceNotify).  32 bytes, like cfc_drop_notify: the `type` byte tells a
 * record of cfc_monitor_events apart. */
#define CFC_NOTIFY_TRACE 4         /* CILIUM_NOTIFY_TRACE (common.h:214) */
typedef struct {
    uint8_t type;        /* CFC_NOTIFY_TRACE */
    uint8_t subtype;     /* observation point TRACE_TO_* */
    uint16_t source;     /* EVENT_SOURCE */
    uint32_t hash;       /* symmetric flow hash (see cfc_drop_notify) */
    uint32_t len_orig;
    uint32_t len_cap;    /* min(monitor length, len_orig) */
    uint32_t src_label;  /* full 32-bit identities */
    uint32_t dst_label;
    uint16_t dst_id;
    uint8_t reason;      /* TRACE_REASON_*: the CT result */
    uint8_t pad;
    uint32_t ifindex;
} cfc_trace_notify;

/* Every monitor event of one classified batch (out->notify set) — drop and
 * trace records, 32 bytes each, in header order — as the perf ring
 * cilium_events would carry them; otherwise as cfc_drop_notify_v4/v6. */
int cfc_monitor_events_v4(cfc_ctx *ctx, const cfc_hdr_v4 *in, const cfc_out *out,
                          int mode, uint16_t ep_lxc, void *records,
                          uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                          void *stream);
int cfc_monitor_events_v6(cfc_ctx *ctx, const cfc_hdr_v6 *in, const cfc_out *out,
                          int mode, uint16_t ep_lxc, void *records,
                          uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                          void *stream);

/* ---------------------------------------------------------------- counters */
/* The device counter block is a flat u64 array:
 *   [n_entries][packets, bytes]   policy entries, in the committed epoch's
 *                                 entry order (policy_entry counters);
 *   [256 reasons][4 dirs][count, bytes]   cilium_metrics (update_metrics);
 *   [2 dirs][65537 identities][fwd, drop][packets, bytes]   the
 *                                 per-identity forward/drop counters below.
 * It is identical in layout on every rank holding the same tables, so it
 * can be all-reduced in place (RCCL) before cfc_counters_sync(). */
int cfc_counters_device(cfc_ctx *ctx, uint64_t **dev_ptr, uint64_t *n_u64);
/* Fold the device counters into the host maps (policy entry packets/bytes,
 * cilium_metrics, the per-identity totals) and zero them.  Synchronises
 * `stream`. */
int cfc_counters_sync(cfc_ctx *ctx, void *stream);
/* Zero the device counters without folding (e.g. on non-root ranks after
 * an all-reduce whose result was folded elsewhere). */
int cfc_counters_clear(cfc_ctx *ctx, void *stream);
/* Copy the counter block into caller device memory `dst` (n_u64 u64, as
 * reported by cfc_counters_device) and zero it — the send side of a
 * counter all-reduce.  cfc_counters_import adds `src` back in. */
int cfc_counters_export(cfc_ctx *ctx, uint64_t *dst, uint64_t n_u64,
                        void *stream);
int cfc_counters_import(cfc_ctx *ctx, const uint64_t *src, uint64_t n_u64,
                        void *stream);

/* Per-identity forward/drop counters (BASELINE north_star: the counters the
 * multi-GPU path all-reduces over RCCL).  One event per policy verdict the
 * datapath makes — every __policy_can_access the reference runs
 * (policy.h:46-110) through ipv{4,6}_policy (bpf_lxc.c:753-1028, dir
 * ingress, identity = the source identity) or handle_ipv4_from_lxc /
 * ipv6_l3_from_lxc (:112-704, dir egress, identity = the destination
 * identity); after egress local delivery the destination's ingress verdict
 * is a second event (identity = the sender's SECLABEL).  The event is a
 * drop when the verdict path drops it (DROP_POLICY: a denied verdict not
 * overridden by CT_REPLY/CT_RELATED), a forward otherwise (including proxy
 * redirects).  Packets and skb->len bytes.  Identities >= 65536 (outside
 * pkg/identity's allocation range, numericidentity.go) are counted in one
 * row with identity CFC_IDENTITY_OUT_OF_RANGE.
 * cfc_identity_counters returns the totals folded by cfc_counters_sync
 * (since the context was opened), one row per (identity, dir) with a
 * non-zero count, sorted by identity then dir: rows[0 .. min(*n, cap)),
 * *n = the number of rows. */
#define CFC_IDENTITY_OUT_OF_RANGE 0xFFFFFFFFu
typedef struct {
    uint32_t identity;
    uint8_t dir;          /* METRIC_INGRESS 1 / METRIC_EGRESS 2 */
    uint8_t pad[3];
    uint64_t fwd_packets, fwd_bytes;
    uint64_t drop_packets, drop_bytes;
} cfc_identity_count;
int cfc_identity_counters(cfc_ctx *ctx, cfc_identity_count *rows, uint64_t cap,
                          uint64_t *n);

/* ------------------------------------------------------------- diagnostics */
typedef struct {
    uint64_t epoch;
    uint64_t device_bytes;      /* bytes of device tables in this epoch */
    uint32_t ipcache_v4_prefixes;
    uint32_t lpm4_tbl8_groups;
    uint32_t policy_entries;
    uint32_t endpoints;
    uint32_t prefilter_v4_fix;
    uint32_t prefilter_v4_dyn;
    uint32_t lpm4_layout;       /* CFC_LPM4_DIR24_8 / _TRIE, 0 = empty */
    uint32_t lpm4_kib;          /* device KiB of the IPv4 ipcache layout */
    uint32_t ipcache_v6_prefixes;
    uint32_t lpm6_lengths;      /* distinct IPv6 prefix lengths (> 0) */
    uint32_t lpm6_groups;       /* Bloom groups over them */
    uint32_t lpm6_kib;          /* device KiB of the IPv6 ipcache layout */
    uint32_t endpoints_v6;
    uint32_t prefilter_v6_fix;
    uint32_t prefilter_v6_dyn;
    uint32_t ct4_entries;       /* CT entries a lookup can reach (as of the
                                   last host synchronisation) */
    uint32_t ct6_entries;
    uint32_t ct_apply_device;   /* cfc_ct_apply_* calls run on the device */
    uint32_t ct_apply_host;     /* ... and on the host */
    /* CT slots of the device tables (both families) */
    uint32_t ct_slots;
    /* times a device CT table grew on the device (cfc_ct_apply_*: a batch
     * that would take it past 3/4 load moves it into a table of more slots,
     * no host rebuild), since the context opened (was pad0) */
    uint32_t ct_grown;
    /* CT stages whose result the packet order changed from the batch-start
     * lookup (cfc_ct_apply: a later packet of a flow the batch created,
     * a packet after a delete), since the context opened (ABI 12: 64-bit,
     * read after the last call on any stream has finished) */
    uint64_t ct_order_changed;
    /* headers that took a NAT46 / NAT64 hop (cfc_classify_*), since the
     * context opened */
    uint64_t nat_hops;
    /* CT entries deleted to make room at a map's max_entries before a device
     * apply (CFC_OPT_CT_EVICT), since the context opened */
    uint64_t ct_evicted;
    /* headers whose service step found the CT_SERVICE entry an earlier
     * header of the same batch created or re-selected (cfc_classify_*) */
    uint64_t svc_ordered;
    /* device applies whose scan and ordering passes read the classify
     * launch's work list (the headers with a CT stage that is not a plain
     * hit) rather than the whole batch */
    uint64_t ct_apply_sparse;
    /* (ABI 13) segments an egress batch with traffic to itself was cut into
     * beyond its first, each classified after the ones before it were
     * folded into CT (cfc_classify_*: a header whose lookup key an earlier
     * header of the batch may have written — an endpoint talking to its own
     * address, a service flow looped back into it; conntrack.h:487-494,
     * 725-748), since the context opened */
    uint64_t ct_self_segments;
} cfc_stats;
int cfc_get_stats(cfc_ctx *ctx, cfc_stats *st);
const char *cfc_strerror(int err);

/* Device time of the kernels of the cfc_classify_* calls made since the
 * previous collect with CFC_OPT_TIMING on (waits for them to finish):
 * classify_ms sums the lookup kernel, count_ms the counter kernels, over
 * every call; the *_v6 fields the cfc_classify_v6 calls among them. */
typedef struct {
    uint64_t launches;
    double classify_ms;
    double count_ms;
    uint64_t launches_v6;
    double classify_v6_ms;
    double count_v6_ms;
} cfc_timing;
int cfc_timing_collect(cfc_ctx *ctx, cfc_timing *out);

#ifdef __cplusplus
}
#endif
#endif /* CFC_H */
