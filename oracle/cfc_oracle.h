/*
 * cfc_oracle — CPU restatement of the reference verdict path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the GPU engine is compared
 * against (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg).
 * It is never linked into or called by the product (cilium_amd/libcfc.so).
 *
 * Pinned against golden vectors produced by the reference's own BPF programs
 * run with BPF_PROG_TEST_RUN (oracle/gen_golden.py -> tests/golden/).
 *
 * Conventions are the reference datapath's: addresses/ports are raw
 * network-order bytes loaded little-endian (be32/be16 "raw"), identities are
 * host-order u32, verdicts follow bpf/lib/policy.h (<0 drop reason, 0 allow,
 * >0 proxy port as stored in policy_entry.proxy_port).
 */
#ifndef CFC_ORACLE_H
#define CFC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfo cfo_t;

enum { CFO_MODE_INGRESS = 0, CFO_MODE_EGRESS = 1, CFO_MODE_XDP = 2,
       CFO_MODE_FULL = 3 };

cfo_t *cfo_new(void);
void cfo_free(cfo_t *o);

/* family: 1 = IPv4, 2 = IPv6 (ENDPOINT_KEY_IPV4/6, common.h:139-140) */
int cfo_ipcache_add(cfo_t *o, int family, int plen, const uint8_t addr[16],
                    uint32_t label);
/* ipcache_lookup4/6 (eps.h:56-80): the longest prefix holding each of n
 * addresses (IPv4: 4 bytes each, IPv6: 16) -> label[i], hit[i] = 1 when a
 * prefix matched; the lookup the identity derivations make */
void cfo_ipcache_lookup(cfo_t *o, int family, size_t n, const uint8_t *addrs,
                        uint32_t *label, uint8_t *hit);
int cfo_endpoint_add(cfo_t *o, int family, const uint8_t addr[16],
                     uint32_t ifindex, uint16_t lxc_id, uint32_t flags);
int cfo_seclabel_set(cfo_t *o, uint16_t lxc_id, uint32_t seclabel);
/* node_config.h IPV4_CLUSTER_RANGE / IPV4_CLUSTER_MASK (raw be32 as loaded)
 * and ROUTER_IP; cfo_new() starts with the reference's values */
/* per-identity forward/drop counters: rows of 6 u64 {identity (0xFFFFFFFF
 * for >= 65536), dir (1 ingress / 2 egress), fwd packets, fwd bytes, drop
 * packets, drop bytes}, sorted; returns the row count */
size_t cfo_identity_dump(cfo_t *o, uint64_t *rows, size_t cap);
void cfo_node_config(cfo_t *o, uint32_t v4_cluster_range,
                     uint32_t v4_cluster_mask, const uint8_t router_ip6[16],
                     uint32_t host_ifindex);
/* An endpoint program (and its policymap) exists for lxc_id.  Endpoints in
 * cilium_lxc without one drop with DROP_MISSED_TAIL_CALL. */
int cfo_policy_create(cfo_t *o, uint16_t lxc_id);
int cfo_policy_add(cfo_t *o, uint16_t lxc_id, uint32_t identity,
                   uint16_t dport_be, uint8_t proto, uint8_t egress,
                   uint16_t proxy_port_be);
int cfo_prefilter_add(cfo_t *o, int family, int plen, const uint8_t addr[16],
                      int dyn);

/* Classify n IPv4 headers (SoA).  mark may be NULL.  Outputs: action = the
 * return code of the last reference program run (TC_ACT_* or XDP_*),
 * verdict (policy.h convention; -1 = XDP prefilter drop), identity (ingress:
 * source security identity used for policy; egress: destination identity).
 * Counters accumulate in the oracle's policy entries and metrics table.
 * lookups (may be NULL) receives, per header, the number of map lookups
 * the reference executes (prefilter, endpoint, ipcache, policy): the L of
 * SURVEY.md §8d's algorithmic-bytes formula. */
void cfo_classify_v4(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint32_t *saddr, const uint32_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint32_t *mark,
                     const uint8_t *tcpflags, int32_t *action, int32_t *verdict,
                     uint32_t *identity, uint8_t *lookups, uint8_t *ct,
                     int nthreads);

/* The same for IPv6: saddr/daddr are n x 16 raw address bytes; proto is the
 * next header ipv6_hdrlen() stops at (44 / 59 drop); flags bit 2 (4) marks
 * extension headers in front of it.  ICMPv6 neighbour solicitations and echo
 * requests to ROUTER_IP, which the datapath answers itself
 * (icmp6.h:390-412), come back as verdict -2 (punted). */
void cfo_classify_v6(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint8_t *saddr, const uint8_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint32_t *mark,
                     const uint8_t *tcpflags, int32_t *action, int32_t *verdict,
                     uint32_t *identity, uint8_t *lookups, uint8_t *ct,
                     int nthreads);

/* rows of 7 u64: identity, dport, proto, egress, proxy_port, packets, bytes
 * (sorted); returns the number of rows (writes at most cap). */
/* The monitor event of every header of the next classify calls (a drop
 * site or a trace_notify observation point, cfc_oracle.c NT_*), one u32 per
 * header into `words`, and each CT stage's monitor length (stage 1 in bits
 * 0-15, stage 2 in 16-31) into `mon`; NULL = off.  tcpflags (classify, may
 * be NULL = 0) is TCP header byte 13 of each header, the flags ct_lookup
 * accumulates into the CT entry. */
void cfo_set_notify_out(cfo_t *o, uint32_t *words, uint32_t *mon);
/* bpf_ktime_get_sec() for the next classify / ct_apply calls: the clock of
 * the CT lifetimes and report intervals (conntrack.h:125-205) */
void cfo_set_clock(cfo_t *o, uint32_t now);

size_t cfo_policy_dump(cfo_t *o, uint16_t lxc_id, uint64_t *rows, size_t cap);
/* rows of 4 u64: reason, dir, count, bytes (sorted, non-zero only) */
size_t cfo_metrics_dump(cfo_t *o, uint64_t *rows, size_t cap);
void cfo_counters_reset(cfo_t *o);

/* ---- conntrack (bpf/lib/conntrack.h) ----
 * cfo_classify_* look CT up against the maps as they are when the call
 * starts and report, per header, a CT byte (ct may be NULL):
 *   bits 0-1 CT result of stage 1 (CT_NEW 0, ESTABLISHED 1, REPLY 2,
 *   RELATED 3), bit 2 stage 1 looked up, bit 3 stage 1 creates; bits 4-7 the
 *   same for stage 2 (the destination's ingress policy after egress local
 *   delivery).  cfo_ct_apply_* then folds the batch into the maps.
 * Entries: lxc = -1 for the global maps, else the endpoint's local maps;
 * tuple = struct ipv{4,6}_ct_tuple bytes; entry = struct ct_entry (56 B). */
int cfo_ct_add(cfo_t *o, int family, int lxc, int any_map,
               const uint8_t *tuple, const uint8_t entry[56]);
int cfo_ct_add_n(cfo_t *o, size_t n, const uint8_t *records);
void cfo_ct_apply_v4(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint32_t *saddr, const uint32_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint8_t *tcpflags,
                     const uint32_t *identity, const int32_t *verdict,
                     const uint8_t *ct, const uint32_t *mon, uint8_t *hazard);
void cfo_ct_apply_v6(cfo_t *o, int mode, uint16_t ep_lxc, size_t n,
                     const uint8_t *saddr, const uint8_t *daddr,
                     const uint16_t *sport, const uint16_t *dport,
                     const uint8_t *proto, const uint8_t *flags,
                     const uint16_t *len, const uint8_t *tcpflags,
                     const uint32_t *identity, const int32_t *verdict,
                     const uint8_t *ct, const uint32_t *mon, uint8_t *hazard);
/* live CT entries as rows of CFO_CT_ROW bytes: u16 owner (0 global, else
 * lxc_id + 1), u8 map (0 TCP, 1 ANY), u8 family, tuple (40 B, zero padded),
 * struct ct_entry (56 B), 4 B pad; sorted by the first 44 bytes. */
/* service load balancing (bpf/lib/lb.h, IPv4): cilium_lb4_services
 * (key struct lb4_key 8 B, value struct lb4_service 12 B) and
 * cilium_lb4_reverse_nat (value struct lb4_reverse_nat 6 B) */
int cfo_lb4_service_add(cfo_t *o, const uint8_t key[8], const uint8_t val[12]);
int cfo_lb4_revnat_add(cfo_t *o, uint16_t index, const uint8_t val[6]);
/* IPv6: cilium_lb6_services (key struct lb6_key 20 B, value struct
 * lb6_service 24 B) and cilium_lb6_reverse_nat (value 18 B) */
int cfo_lb6_service_add(cfo_t *o, const uint8_t key[20], const uint8_t val[24]);
int cfo_lb6_revnat_add(cfo_t *o, uint16_t index, const uint8_t val[18]);
/* per-header inputs / outputs of the next classify / ct_apply calls: hash =
 * skb->hash (NULL: cfo_flow_hash4/6), pkt = the packet's saddr, daddr and
 * first L4 word after the program's rewrites (IPv4 3 u32 per header, IPv6
 * 9: saddr[4], daddr[4], L4 word; or NULL) */
void cfo_set_lb_io(cfo_t *o, const uint32_t *hash, uint32_t *pkt);
uint32_t cfo_flow_hash4(uint32_t sa, uint32_t da, uint16_t sport, uint16_t dport,
                        uint8_t proto);
uint32_t cfo_flow_hash6(const uint8_t sa[16], const uint8_t da[16], uint16_t sport,
                        uint16_t dport, uint8_t proto);
#define CFO_CT_ROW 104
size_t cfo_ct_dump(cfo_t *o, uint8_t *rows, size_t cap);
/* the reference's semantics: headers one at a time, each folded into the CT
 * maps before the next, at clock[i] (NULL: the clock as set) */
void cfo_run_seq(cfo_t *o, int family, int mode, uint16_t ep_lxc, size_t n,
                 const uint8_t *saddr, const uint8_t *daddr, const uint16_t *sport,
                 const uint16_t *dport, const uint8_t *proto, const uint8_t *flags,
                 const uint16_t *len, const uint32_t *mark, const uint8_t *tcpflags,
                 const uint32_t *clock, int32_t *action, int32_t *verdict,
                 uint32_t *identity, uint8_t *ct, uint32_t *words);
/* ctmap.GC with doFiltering (pkg/maps/ctmap/ctmap.go:303-350) on the
 * selected maps (family 0/1/2, owner -1/0/lxc_id + 1, kind -1/0 TCP/1 ANY);
 * IP sets are 17-byte {family, address[16]} records, n = SIZE_MAX: no set */
size_t cfo_ct_gc(cfo_t *o, int family, int owner, int kind, int remove_expired,
                 uint32_t time, const uint8_t *valid, size_t n_valid,
                 const uint8_t *match, size_t n_match);

#ifdef __cplusplus
}
#endif
#endif
