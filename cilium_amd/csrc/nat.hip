// LXC_NAT46: the NAT hops between the IPv6 and IPv4 paths of an endpoint
// (lxc_config.h:28 ENABLE_NAT46, with IPv4 and CONNTRACK: nat46.h:30-32).
//
//   NAT64  bpf_lxc.c:353-360 -> tail_ipv6_to_ipv4 (:1070-1083): an IPv6
//          egress header to a v4-mapped peer (::ffff:0:0/96, ipv6.h:279-282)
//          outside the cluster is translated (ipv6_to_ipv4, nat46.h:336-420:
//          saddr LXC_IPV4, daddr the address's last 32 bits, ICMPv6 as
//          ICMP) and classified again by handle_ipv4_from_lxc with
//          cb[CB_NAT46_STATE] = NAT64, whose ct_create4 sets nat46
//          (conntrack.h:714-716).
//   NAT46  bpf_lxc.c:939-944 -> tail_ipv4_to_ipv6 (:1098-1110): an IPv4
//          ingress header whose ct_lookup4 hit an entry with nat46
//          (conntrack.h:241-244) is translated (ipv4_to_ipv6,
//          nat46.h:236-328: saddr NAT46_PREFIX/96 + the IPv4 source, daddr
//          LXC_IP, ICMP as ICMPv6) and checked by ipv6_policy with the IPv4
//          path's source identity.
//
// The classify kernels list the headers that take a hop (EgressArgs.nat_idx);
// cfc_classify sorts the list into header order, gathers those headers
// translated into a batch of the other family (the "hop batch"), classifies
// it with the same tables and counters, and scatters its results back: the
// hop's verdict, identity, action and event are the header's, its CT stage
// the header's CT byte bits 4-7.  cfc_ct_apply folds the header's own stage
// with its family's batch and the hop batch into the other family's maps.
#include <hipcub/hipcub.hpp>

#include "kern_common.hpp"

namespace cfc {

namespace {

// icmp4_to_icmp6 (nat46.h:60-141) on {type, code}.  Its callers take the
// return value as a checksum difference and never test it (nat46.h:303,
// :384): an unknown type or code leaves the ICMP header as it was.
__device__ __forceinline__ uint32_t icmp4_to_icmp6(uint32_t w)
{
    const uint32_t type = w & 0xFF, code = (w >> 8) & 0xFF;
    uint32_t t6 = 0, c6 = 0;
    switch (type) {
    case 8: t6 = 128; break;   // ECHO -> ECHO_REQUEST
    case 0: t6 = 129; break;   // ECHOREPLY
    case 3:                    // DEST_UNREACH
        t6 = 1;
        switch (code) {
        case 0: case 1: case 5: case 6: case 7: case 8: case 11: case 12: c6 = 0; break;
        case 2: t6 = 4; c6 = 1; break;   // PARAMPROB / UNK_NEXTHDR
        case 3: c6 = 4; break;           // PORT_UNREACH
        case 4: t6 = 2; c6 = 0; break;   // PKT_TOOBIG
        case 9: case 10: case 13: c6 = 1; break;   // ADM_PROHIBITED
        default: return w;
        }
        break;
    case 11: t6 = 3; break;    // TIME_EXCEEDED
    case 12: t6 = 4; break;    // PARAMETERPROB
    default: return w;
    }
    return (w & 0xFFFF0000u) | t6 | c6 << 8;
}

// icmp6_to_icmp4 (nat46.h:143-220), its fall-throughs included: a
// destination unreachable with a known code ends as FRAG_NEEDED (no break
// after the inner switch), a parameter problem as an unknown type
__device__ __forceinline__ uint32_t icmp6_to_icmp4(uint32_t w)
{
    const uint32_t type = w & 0xFF, code = (w >> 8) & 0xFF;
    uint32_t t4 = 0, c4 = 0;
    switch (type) {
    case 128: t4 = 8; break;
    case 129: t4 = 0; break;
    case 1:
        if (code > 4)
            return w;
        t4 = 3;
        c4 = 4;
        break;
    case 2: t4 = 3; c4 = 4; break;
    case 3: t4 = 11; c4 = code; break;
    default: return w;   // (4: unknown type or code either way)
    }
    return (w & 0xFFFF0000u) | t4 | c4 << 8;
}

// NAT64: hop batch row k <- header idx[k] of the IPv6 egress batch
__global__ __launch_bounds__(256) void k_nat64_gather(cfc_hdr_v6 in, const uint32_t *idx,
                                                      uint32_t m, uint32_t sa4, NatHop4 h)
{
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= m)
        return;
    const uint32_t i = idx[k];
    const uint32_t *da = reinterpret_cast<const uint32_t *>(in.daddr) + 4ull * i;
    const uint32_t mt = in.meta[i], proto = mt & 0xFF;
    uint32_t pt = in.ports[i];
    if (proto == 58)
        pt = icmp6_to_icmp4(pt);
    h.sa[k] = sa4;
    h.da[k] = da[3];   // the v4-mapped address's last 32 bits
    h.pt[k] = pt;
    // (the IPv4 header is 20 bytes shorter: skb->len - 20)
    h.mt[k] = (proto == 58 ? 1u : proto) | (mt & 0xFF00u) | ((mt >> 16) - 20u) << 16;
    h.tf[k] = in.tcp_flags ? in.tcp_flags[i] : 0;
    // skb->hash stays the one the IPv6 packet had (lb4_select_slave)
    if (h.hash) {
        const uint32_t *sa = reinterpret_cast<const uint32_t *>(in.saddr) + 4ull * i;
        h.hash[k] = in.hash ? in.hash[i]
                            : flow_hash6(make_uint4(sa[0], sa[1], sa[2], sa[3]),
                                         make_uint4(da[0], da[1], da[2], da[3]), in.ports[i],
                                         proto);
    }
}

// NAT46: hop batch row k <- header idx[k] of the IPv4 ingress batch; the
// destination endpoint found again by daddr, its LXC_IP from ep6
__global__ __launch_bounds__(256) void k_nat46_gather(DevTables T, cfc_hdr_v4 in,
                                                      const uint32_t *ident, const uint32_t *idx,
                                                      uint32_t m, const uint4 *ep6, NatHop6 h)
{
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= m)
        return;
    const uint32_t i = idx[k];
    const uint32_t da = in.daddr[i];
    Lds S{};
    const uint32_t s0 = hash32(da, T.lxc4_mask);
    const uint4 rec = lxc_resolve(T, S, da, s0, lxc_slot(T, S, s0));
    const uint32_t mt = in.meta[i], proto = mt & 0xFF;
    uint32_t pt = in.ports[i];
    if (proto == 1)
        pt = icmp4_to_icmp6(pt);
    // NAT46_PREFIX beef::a00:0/96 (node_config.h:40) + the IPv4 source, raw
    h.sa[k] = make_uint4(0x0000EFBEu, 0u, 0x000A0000u, in.saddr[i]);
    h.da[k] = ep6[rec.w & 0xFFFF];
    h.pt[k] = pt;
    h.mt[k] = (proto == 1 ? 58u : proto) | (mt & 0xFF00u) | ((mt >> 16) + 20u) << 16;
    // tc_index carries the skip-proxy mark across the tail calls
    h.mk[k] = in.mark ? (in.mark[i] & 0xF00u) : 0u;
    h.tf[k] = in.tcp_flags ? in.tcp_flags[i] : 0;
    h.id[k] = ident[i];
}

// the hop's results into the header's outputs: verdict, identity, action,
// event (CFC_NT_NATLEN), and its CT stage as the header's bits 4-7 (the
// hop's own local delivery — a third stage — is not carried: cleared)
__global__ __launch_bounds__(256) void k_nat_scatter(const uint32_t *idx, uint32_t m, cfc_out sub,
                                                     cfc_out out)
{
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= m)
        return;
    const uint32_t i = idx[k];
    out.verdict[i] = sub.verdict[k];
    out.identity[i] = sub.identity[k];
    if (out.action)
        out.action[i] = sub.action[k];
    if (out.ct) {
        // (the hop batch keeps its own second stage — a NAT64 hop's local
        // delivery, the destination's ipv4_policy lookup: a third CT stage
        // its apply folds — the header's byte has room for the hop's first)
        const uint32_t c = sub.ct[k] & 0x0F;
        out.ct[i] = (uint8_t)((out.ct[i] & 0x0F) | c << 4);
    }
    if (out.notify) {
        const uint32_t w = sub.notify[k];
        out.notify[i] = w ? w | CFC_NT_NATLEN : 0u;
    }
}

// before the apply of the header's own family: its stage alone — allowed
// (it led to the hop), no second stage, no event to re-decide
__global__ __launch_bounds__(256) void k_nat_pre(const uint32_t *idx, uint32_t m, cfc_out out)
{
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= m)
        return;
    const uint32_t i = idx[k];
    out.verdict[i] = 0;
    out.ct[i] &= 0x0F;
    if (out.notify)
        out.notify[i] = 0;
}

}  // namespace

size_t nat_sort_tmp_bytes(uint32_t m)
{
    size_t b = 0;
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const uint32_t *)nullptr,
                                            (uint32_t *)nullptr, (int)m, 0, 32);
    return b;
}

int nat_sort(const uint32_t *in, uint32_t *out, uint32_t m, uint64_t n, void *tmp,
             size_t tmp_bytes, hipStream_t s)
{
    int bits = 1;
    while (bits < 32 && (1ull << bits) < n)
        bits++;
    return hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, in, out, (int)m, 0, bits, s) ==
                   hipSuccess
               ? 0
               : -5;
}

int nat64_gather(const cfc_hdr_v6 &in, const uint32_t *idx, uint32_t m, uint32_t sa4,
                 const NatHop4 &h, hipStream_t s)
{
    if (m)
        hipLaunchKernelGGL(k_nat64_gather, dim3((m + 255) / 256), dim3(256), 0, s, in, idx, m,
                           sa4, h);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int nat46_gather(const DevTables &T, const cfc_hdr_v4 &in, const uint32_t *ident,
                 const uint32_t *idx, uint32_t m, const uint4 *ep6, const NatHop6 &h,
                 hipStream_t s)
{
    if (m)
        hipLaunchKernelGGL(k_nat46_gather, dim3((m + 255) / 256), dim3(256), 0, s, T, in, ident,
                           idx, m, ep6, h);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int nat_scatter(const uint32_t *idx, uint32_t m, const cfc_out &sub, const cfc_out &out,
                hipStream_t s)
{
    if (m)
        hipLaunchKernelGGL(k_nat_scatter, dim3((m + 255) / 256), dim3(256), 0, s, idx, m, sub,
                           out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int nat_pre(const uint32_t *idx, uint32_t m, const cfc_out &out, hipStream_t s)
{
    if (m)
        hipLaunchKernelGGL(k_nat_pre, dim3((m + 255) / 256), dim3(256), 0, s, idx, m, out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace cfc
