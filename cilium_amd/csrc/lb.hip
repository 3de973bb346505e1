// Service load balancing of an egress batch (gfx950), ahead of the classify
// kernel: what handle_ipv4_from_lxc does to the tuple and the packet before
// its conntrack lookup (bpf_lxc.c:476-492, lb.h:590-776) and, for a reply
// of a load-balanced flow, right after it (bpf_lxc.c:565-576, lb4_rev_nat).
// One thread per header; all lookups are against the tables as committed,
// but for the CT_SERVICE entry an earlier header of the batch created or
// re-slaved (LbArgs.svo, svcorder.hip); the batch's CT_SERVICE writes are
// folded in by cfc_ct_apply_v4.
//
// Per header it leaves, for the classify kernel:
//   tda, tpt  the tuple's daddr and L4 word for the sending endpoint's CT
//             lookup, ipcache lookup and policy (a backend's, or for a flow
//             looped back into its sender the service's address)
//   psa, pda, ppt  the packet as the destination's program (local delivery)
//             and the caller see it: translated, reverse-NATed
//   fl        LBF_DROP (DROP_NO_SERVICE), LBF_SVC, LBF_LOOP, and the
//             backend's rev_nat_index in bits 16-31
#include "kern_common.hpp"

namespace cfc {

namespace {

__global__ __launch_bounds__(256) void k_lb4_egress(DevTables T, LbArgs A)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n)
        return;
    const uint32_t sa = A.sa[i], da = A.da[i], pt = A.pt[i];
    const uint32_t proto = A.mt[i] & 0xFF;
    uint32_t tda = da, tpt = pt, psa = sa, pda = da, ppt = pt, fl = 0;
    const bool l4 = proto == 6 || proto == 17;
    // lb4_extract_key: TCP/UDP carry their dport, ICMP none; any other
    // protocol skips the service step (DROP_UNKNOWN_L4 -> skip_service_lookup)
    uint32_t kd = l4 ? pt >> 16 : 0u;
    uint4 a, b;
    if (T.lb4 && (l4 || proto == 1) && lb4_service(T, da, kd, 0, a, b)) {
        const uint32_t hash = A.hash ? A.hash[i] : flow_hash4(sa, da, pt, proto);
        // lb4_local: ct_lookup4(CT_SERVICE) — the tuple as loaded, one probe
        uint32_t slave, loop = 0;
        const uint32_t ov = A.svo ? A.svo[i] : 0u;
        if (ov & SVO_SET) {   // the entry as an earlier header of the batch left it
            slave = ov & 0xFFFF;
            loop = (ov & SVO_LOOP) ? 1u : 0u;
        } else {
            const CtProbe k = ct_probe<false>(proto, pt, CT_SERVICE, A.ct_owner);
            const uint32_t slot = ct4_find(T, da, sa, k.z1, k.w1);
            if (slot != NONE && T.ct4_lb) {   // the entry's ct_state (conntrack.h:235-239)
                const uint4 lw = ld16(T.ct4_lb + slot);
                slave = lw.y;
                loop = (lw.x >> 16) & 1;
            } else {
                slave = slot != NONE ? 0u : hash % (a.w >> 16) + 1;   // lb4_select_slave
            }
        }
        uint4 c, d;
        bool ok = lb4_get(T, da, kd, slave, c, d);   // lb4_lookup_slave
        if (!ok)   // the fall-back: the key as it stands, slave set
            ok = lb4_service(T, da, kd, slave, c, d);
        if (!ok) {
            fl = LBF_DROP;
        } else {
            const uint32_t target = c.z, port = c.w & 0xFFFF;
            fl = LBF_SVC | (d.x & 0xFFFF) << 16;
            if (sa == target) {   // loopback (lb.h:753-767)
                loop = 1;
                psa = IPV4_LOOPBACK;
            }
            if (loop)
                fl |= LBF_LOOP;
            else
                tda = target;
            pda = target;
            if (port && kd != port && l4)   // lb4_xlate's L4 dport
                ppt = (ppt & 0xFFFFu) | port << 16;
            tpt = ppt;
        }
    }
    // a reply of a load-balanced flow: the sending endpoint's ct_lookup4 hit
    // (k1: CT_REPLY / CT_RELATED) on an entry with rev_nat_index
    if (!(fl & LBF_DROP) && T.ct4_lb && (l4 || proto == 1)) {
        const CtProbe k = ct_probe<false>(proto, tpt, CT_EGRESS, A.ct_owner);
        const uint32_t slot = ct4_find(T, tda, sa, k.z1, k.w1);
        if (slot != NONE)
            lb4_rev_nat(T, ld16(T.ct4_lb + slot), proto, psa, pda, ppt);
    }
    A.tda[i] = tda;
    A.tpt[i] = tpt;
    A.psa[i] = psa;
    A.pda[i] = pda;
    A.ppt[i] = ppt;
    A.fl[i] = fl;
}

}  // namespace

int launch_lb4_egress(const DevTables &T, const LbArgs &A, hipStream_t s)
{
    if (!A.n)
        return 0;
    hipLaunchKernelGGL(k_lb4_egress, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, s,
                       T, A);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace cfc
