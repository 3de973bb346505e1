// The cut rule of an egress batch with traffic to itself (cfc_api.cpp
// self_cuts; DESIGN.md §4 "Traffic to itself"), host-only so selftest.cpp
// can check it without a GPU.
//
// rows: the listed headers (k_self_mark, selfseg.hip) in header order, each
// {x: header index, y: L4 word, z: meta, w: which address it matched — the
// endpoint's own addresses first (w < n_own), then the loopback ones: a
// service with the endpoint as a backend, IPV4_LOOPBACK}.  Header j is cut
// from an earlier listed header i of its segment when i's writes may hold
// one of j's lookup keys (conntrack.h:487-494, 691-772): any pair that
// involves a loopback address (the translated ports are not in the
// header); an ICMP error (its RELATED key is every create's ICMP entry); an
// ICMP echo / other ICMP after an ICMP one; TCP / UDP after the same
// protocol on the same two ports, in either order.  cuts: the header index
// each later segment starts at, ascending.
#pragma once

#include <algorithm>
#include <cstdint>
#include <set>
#include <vector>

namespace cfc {

template <class Row>
void self_cut_rule(const std::vector<Row> &rows, uint32_t n_own, bool v6,
                   std::vector<uint64_t> *cuts)
{
    const uint32_t icmp = v6 ? 58 : 1;
    std::set<uint64_t> l4;           // (proto, unordered ports) in the segment
    bool any = false, svc = false, icmp_plain = false;
    for (const Row &r : rows) {
        const uint32_t proto = r.z & 0xFF, pt = r.y;
        const bool lo = r.w >= n_own;   // a service or IPV4_LOOPBACK
        const uint32_t type = pt & 0xFF;
        const bool is_icmp = proto == icmp;
        const bool err = is_icmp && (v6 ? (type >= 1 && type <= 4)
                                        : (type == 3 || type == 11 || type == 12));
        const uint64_t a = pt & 0xFFFF, b = pt >> 16;
        const uint64_t key = (uint64_t)proto << 32 | std::min(a, b) << 16 | std::max(a, b);
        const bool l4p = proto == 6 || proto == 17;
        bool dep = false;
        if (any) {
            if (lo || svc || err)
                dep = true;
            else if (is_icmp)
                dep = icmp_plain;
            else if (l4p)
                dep = l4.count(key) != 0;
        }
        if (dep) {
            cuts->push_back(r.x);
            l4.clear();
            svc = icmp_plain = false;
        }
        any = true;
        svc |= lo;
        icmp_plain |= is_icmp && !err;
        if (l4p)
            l4.insert(key);
    }
}

}  // namespace cfc
