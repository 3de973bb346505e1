// Host self-test of the IPv6 LPM flattener (flatten.cpp build_lpm6): the
// lookup the device performs (lpm6_lookup_host restates k_classify_v6's
// lpm6_lookup over the same image) against a brute-force longest-prefix
// match, on prefix sets that exercise the Bloom grouping: random C3-like
// sets, prefixes piled under one /48 or /64 (groups must split), a ::/0,
// and label-0 prefixes that shadow shorter ones.  No GPU needed.
#include <cstdio>
#include <cerrno>
#include <cstring>
#include <map>
#include <random>
#include <vector>

#include "flatten.hpp"
#include "maps.hpp"
#include "selfcut.hpp"

using namespace cfc;

// the cut rule of an egress batch with traffic to itself (selfcut.hpp)
struct Row {
    uint32_t x, y, z, w;   // header index, L4 word, meta, address matched
};
static uint32_t ports(uint32_t sp, uint32_t dp) { return sp | dp << 16; }
static int cuts_case(const char *name, const std::vector<Row> &rows, bool v6,
                     const std::vector<uint64_t> &want)
{
    std::vector<uint64_t> got;
    self_cut_rule(rows, 1, v6, &got);   // (address 0 the endpoint's own, 1 a loopback one)
    const bool ok = got == want;
    printf("selfcut %-24s %s (%zu cuts)\n", name, ok ? "ok" : "FAIL", got.size());
    return ok ? 0 : 1;
}
static int selfcut_tests()
{
    const uint32_t TCP = 6, UDP = 17, ICMP = 1, ICMP6 = 58;
    int fail = 0;
    // an opening packet and its answer (ports swapped): cut at the answer
    fail |= cuts_case("tcp-answer", {{3, ports(1000, 80), TCP, 0}, {9, ports(80, 1000), TCP, 0}},
                      false, {9});
    // a second packet of the same direction: also cut (conservative)
    fail |= cuts_case("tcp-same-dir", {{3, ports(1000, 80), TCP, 0}, {5, ports(1000, 80), TCP, 0}},
                      false, {5});
    // two flows on other ports, or another protocol: one segment
    fail |= cuts_case("tcp-unrelated", {{3, ports(1000, 80), TCP, 0}, {4, ports(1001, 80), TCP, 0},
                                        {6, ports(80, 1000), UDP, 0}}, false, {});
    // an ICMP error after anything: cut; echo after echo: cut; TCP after echo: none
    fail |= cuts_case("icmp-error", {{1, ports(1000, 80), TCP, 0}, {2, 3, ICMP, 0}}, false, {2});
    fail |= cuts_case("icmp-echo", {{1, 8, ICMP, 0}, {2, ports(1000, 80), TCP, 0}, {7, 0, ICMP, 0}},
                      false, {7});
    fail |= cuts_case("icmp6-error", {{1, ports(1000, 80), UDP, 0}, {2, 1, ICMP6, 0}}, true, {2});
    // (IPv4 type 1 is no error: an ICMPv4 "other" after a TCP flow, none)
    fail |= cuts_case("icmp4-type1", {{1, ports(1000, 80), TCP, 0}, {2, 1, ICMP, 0}}, false, {});
    // a loopback address on either side: cut
    fail |= cuts_case("loopback", {{1, ports(1000, 80), TCP, 1}, {2, ports(2000, 90), TCP, 0},
                                   {3, ports(3000, 90), TCP, 1}}, false, {2, 3});
    // a cut starts a new segment: a key of the segment before no longer counts
    fail |= cuts_case("reset", {{1, ports(1000, 80), TCP, 0}, {2, ports(80, 1000), TCP, 0},
                                {3, ports(2000, 80), TCP, 0}, {4, ports(1000, 80), TCP, 0}},
                      false, {2, 4});
    fail |= cuts_case("one-header", {{5, ports(1000, 80), TCP, 0}}, false, {});
    return fail;
}

static uint32_t brute(const std::vector<Pfx6> &pfx, const uint32_t w[4])
{
    int best = -1;
    uint32_t label = 0;
    for (const Pfx6 &p : pfx) {
        bool ok = true;
        for (int i = 0; i < 4 && ok; i++)
            ok = (w[i] & l6_word_mask(p.plen, i)) == p.w[i];
        if (ok && (int)p.plen > best) {
            best = p.plen;
            label = p.label;
        }
    }
    return label;
}

static void add(std::vector<Pfx6> &v, const uint32_t a[4], int len, uint32_t label)
{
    Pfx6 p;
    p.plen = (uint8_t)len;
    p.label = label;
    for (int i = 0; i < 4; i++)
        p.w[i] = a[i] & l6_word_mask(len, i);
    for (const Pfx6 &q : v)
        if (q.plen == p.plen && !memcmp(q.w, p.w, 16))
            return;   // unique (prefix, length) like the map
    v.push_back(p);
}

template <class R>
static int run(const char *name, const std::vector<Pfx6> &pfx, R &rng,
               int queries)
{
    Lpm6Host t;
    build_lpm6(pfx, &t);
    int bad = 0;
    for (int q = 0; q < queries; q++) {
        uint32_t w[4];
        for (int i = 0; i < 4; i++)
            w[i] = rng();
        if (!pfx.empty() && (q & 3)) {   // mostly inside some prefix
            const Pfx6 &p = pfx[rng() % pfx.size()];
            for (int i = 0; i < 4; i++)
                w[i] = p.w[i] | (w[i] & ~l6_word_mask(p.plen, i));
        }
        const uint32_t a = lpm6_lookup_host(t, w), b = brute(pfx, w);
        if (a != b && bad++ < 5)
            printf("%s: %08x:%08x:%08x:%08x -> %u, want %u\n", name, w[0], w[1],
                   w[2], w[3], a, b);
    }
    printf("%-12s prefixes %5zu lengths %3zu groups %3u bloom %6zu slots %6zu: %s\n",
           name, pfx.size(), t.lens.size(), t.groups, t.bloom.size(), t.slots.size(),
           bad ? "FAIL" : "ok");
    return bad != 0;
}

// test/bpf/unit-test.c test_ipv6_addr_clear_suffix: the words an all-ones
// address keeps under a prefix length (ipv6_addr_clear_suffix, ipv6.h:136-150),
// here as l6_word_mask (layout.h), which builds and probes the IPv6 LPM
static int clear_suffix_kats()
{
    struct { uint32_t len, w[4]; } k[] = {
        {128, {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}},
        {127, {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu}},
        {95, {0xffffffffu, 0xffffffffu, 0xfffffffeu, 0}},
        {1, {0x80000000u, 0, 0, 0}},
        {0, {0, 0, 0, 0}},   // (the reference's -1 case: no prefix bits)
    };
    int bad = 0;
    for (const auto &c : k)
        for (int i = 0; i < 4; i++)
            bad += l6_word_mask(c.len, i) != c.w[i];
    printf("clear_suffix kats: %s\n", bad ? "FAIL" : "ok");
    return bad != 0;
}

// the IPv4 LPM builders (flatten.cpp build_dir24_8, build_l4trie) through
// host restatements of the device lookups (classify.hip's DIR-24-8 probe,
// kern_common.hpp l4_lookup) against a brute-force longest-prefix match:
// random lengths, prefixes piled under one /16 (lists, then chunk splits),
// a /0, labels past a list entry's 26 bits (lbl_ovf)
static uint32_t dir24_lookup_host(const std::vector<uint32_t> &t24,
                                  const std::vector<uint32_t> &t8, uint32_t a)
{
    uint32_t e = t24[a >> 8];
    if (e & LPM_GROUP)
        e = t8[((size_t)(e & ~LPM_GROUP) << 8) | (a & 255)];
    return e;
}
static uint32_t l4_lookup_host(const std::vector<uint32_t> &d, const std::vector<uint32_t> &c,
                               const std::vector<uint64_t> &l, const std::vector<uint32_t> &ovf,
                               uint32_t a)
{
    auto list_leaf = [&](uint32_t hi) {
        const uint32_t x = hi & (LL_INDIRECT | LL_PAYLOAD);
        return (x & LL_INDIRECT) ? ovf[x & LL_PAYLOAD] : x;
    };
    const uint32_t *D = &d[4 * (a >> 16)];
    const uint32_t e1 = (D[2] >> 16) | (D[3] << 16);
    if (l4_inline_match(a, D[1]))
        return list_leaf((D[1] >> 21) | (D[2] << 11));
    if (l4_inline_match(a, e1))
        return list_leaf(D[3] >> 5);
    uint32_t e = D[0], shift = 16;
    while (e & L4_PTR) {
        const uint32_t cnt = (e >> 24) & 127, off = e & L4_OFF;
        if (cnt == 0) {
            shift -= 8;
            e = c[off + ((a >> shift) & 255)];
            continue;
        }
        for (uint32_t i = 0; i < cnt; i += 2) {
            const uint64_t u = l[off + i], v = l[off + i + 1];
            const bool m0 = l4_match(a, (uint32_t)u, (uint32_t)(u >> 32));
            if (m0 || l4_match(a, (uint32_t)v, (uint32_t)(v >> 32)))
                return list_leaf(m0 ? (uint32_t)(u >> 32) : (uint32_t)(v >> 32));
        }
        return 0;
    }
    return (e & LPM_INDIRECT) ? ovf[e & LPM_PAYLOAD] : e;
}
static int lpm4_case(const char *name, std::vector<Pfx4> pfx, std::mt19937 &gen, int nq)
{
    {   // one prefix per (masked address, length), as the ipcache map holds
        std::map<std::pair<uint32_t, int>, Pfx4> u;
        for (Pfx4 p : pfx) {
            p.addr &= p.plen ? 0xFFFFFFFFu << (32 - p.plen) : 0u;
            u.emplace(std::make_pair(p.addr, (int)p.plen), p);
        }
        pfx.clear();
        for (auto &kv : u)
            pfx.push_back(kv.second);
    }
    std::vector<uint32_t> t24, t8, ovf, d, c;
    std::vector<uint64_t> l;
    build_dir24_8(pfx, &t24, &t8);
    const bool ok = build_l4trie(pfx, &ovf, &d, &c, &l);
    int bad = !ok;
    for (int q = 0; q < nq; q++) {
        uint32_t a = gen();
        if (!pfx.empty() && (q & 3)) {   // mostly inside some prefix
            const Pfx4 &p = pfx[gen() % pfx.size()];
            const uint32_t m = p.plen ? 0xFFFFFFFFu << (32 - p.plen) : 0u;
            a = p.addr | (a & ~m);
        }
        uint32_t want = 0;
        int best = -1;
        for (const Pfx4 &p : pfx) {
            const uint32_t m = p.plen ? 0xFFFFFFFFu << (32 - p.plen) : 0u;
            if ((int)p.plen > best && (a & m) == p.addr)
                best = p.plen, want = p.leaf;
        }
        const uint32_t x = dir24_lookup_host(t24, t8, a), y = l4_lookup_host(d, c, l, ovf, a);
        if ((x != want || y != want) && bad++ < 5)
            printf("%s: %08x -> dir24 %u, trie %u, want %u\n", name, a, x, y, want);
    }
    printf("lpm4 %-14s prefixes %5zu chunks %5zu list %6zu: %s\n", name, pfx.size(),
           c.size() / 256, l.size(), bad ? "FAIL" : "ok");
    return bad != 0;
}
static int lpm4_tests(std::mt19937 &gen)
{
    int fail = 0;
    std::vector<Pfx4> v;
    for (int i = 0; i < 4000; i++)   // random lengths, some wide labels
        v.push_back({(uint32_t)gen(), (uint8_t)(gen() % 33),
                     (i % 9) ? 1 + (uint32_t)(gen() % 100000) : (1u << 27) + i});
    fail |= lpm4_case("random", v, gen, 40000);
    v.clear();   // piled under 10.20.0.0/16: lists, then chunks, then deeper
    for (int i = 0; i < 3000; i++)
        v.push_back({0x0A140000u | (uint32_t)(gen() & 0xFFFF), (uint8_t)(17 + gen() % 16),
                     1 + (uint32_t)i});
    v.push_back({0x0A140000u, 16, 77});
    v.push_back({0, 0, 5});
    fail |= lpm4_case("piled", v, gen, 40000);
    v.clear();   // piled under one /24 too: a second chunk level
    for (int i = 0; i < 600; i++)
        v.push_back({0x0A141E00u | (uint32_t)(gen() & 0xFF), (uint8_t)(25 + gen() % 8),
                     1 + (uint32_t)i});
    for (int i = 0; i < 40; i++)
        v.push_back({0x0A140000u | (uint32_t)(gen() & 0xFFFF), (uint8_t)(17 + gen() % 16),
                     (1u << 26) + (uint32_t)i});
    fail |= lpm4_case("deep", v, gen, 40000);
    for (int n : {1, 2, 3, 15, 16, 17}) {   // around the inline and list limits
        v.clear();
        for (int i = 0; i < n; i++)
            v.push_back({0xC0A80000u | (uint32_t)(gen() & 0xFFFF), (uint8_t)(17 + gen() % 16),
                         100 + (uint32_t)i});
        char nm[32];
        snprintf(nm, sizeof nm, "small-%d", n);
        fail |= lpm4_case(nm, v, gen, 5000);
    }
    return fail;
}

// the host map store (maps.cpp) against a plain model under random
// operations: a HASH (hashtab.c: -EEXIST / -ENOENT by flag, -E2BIG when
// full, get_next_key visits every key once) and an LPM_TRIE (lpm_trie.c:
// longest stored prefix no longer than the key's, data past the prefix
// ignored, -ENOSPC when full, -EINVAL past 32 bits)
static int map_fuzz(std::mt19937 &gen)
{
    int bad = 0;
    {
        Map m;
        m.type = MT_HASH, m.ksz = 8, m.vsz = 8, m.max_entries = 64;
        std::map<uint64_t, uint64_t> model;
        for (int it = 0; it < 200000; it++) {
            const uint64_t k = gen() % 96, v = gen();
            const int op = gen() % 4;
            if (op <= 1) {
                const uint64_t fl = gen() % 3;
                const bool has = model.count(k) != 0;
                const int want = fl == 1 && has ? -EEXIST : fl == 2 && !has ? -ENOENT
                                 : !has && model.size() >= 64 ? -E2BIG : 0;
                bad += m.update(&k, &v, fl) != want;
                if (!want)
                    model[k] = v;
            } else if (op == 2) {
                uint64_t got = 0;
                const int rc = m.lookup(&k, &got);
                bad += model.count(k) ? (rc != 0 || got != model[k]) : rc != -ENOENT;
            } else {
                bad += m.erase(&k) != (model.erase(k) ? 0 : -ENOENT);
            }
        }
        std::map<uint64_t, int> seen;   // a get_next_key walk from no key
        uint64_t cur = 0, nxt = 0;
        for (int rc = m.next_key(nullptr, &nxt); !rc; rc = m.next_key(&cur, &nxt))
            seen[cur = nxt]++;
        bad += seen.size() != model.size();
        for (auto &kv : seen)
            bad += kv.second != 1 || !model.count(kv.first);
    }
    {
        Map m;
        m.type = MT_LPM_TRIE, m.ksz = 8, m.vsz = 4, m.max_entries = 48;
        std::map<std::pair<uint32_t, uint32_t>, uint32_t> model;   // (plen, masked) -> v
        auto msk = [](uint32_t a, uint32_t p) { return p ? a & (0xFFFFFFFFu << (32 - p)) : 0u; };
        for (int it = 0; it < 100000; it++) {
            const uint32_t plen = gen() % 34, a = gen() & 0xFF0F00FFu, v = gen();
            uint8_t key[8];
            const uint32_t be = __builtin_bswap32(a);   // data in network order
            memcpy(key, &plen, 4);
            memcpy(key + 4, &be, 4);
            const int op = gen() % 3;
            if (op == 0) {
                const auto mk = std::make_pair(plen, plen <= 32 ? msk(a, plen) : 0u);
                const int want = plen > 32 ? -EINVAL
                                 : !model.count(mk) && model.size() >= 48 ? -ENOSPC : 0;
                bad += m.update(key, &v, 0) != want;
                if (!want)
                    model[mk] = v;
            } else if (op == 1) {
                uint32_t got = 0, want = 0;
                int best = -1;
                for (auto &e : model)
                    if ((int)e.first.first > best && e.first.first <= std::min(plen, 32u) &&
                        msk(a, e.first.first) == e.first.second)
                        best = (int)e.first.first, want = e.second;
                const int rc = m.lookup(key, &got);
                bad += best < 0 ? rc != -ENOENT : (rc != 0 || got != want);
            } else if (plen <= 32) {
                bad += m.erase(key) != (model.erase(std::make_pair(plen, msk(a, plen))) ? 0
                                                                                         : -ENOENT);
            }
        }
    }
    printf("map fuzz (hash, lpm): %s\n", bad ? "FAIL" : "ok");
    return bad != 0;
}

int main()
{
    std::mt19937 gen(12345);
    auto rng = [&gen]() -> uint32_t { return (uint32_t)gen(); };
    int fail = 0;
    {   // C3-like: /32../128, mass at /48 /56 /64 /128
        const int lens[] = {32, 40, 48, 48, 48, 56, 56, 64, 64, 64, 96, 128, 128};
        std::vector<Pfx6> v;
        for (int i = 0; i < 3000; i++) {
            uint32_t a[4] = {0x20000000u | (rng() & 0x0FFFFFFFu), rng(), rng(), rng()};
            add(v, a, lens[rng() % 13], 256 + i);
        }
        fail |= run("c3-like", v, rng, 20000);
    }
    {   // piled: pods (/128) under few /64s, /64s under one /48, a /0
        std::vector<Pfx6> v;
        uint32_t base[4] = {0x20010db8u, 0x00050000u, 0, 0};
        add(v, base, 48, 1000);
        for (int n = 0; n < 40; n++) {
            uint32_t a[4] = {base[0], base[1] | (rng() & 0xFFFF), rng(), rng()};
            add(v, a, 64, 2000 + n);
            for (int k = 0; k < 30; k++) {
                uint32_t b[4] = {a[0], a[1], rng(), rng()};
                add(v, b, 128, 5000 + 100 * n + k);
            }
        }
        uint32_t z[4] = {0, 0, 0, 0};
        add(v, z, 0, 7);
        fail |= run("piled", v, rng, 20000);
    }
    {   // every length 1..128, label 0 shadows, overlapping chains
        std::vector<Pfx6> v;
        uint32_t a[4] = {0x20010db8u, 0x12345678u, 0x9abcdef0u, 0x0fedcba9u};
        for (int len = 1; len <= 128; len++)
            add(v, a, len, (len % 7) ? 100 + len : 0);
        for (int i = 0; i < 500; i++) {
            uint32_t b[4] = {rng(), rng(), rng(), rng()};
            add(v, b, 1 + rng() % 128, (i % 5) ? 300 + i : 0);
        }
        fail |= run("all-lengths", v, rng, 20000);
    }
    {   // exact /128 set (the prefilter's fix map) and an empty table
        std::vector<Pfx6> v;
        for (int i = 0; i < 5000; i++) {
            uint32_t a[4] = {rng(), rng(), rng(), rng()};
            add(v, a, 128, 1);
        }
        fail |= run("exact128", v, rng, 20000);
        fail |= run("empty", std::vector<Pfx6>(), rng, 1000);
    }
    fail |= selfcut_tests();
    fail |= clear_suffix_kats();
    fail |= map_fuzz(gen);
    fail |= lpm4_tests(gen);
    return fail;
}
