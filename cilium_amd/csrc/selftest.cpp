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
                const auto mk = std::make_pair(plen, msk(a, plen));
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
    return fail;
}
