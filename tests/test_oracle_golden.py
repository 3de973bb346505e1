"""The CPU restatement (oracle/cfc_oracle.c) against the golden vectors the
reference's own BPF programs produced (oracle/gen_golden.py).  This pins the
oracle; the GPU parity tests then compare the HIP engine with it."""
import numpy as np
import pytest

import golden_io as G
import oracle as O
from cilium_amd import synth as S

# (the oracle-only fixtures too: tests/golden_oracle, golden_io.ORACLE_ONLY_DIR)
NAMES = G.names() + G.oracle_only_names()


def test_have_goldens():
    assert len(NAMES) >= 12, NAMES
    assert any(n.endswith("_v6") for n in NAMES)


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("threads", [1, 4])
def test_oracle_matches_reference(name, threads):
    g = G.Golden(name)
    o = O.Oracle(g.tables)
    act, ver, ide = o.classify(g.headers, g.mode, g.ep_lxc, nthreads=threads,
                               apply_ct=g.ct_after is not None)
    bad = G.mismatches(g, act, ver, ide)
    assert len(bad) == 0, f"{len(bad)} headers differ, first {bad[:10]}"
    for lxc, exp in g.counters.items():
        np.testing.assert_array_equal(o.policy_counters(lxc), exp)
    np.testing.assert_array_equal(o.metrics(), g.metrics)
    if g.ct_after is not None:
        # CT maps after the stream: same keys, same accounting, closing bits,
        # src_sec_id, rev_nat (clock-derived fields masked, golden_io)
        np.testing.assert_array_equal(G.ct_masked(o.ct_dump()),
                                      G.ct_masked(g.ct_after))


def test_goldens_cover_every_outcome():
    """The fixtures exercise every verdict the path can produce."""
    seen = set()
    for name in NAMES:
        g = G.Golden(name)
        seen |= {(int(a), int(v) if v <= 0 else 1)
                 for a, v in zip(g.action, g.verdict)}
    for want in [(7, 0), (7, 1), (0, 0), (2, -133), (2, -137), (2, -132),
                 (1, -1), (2, 0), (2, -156), (2, -157)]:
        assert want in seen, want


def test_ct_goldens_cover_every_ct_state():
    """The CT fixtures hit every lookup result in both directions, creates,
    deletes of denied established flows, and closing flows."""
    for name in [n for n in NAMES if n.startswith("ct_")]:
        g = G.Golden(name)
        o = O.Oracle(g.tables)
        act, ver, ide, ct = o.classify(g.headers, g.mode, g.ep_lxc,
                                       want_ct=True)
        res = ct[(ct & 4) != 0] & 3
        assert set(np.unique(res)) == {0, 1, 2, 3}, (name, np.unique(ct))
        assert (ct & 8).any(), name
        est_denied = ((ct & 0x7) == 5) & (ver == -133)
        est_denied |= ((ct & 0x70) == 0x50) & (ver == -133)
        assert est_denied.any(), name
        assert (g.headers.flags & 2).any(), name


NOTIFY_NAMES = [n for n in NAMES if G.Golden(n).cb is not None]


def test_drop_notify_goldens_present():
    assert len(NOTIFY_NAMES) >= 10, NOTIFY_NAMES


@pytest.mark.parametrize("name", NOTIFY_NAMES)
def test_oracle_drop_notify_matches_reference(name):
    """Every drop-notify record of the restatement carries the arguments the
    reference's send_drop_notify left in skb->cb[] for the same header."""
    g = G.Golden(name)
    o = O.Oracle(g.tables)
    # (in the reference's packet order when the fixture has CT state: a
    # stream may hold intra-batch CT dependencies)
    act, ver, ide, nt = o.classify(g.headers, g.mode, g.ep_lxc,
                                   want_notify=True, apply_ct=g.ct_after is not None)
    rec, idx = o.drop_notify(g.headers, g.mode, g.ep_lxc, ver, ide, nt)
    want_idx, want = G.expected_drop_notify(g)
    np.testing.assert_array_equal(idx, want_idx)
    # LXC_ID is compiled into each endpoint program (lxc_config.h); the
    # harness runs one bpf_lxc.o (LXC_ID 0x1010) behind every endpoint, so
    # its dst_id is 0x1010 where the engine (one program per endpoint, as
    # the agent compiles them) reports the destination's own id
    other = (rec["dst_id"] != 0) & (rec["dst_id"] != S.EP_LXC_ID)
    assert (want["dst_id"][other] == S.EP_LXC_ID).all()
    want["dst_id"] = np.where(other, rec["dst_id"], want["dst_id"])
    for k, v in want.items():
        np.testing.assert_array_equal(rec[k].astype(np.int64), v, err_msg=k)
    assert (rec["type"] == 1).all()
    np.testing.assert_array_equal(rec["len_cap"],
                                  np.minimum(rec["len_orig"], 128))
    if g.mode == O.MODE_EGRESS:
        assert ((rec["source"] == g.ep_lxc) | (rec["source"] == rec["dst_id"])).all()
    if len(rec) and g.mode != O.MODE_XDP:
        # records from both an endpoint program and (where present) netdev
        assert (rec["source"] != 0).any(), name


def test_oracle_node_config():
    """cfo_node_config: the reference's own values reproduce the golden
    (pinned above); another IPV4_CLUSTER_RANGE/MASK moves exactly the egress
    destinations inside it to CLUSTER_ID (bpf_lxc.c:521-529) and leaves every
    other output unchanged."""
    g = G.Golden("c2_egress_v4")
    o = O.Oracle(g.tables)
    o.node_config(0x100000, 0xFF0000, S.ROUTER_IPV6)
    a0, v0, i0 = o.classify(g.headers, g.mode, g.ep_lxc)
    assert len(G.mismatches(g, a0, v0, i0)) == 0
    o = O.Oracle(g.tables)
    o.node_config(0x0000000A, 0x000000FF, S.ROUTER_IPV6)
    a1, v1, i1 = o.classify(g.headers, g.mode, g.ep_lxc)
    d = np.asarray(g.headers.daddr, np.uint32)
    in_old = (d & 0xFF0000) == 0x100000
    in_new = (d & 0xFF) == 0x0A
    changed = i0 != i1
    assert changed.any()
    assert not (changed & ~(in_old | in_new)).any()
    assert (i1[changed & in_new] == S.CLUSTER_ID).all()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_identity_counters_consistent(name):
    """The per-identity forward/drop counters (cfc.h cfc_identity_counters)
    against what the reference's own outputs in the fixture imply: every
    DROP_POLICY of the batch's direction is one drop event, and (without
    conntrack) every forwarded ingress header that reached the endpoint's
    policy is a forward event — TRACE_TO_LXC's update_metrics(FORWARDED,
    INGRESS) plus the proxy redirects (bpf_lxc.c:985-1008)."""
    g = G.Golden(name)
    o = O.Oracle(g.tables)
    act, ver, ide = o.classify(g.headers, g.mode, g.ep_lxc,
                               apply_ct=g.ct_after is not None)
    rows = o.identity_counters()
    if g.mode == O.MODE_XDP:
        assert len(rows) == 0
        return
    met = {(int(r[0]), int(r[1])): int(r[2]) for r in g.metrics}
    drops = {d: int(rows[rows[:, 1] == d][:, 4].sum()) for d in (1, 2)}
    fwd = {d: int(rows[rows[:, 1] == d][:, 2].sum()) for d in (1, 2)}
    if g.mode == O.MODE_EGRESS:
        assert drops[2] == met.get((133, 2), 0)
        assert drops[1] == met.get((133, 1), 0)
    else:
        assert drops[1] == met.get((133, 1), 0)
        assert drops[2] == fwd[2] == 0
        if g.ct_after is None:
            redirects = int(((act == 7) & (ver > 0)).sum())
            assert fwd[1] == met.get((0, 1), 0) + redirects
    # identities are the verdict's: every drop row's identity dropped a header
    v = np.asarray(ver)
    dropped = set(int(x) for x in np.asarray(ide)[v == -133])
    for r in rows[rows[:, 4] > 0]:
        if g.mode != O.MODE_EGRESS or r[1] == 2:
            assert int(r[0]) in dropped or int(r[0]) == 0xFFFFFFFF


def _events_oracle(g):
    """the reference's semantics: one header at a time, CT folded after
    each, at the clock each header ran at"""
    o = O.Oracle(g.tables)
    # a header whose run straddled a second boundary ran at the next
    # header's second or the one before: take the next header's (it is not
    # compared itself)
    clock = g.clock.astype(np.int64)
    for i in range(len(clock) - 1, -1, -1):
        if clock[i] == 0xFFFFFFFF:
            clock[i] = clock[i + 1] if i + 1 < len(clock) else clock[i - 1] + 1
    act, ver, ide, words = o.run_sequential(g.headers, g.mode, g.ep_lxc, clock)
    assert len(G.mismatches(g, act, ver, ide)) == 0
    if g.ct_after is not None:
        # run packet by packet at the reference's clock, the CT maps end up
        # byte-identical to the reference's — lifetimes, report times, seen
        # TCP flags and seen_non_syn included (conntrack.h:125-285, 615-772)
        np.testing.assert_array_equal(o.ct_dump(), g.ct_after)
    return o.events(g.headers, g.mode, g.ep_lxc, ver, ide, words)


def _events_pinned(g):
    return g.ev is not None and g.clock is not None


@pytest.mark.parametrize("name", NAMES)
def test_oracle_events_match_reference(name):
    """Every perf-ring sample the reference's programs emitted on
    cilium_events while the fixture ran — trace_notify at each observation
    point (TO_LXC, TO_PROXY, TO_HOST, TO_STACK; trace.h:97-155 with
    MONITOR_AGGREGATION 5) and drop_notify (drop.h:50-78) — against the
    oracle's records for the same headers, field by field.  The flow hash
    (get_hash_recalc: the kernel's skb hash under a boot-time random key) is
    the one field no restatement can reproduce; it is left out."""
    g = G.Golden(name)
    if not _events_pinned(g):
        pytest.skip("fixture without perf-ring samples / clock")
    rec, idx = _events_oracle(g)
    # a header whose run straddled a second boundary has no exact clock
    amb = set(np.flatnonzero(g.clock == 0xFFFFFFFF).tolist())
    if amb:
        keep = ~np.isin(idx, list(amb))
        rec, idx = rec[keep], idx[keep]
        keep = ~np.isin(g.ev_hdr, list(amb))
        g.ev, g.ev_hdr = g.ev[keep], g.ev_hdr[keep]
    np.testing.assert_array_equal(idx.astype(np.uint32), g.ev_hdr)
    # LXC_ID is compiled into each endpoint program (lxc_config.h); the
    # harness runs one bpf_lxc.o (LXC_ID 0x1010) behind every endpoint, so
    # its records carry 0x1010 as EVENT_SOURCE and dst_id where the engine
    # (one program per endpoint, as the agent compiles them) reports the
    # endpoint's own id
    rec = rec.copy()
    other = (rec["source"] != 0) & (rec["source"] != S.EP_LXC_ID)
    has_id = other & (((rec["type"] == 1) & (rec["w6"] != 0)) |
                      ((rec["type"] == 4) & (rec["subtype"] == O.TRACE_TO_LXC)))
    rec["w6"][has_id] = (rec["w6"][has_id] & ~np.uint32(0xFFFF)) | S.EP_LXC_ID
    rec["source"][other] = S.EP_LXC_ID
    for f in O.EVENT_DT.names:
        if f == "hash":
            continue
        bad = np.nonzero(rec[f] != g.ev[f])[0]
        assert len(bad) == 0, (f"{f}: {len(bad)} of {len(rec)} differ; first at "
                               f"header {g.ev_hdr[bad[0]]}: oracle {rec[bad[0]]} "
                               f"reference {g.ev[bad[0]]}")


def test_events_pin_identities():
    """With the trace records the fixtures pin the full 32-bit identity of
    every forwarded header the reference reports: ingress headers delivered
    to an endpoint (TRACE_TO_LXC src_label, or the proxy map entry of a
    redirect) and egress headers sent to the stack (TRACE_TO_STACK
    dst_label).  Forwarded headers it never reports — ingress to the stack
    (bpf_netdev has no TRACE_NOTIFY), repeats inside the 5 s report interval
    of an active flow — are pinned by the kernel's LPM instead
    (test_lpm_identities_pin_every_tc_header)."""
    for name in G.names():
        g = G.Golden(name)
        if g.ev is None or g.mode == O.MODE_XDP:
            continue
        ev = g.ev
        obs = (O.TRACE_TO_STACK if g.mode == O.MODE_EGRESS else O.TRACE_TO_LXC)
        reported = g.ev_hdr[(ev["type"] == 4) & (ev["subtype"] == obs)]
        assert (g.idmask_reported[reported] == 0xFFFFFFFF).all(), name
        if g.mode != O.MODE_EGRESS:   # proxy redirects: the proxy map
            prox = (g.action == 7) & (g.verdict > 0)
            assert (g.idmask_reported[prox] == 0xFFFFFFFF).all(), name


LPM_NAMES = [n for n in NAMES if G.Golden(n).lpm is not None]


def test_every_fixture_has_kernel_lpm():
    assert LPM_NAMES == NAMES


@pytest.mark.parametrize("name", LPM_NAMES)
def test_oracle_lpm_matches_kernel(name):
    """ipcache_lookup4/6 of the restatement against the kernel's own LPM
    trie (BPF_MAP_LOOKUP_ELEM on cilium_ipcache, oracle/pin_lpm.py) for
    every address of every header: label and hit, 100%."""
    g = G.Golden(name)
    o = O.Oracle(g.tables)
    h = g.headers
    cols = [h.saddr, h.daddr] + ([h.saddr, h.daddr] if g.pkt is None else list(g.pkt_addrs()))
    for c, a in enumerate(cols):
        lab, hit = o.ipcache_lookup(h.family, a)
        np.testing.assert_array_equal(hit, g.lpm_hit[:, c], err_msg=f"hit, column {c}")
        np.testing.assert_array_equal(lab, g.lpm[:, c], err_msg=f"label, column {c}")


@pytest.mark.parametrize("name", LPM_NAMES)
def test_lpm_identities_pin_every_tc_header(name):
    """The identities derived from the kernel's LPM (golden_io.lpm_identity)
    agree with every identity bit the reference reported itself (trace
    records, drop cb[1], proxy map), and together they pin the full 32-bit
    identity of every tc-path header whose program reached the ipcache
    lookup — forwarded headers the reference never reports included."""
    g = G.Golden(name)
    m = g.idmask_reported
    both = g.lpm_applies & (m != 0)
    np.testing.assert_array_equal(g.lpm_expected[both] & m[both],
                                  g.identity_reported[both] & m[both])
    tc = g.mode != 2
    if g.mode == 3:
        tc = ~((g.action == 1) & (g.verdict == -1))
    reached = tc & ~G.no_identity(g)
    assert (g.idmask[reached] == 0xFFFFFFFF).all()
    unreported = reached & (m != 0xFFFFFFFF)
    if g.mode != 2 and len(g.verdict) > 100:
        assert unreported.any(), "the LPM pins headers the reference never reports"


LB_NAMES = [n for n in NAMES if G.Golden(n).pkt is not None]


def test_lb_goldens_cover_the_service_path():
    """The load-balancing fixtures exercise the service translation, the
    loopback case, DROP_NO_SERVICE, and reverse NAT in both directions."""
    assert {"lb_egress_v4", "lb_reply_v4"} <= set(LB_NAMES)
    g = G.Golden("lb_egress_v4")
    vips = set(int(x) for x in g.tables.lb4["addr"])
    assert (g.pkt[:, 1] != g.headers.daddr).sum() > 1000        # translated
    assert (g.pkt[:, 0] == S.IPV4_LOOPBACK).any()               # loopback
    assert (g.verdict == -158).any()                            # no backend
    assert any(int(x) in vips for x in g.pkt[:, 0])             # egress rev NAT
    r = G.Golden("lb_reply_v4")
    assert sum(int(x) in vips for x in r.pkt[:, 0]) > 1000      # ingress rev NAT
    # IPv6 (lb6_local has no loopback case)
    assert {"lb_egress_v6", "lb_reply_v6"} <= set(LB_NAMES)
    g = G.Golden("lb_egress_v6")
    vips6 = {bytes(a) for a in g.tables.lb6["addr"]}
    psa, pda = g.pkt_addrs()
    assert (pda != g.headers.daddr).any(1).sum() > 1000           # translated
    assert (g.verdict == -158).any()                              # no backend
    assert any(bytes(a) in vips6 for a in psa)                    # egress rev NAT
    r = G.Golden("lb_reply_v6")
    assert sum(bytes(a) in vips6 for a in r.pkt_addrs()[0]) > 1000   # ingress rev NAT


@pytest.mark.parametrize("name", LB_NAMES)
def test_oracle_packets_match_reference(name):
    """The packet each program left (service translation lb4_xlate, reverse
    NAT lb4_rev_nat: addresses and L4 ports) against the reference's output
    packet, for every header that was not dropped or handed to a proxy (a
    proxy redirect's port is the verdict itself).  skb->hash comes from the
    reference's records, so backend selection is the reference's."""
    g = G.Golden(name)
    o = O.Oracle(g.tables)
    act, ver, ide, pkt = o.classify(g.headers, g.mode, g.ep_lxc, want_pkt=True,
                                    apply_ct=g.ct_after is not None)
    keep = (g.action != 2) & ~((g.action == 7) & (g.verdict > 0))
    np.testing.assert_array_equal(pkt[keep], g.pkt[keep])


@pytest.mark.parametrize("name", LB_NAMES)
def test_record_hash_is_the_batch_hash(name):
    """With skb->hash in the batch, every record carries it (the one field
    test_oracle_events_match_reference leaves out otherwise)."""
    g = G.Golden(name)
    o = O.Oracle(g.tables)
    act, ver, ide, words = o.classify(g.headers, g.mode, g.ep_lxc, want_notify=True,
                                      apply_ct=g.ct_after is not None)
    rec, idx = o.events(g.headers, g.mode, g.ep_lxc, ver, ide, words)
    first = {}
    for j, i in enumerate(g.ev_hdr):
        first.setdefault(int(i), int(g.ev["hash"][j]))
    got = {int(i): int(h) for i, h in zip(idx, rec["hash"])}
    common = set(first) & set(got)
    assert len(common) > 1000
    assert all(first[i] == got[i] for i in common)
