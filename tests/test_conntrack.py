"""Conntrack on the CPU side: the C5 generator's CT entries are what
ct_create4 writes (checked by running the pinned oracle over the flows'
opening packets), the oracle's batch hazards, and the CT byte layout."""
import numpy as np

import oracle as O
from cilium_amd import synth as S


def test_c5_generator_matches_ct_create():
    """Flows opened from outside: classify their first packet with empty CT
    maps and fold the batch — the oracle's CT maps then hold exactly the
    generator's entries for those flows (tuple, counters, src_sec_id,
    ICMP related entry)."""
    t, flows = S.config_c5(7, n_flows=4000, n_prefixes=2000, n_policy=400)
    ct_gen = t.ct
    t.ct = None
    # one L3 allow entry per source identity, so every opening packet creates
    o0 = O.Oracle(t)
    _, _, ide = o0.classify(flows, 0, 0)
    ids = np.unique(ide)
    pol = np.zeros(len(ids), S.POLICY_DT)
    pol["identity"] = ids
    t.policy = {S.EP_LXC_ID: pol}
    o = O.Oracle(t)
    o.ct_add(np.zeros(0, S.CT_DT))
    # inbound flows only: their forward packet (r -> c) is the opening one
    inbound = (ct_gen["tuple"][:, 13] & 1) == 1
    want = ct_gen[inbound & (ct_gen["tuple"][:, 12] != S.IPPROTO_ICMP)]
    # rebuild the opening packets from the generator's k2 = {r, c, dport, sport}
    n = len(want)
    tu = want["tuple"]
    r = tu[:, 0:4].copy().view("<u4").ravel()
    c = tu[:, 4:8].copy().view("<u4").ravel()
    dport = tu[:, 8:10].copy().view("<u2").ravel()
    sport = tu[:, 10:12].copy().view("<u2").ravel()
    ent = want["entry"].view("<u8")[:, :4]
    h = S.Headers(4, r, c, sport, dport, tu[:, 12].copy(), np.zeros(n, np.uint8),
                  ent[:, 1].astype(np.uint16), np.zeros(n, np.uint32))
    act, ver, ide, ct = o.classify(h, 0, 0, want_ct=True, apply_ct=True)
    assert (ver == 0).all(), np.unique(ver)
    assert ((ct & 0xF) == (0 | 4 | 8)).all()    # CT_NEW, looked up, created
    rows = o.ct_dump()
    got = S.ct_from_rows(rows)
    flow_rows = got[got["tuple"][:, 12] != S.IPPROTO_ICMP]
    key = lambda a: {bytes(x["tuple"][:14]): bytes(x["entry"]) for x in a}  # noqa: E731
    gk, wk = key(flow_rows), key(want)
    assert set(gk) == set(wk)
    for k, v in wk.items():
        e_got = np.frombuffer(gk[k], np.uint8).copy()
        e_want = np.frombuffer(v, np.uint8).copy()
        e_got[44:48] = e_want[44:48] = 0      # src_sec_id: generator picks ids
        np.testing.assert_array_equal(e_got, e_want)


def test_hazards_flag_hit_after_delete():
    """An established flow the policy now denies is deleted by its first
    packet; its second packet in the same batch is a hazard (the reference
    sees CT_NEW, the batch CT_ESTABLISHED — same verdict, different CT
    writes)."""
    t = S.config_c2(3, n_prefixes=500, n_policy=50)
    t.policy = {S.EP_LXC_ID: np.zeros(0, S.POLICY_DT)}
    rem = S.ip4("8.8.8.8")
    h = S.Headers(4, np.array([rem, rem], np.uint32),
                  np.array([S.LXC_IPV4] * 2, np.uint32),
                  np.array([S.htons(40000)] * 2, np.uint16),
                  np.array([S.htons(80)] * 2, np.uint16),
                  np.array([6, 6], np.uint8), np.zeros(2, np.uint8),
                  np.array([100, 120], np.uint16), np.zeros(2, np.uint32))
    # the flow as ct_create4 stored it when it was opened from outside
    t.ct = S.ct_entries_v4(np.array([S.byteswap32(np.uint32(rem))]),
                           np.array([S.byteswap32(np.uint32(S.LXC_IPV4))]),
                           h.dport[:1], h.sport[:1], np.array([6], np.uint8),
                           np.array([1], np.uint8), np.array([True]),
                           np.array([60], np.uint64), np.array([300], np.uint32))
    o = O.Oracle(t)
    act, ver, ide, ct = o.classify(h, 0, 0, want_ct=True)
    assert list(ver) == [-133, -133] and list(ct & 7) == [5, 5]   # EST, denied
    hz = o.ct_apply(h, 0, 0, ide, ver, ct, hazard=True)
    assert list(hz) == [0, 1]
    rows = S.ct_from_rows(o.ct_dump())
    assert not (rows["tuple"][:, 12] == 6).any()      # ct_delete4


def test_new_flow_twice_in_one_batch():
    """A new flow seen twice in one batch is created once and counted on its
    second packet, as the reference's per-packet CT would."""
    t = S.config_c2(3, n_prefixes=500, n_policy=50)
    pol = np.zeros(1, S.POLICY_DT)
    pol["identity"] = 0
    pol["dport"] = S.htons(80)
    pol["proto"] = S.IPPROTO_TCP
    t.policy = {S.EP_LXC_ID: pol}
    t.ct = np.zeros(0, S.CT_DT)
    rem = S.ip4("8.8.8.8")
    fwd = S.Headers(4, np.array([rem], np.uint32), np.array([S.LXC_IPV4], np.uint32),
                    np.array([S.htons(40000)], np.uint16),
                    np.array([S.htons(80)], np.uint16), np.array([6], np.uint8),
                    np.zeros(1, np.uint8), np.array([100], np.uint16),
                    np.zeros(1, np.uint32))
    h = S.concat([fwd, fwd, S.reverse(fwd)])
    o = O.Oracle(t)
    act, ver, ide, ct = o.classify(h, 0, 0, want_ct=True)
    # the second packet of the new flow is benign: created once, counted
    hz = o.ct_apply(h, 0, 0, ide, ver, ct, hazard=True)
    assert list(hz[:2]) == [0, 0]
    rows = S.ct_from_rows(o.ct_dump())
    flow = rows[rows["tuple"][:, 12] == 6]
    assert len(flow) == 1
    pk = flow["entry"][0].view("<u8")
    assert pk[0] == 2 and pk[1] == 200      # rx: created + counted once more


def test_oracle_gc_filtering():
    """cfo_ct_gc restates doFiltering (pkg/maps/ctmap/ctmap.go:303-325):
    checked against the rule written out on the dump rows of a reference
    fixture's CT state — RemoveExpired (lifetime < Time), ValidIPs (neither
    address in the set), MatchIPs (either address in it), per-map
    selection."""
    import golden_io as G
    for name in ("ct_ingress_v4", "ct_egress_v6"):
        g = G.Golden(name)
        rows0 = O.Oracle(g.tables).ct_dump()
        al = 4 if rows0[0, 3] == 1 else 16
        life = rows0[:, 44 + 32:44 + 36].copy().view("<u4").ravel()
        da, sa = rows0[:, 4:4 + al], rows0[:, 4 + al:4 + 2 * al]
        t = int(np.median(life))
        o = O.Oracle(g.tables)
        assert o.ct_gc(time=t) == int((life < t).sum())
        np.testing.assert_array_equal(o.ct_dump(), rows0[life >= t])
        # MatchIPs: either address; ValidIPs: neither address
        pick = [bytes(x) for x in np.unique(da, axis=0)[:3]]
        inset = lambda a, s: np.array([bytes(x) in s for x in a])   # noqa: E731
        fam = 4 if al == 4 else 6
        o = O.Oracle(g.tables)
        o.ct_gc(remove_expired=False, match=[(fam, b) for b in pick])
        keep = ~(inset(da, pick) | inset(sa, pick))
        np.testing.assert_array_equal(o.ct_dump(), rows0[keep])
        o = O.Oracle(g.tables)
        o.ct_gc(remove_expired=False, valid=[(fam, b) for b in pick])
        keep = inset(da, pick) | inset(sa, pick)
        np.testing.assert_array_equal(o.ct_dump(), rows0[keep])
        # an empty ValidIPs set (the initial scan with no endpoint) clears all
        o = O.Oracle(g.tables)
        assert o.ct_gc(remove_expired=False, valid=[]) == len(rows0)
        # one map only: the TCP map of the first owner in the dump
        o = O.Oracle(g.tables)
        ow = int(rows0[0, 0]) | int(rows0[0, 1]) << 8
        sel = (rows0[:, 0].astype(int) | rows0[:, 1].astype(int) << 8) == ow
        sel &= rows0[:, 2] == 0
        o.ct_gc(time=0xFFFFFFFF, owner=ow, kind=0)
        np.testing.assert_array_equal(o.ct_dump(), rows0[~sel])
