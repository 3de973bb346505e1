"""The CPU restatement (oracle/cfc_oracle.c) against the golden vectors the
reference's own BPF programs produced (oracle/gen_golden.py).  This pins the
oracle; the GPU parity tests then compare the HIP engine with it."""
import numpy as np
import pytest

import golden_io as G
import oracle as O

NAMES = G.names()


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
