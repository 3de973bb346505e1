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
    act, ver, ide = o.classify(g.headers, g.mode, g.ep_lxc, nthreads=threads)
    bad = G.mismatches(g, act, ver, ide)
    assert len(bad) == 0, f"{len(bad)} headers differ, first {bad[:10]}"
    for lxc, exp in g.counters.items():
        np.testing.assert_array_equal(o.policy_counters(lxc), exp)
    np.testing.assert_array_equal(o.metrics(), g.metrics)


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
