"""A CT map at capacity stays on the device (CFC_OPT_CT_EVICT, cfc_api.cpp
ct_evict): per-endpoint CT maps of 4096 entries (CT_MAP_SIZE_TCP/ANY,
lxc_config.h:44-45) nearly full, then a batch with thousands of new flows.
The reference's LRU hash evicts least-recently-used entries as the inserts
come; the engine deletes, before the inserts, the map's entries closest to
expiry that the batch did not hit.  Checked: the apply stays
on the device, no map passes max_entries, every verdict and CT byte is the
oracle's (the batch's results do not depend on the evicted entries), every
surviving entry is byte-equal to the oracle's (which has no capacity), and
the evicted ones are exactly those with the earliest lifetimes that no
header of the batch hit.  Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import oracle as O
from cilium_amd import synth as S

pytestmark = pytest.mark.gpu
MODE_INGRESS = 0
CAP = 4096


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def full_tables(n_flows=2900, seed=5):
    t, flows = S.config_c5(seed, n_flows=n_flows, n_prefixes=5000, n_policy=500, now=1000)
    rng = np.random.default_rng(seed + 3)
    ct = t.ct
    ct["lxc"] = S.EP_LXC_ID                       # the endpoint's own CT maps
    life = (1000 + rng.integers(30, 3000, size=len(ct))).astype(np.uint32)
    ct["entry"][:, 32:36] = life.view(np.uint8).reshape(-1, 4)
    t.ct = ct
    return t, flows


def load_capped(dp, t):
    from cilium_amd.loader import load_tables, open_ct_maps
    ct = t.ct
    t.ct = None
    pms = load_tables(dp, t, commit=False)
    t.ct = ct
    fds = open_ct_maps(dp, [-1, S.EP_LXC_ID], max_entries=CAP)
    for (fam, lxc, any_map), fd in fds.items():
        sel = ct[(ct["family"] == fam) & (ct["lxc"] == lxc) & (ct["any"] == any_map)]
        if len(sel):
            dp.update_batch(fd, np.ascontiguousarray(sel["tuple"][:, :14]),
                            np.ascontiguousarray(sel["entry"]))
    dp.ct_fds = fds
    dp.commit()
    return pms


def test_full_endpoint_map_stays_on_device(torch):
    from cilium_amd.datapath import Datapath, pack
    from cilium_amd.loader import ct_rows
    t, flows = full_tables()
    n_tcp = int(((t.ct["any"] == 0)).sum())
    assert CAP - 200 < n_tcp <= CAP, n_tcp          # the TCP map nearly full
    h = S.headers_c5(t, flows, 8000, seed=9, new_frac=0.1)
    dp = Datapath(0)
    load_capped(dp, t)
    dp.set_clock(1003)
    b = pack(h)
    out = dp.classify(b, MODE_INGRESS, 0, want_ct=True)
    dp.ct_apply(b, out, MODE_INGRESS, 0)
    torch.cuda.synchronize()
    ver = out.verdict.cpu().numpy()
    ctb = out.ct.cpu().numpy()
    dp.counters_sync()   # (the CT accounting into the maps)
    rows = ct_rows(dp, dp.ct_fds)
    st = dp.stats()
    sizes = {k: len(dp.dump(fd)[0]) for k, fd in dp.ct_fds.items()}
    dp.close()
    assert st["ct_apply_host"] == 0 and st["ct_apply_device"] == 1, st
    assert st["ct_evicted"] > 0, st
    assert all(v <= CAP for v in sizes.values()), sizes
    o = O.Oracle(t)
    o.set_clock(1003)
    before = o.ct_dump()
    _, over, _, _, oct_ = o.run_sequential(h, MODE_INGRESS, 0, want_ct=True)
    np.testing.assert_array_equal(ver, over)
    np.testing.assert_array_equal(ctb, oct_)
    want = o.ct_dump()
    key = lambda r: r[:44].tobytes()             # noqa: E731
    wmap = {key(r): r for r in want}
    for r in rows:                               # survivors: the oracle's bytes
        assert key(r) in wmap
        np.testing.assert_array_equal(r, wmap[key(r)])
    kept = {key(r) for r in rows}
    gone = [r for r in want if key(r) not in kept]
    assert 0 < len(gone) <= st["ct_evicted"], (len(gone), st)
    # the evicted: entries the batch did not touch (unchanged since before
    # it), with the map's earliest lifetimes
    life = lambda r: int(r[76:80].view("<u4")[0])  # noqa: E731  (ct_entry @32)
    untouched = {key(r) for r in before if key(r) in wmap and
                 np.array_equal(r, wmap[key(r)])}
    assert all(key(r) in untouched for r in gone)
    for m in (0, 1):   # per map (TCP, ANY): every evicted lifetime < every kept untouched one
        g = [life(r) for r in gone if r[2] == m]
        k = [life(r) for r in want if r[2] == m and key(r) in untouched and key(r) in kept]
        if g and k:
            assert max(g) < min(k), (m, max(g), min(k))
