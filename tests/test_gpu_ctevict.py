"""CT maps at capacity stay on the device (CFC_OPT_CT_EVICT, cfc_api.cpp
ct_evict_maps), IPv4 and IPv6: per-endpoint CT maps of 4096 entries
(CT_MAP_SIZE_TCP/ANY, lxc_config.h:44-45) nearly full, the global maps
nearly full too but written by no header of the batch, then a batch with
hundreds of new flows.  The reference's LRU hash evicts least-recently-used
entries as the inserts come; the engine deletes, before the inserts, each
overflowing map's excess — the entries the batch did not hit with the
earliest last refresh (lifetime minus the timeout of the entry's state),
ties by key bytes.  Checked: the apply stays on the device,
no map passes max_entries, a map the batch does not write loses nothing,
every verdict and CT byte is the oracle's (the batch's results do not
depend on the evicted entries), every surviving entry is byte-equal to the
oracle's (which has no capacity), and the evicted ones are exactly that
rule's.  Run on an MI355X: pytest -m gpu."""
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


def full_tables(fam, n_flows=2900, seed=5):
    """the endpoint's flows in its own maps, with spread lifetimes and
    states (SYN-only, established, closing); the same entries again in the
    global maps (no lookup of the batch reaches them: the endpoint has its
    own maps)"""
    cfg = S.config_c5 if fam == 4 else S.config_c5_v6
    t, flows = cfg(seed, n_flows=n_flows, n_prefixes=5000, n_policy=500, now=1000)
    rng = np.random.default_rng(seed + 3)
    ct = t.ct
    ct["lxc"] = S.EP_LXC_ID
    life = (1000 + rng.integers(30, 3000, size=len(ct))).astype(np.uint32)
    ct["entry"][:, 32:36] = life.view(np.uint8).reshape(-1, 4)
    st = rng.random(len(ct))
    bits = ct["entry"][:, 36].copy()
    bits = np.where(st < 0.4, bits | 16, bits)           # seen_non_syn
    bits = np.where(st > 0.95, bits | 3, bits)           # both closing bits
    ct["entry"][:, 36] = bits
    glob = ct.copy()
    glob["lxc"] = -1
    t.ct = np.concatenate([ct, glob])
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
        ks = 14 if fam == 1 else 38
        if len(sel):
            dp.update_batch(fd, np.ascontiguousarray(sel["tuple"][:, :ks]),
                            np.ascontiguousarray(sel["entry"]))
    dp.ct_fds = fds
    dp.commit()
    return pms


def refresh(r, ks):
    """lifetime minus the timeout of the entry's state (conntrack.h:125-205)"""
    e = r[44:100]
    life = int(e[32:36].view("<u4")[0])
    bits = int(e[36]) | int(e[37]) << 8
    tcp = r[4 + ks - 2] == 6
    to = 10 if (bits & 3) == 3 else (21600 if (bits & 16) else 60) if tcp else 60
    return life - to


@pytest.mark.parametrize("fam", [4, 6])
def test_full_endpoint_maps_stay_on_device(torch, fam):
    from cilium_amd.datapath import Datapath, pack
    from cilium_amd.loader import ct_rows
    # (IPv6: fewer of the batch's new flows are allowed, so a fuller map)
    t, flows = full_tables(fam, n_flows=2900 if fam == 4 else 2975)
    ks = 14 if fam == 4 else 38
    famb = 1 if fam == 4 else 2
    mine = (t.ct["lxc"] == S.EP_LXC_ID) & (t.ct["family"] == famb)
    n_tcp = int((mine & (t.ct["any"] == 0)).sum())
    assert CAP - 200 < n_tcp <= CAP, n_tcp          # the TCP map nearly full
    h = (S.headers_c5(t, flows, 8000, seed=9, new_frac=0.1) if fam == 4 else
         S.headers_c5_v6(t, flows, 8000, seed=9, new_frac=0.1))
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
    bmap = {key(r): r for r in before}
    total = 0
    for owner in (0, S.EP_LXC_ID + 1):          # global maps, the endpoint's
        for m in (0, 1):                         # TCP, ANY
            sel = lambda rs: [r for r in rs if r[3] == famb and r[2] == m and  # noqa: E731
                              int(r[0]) | int(r[1]) << 8 == owner]
            b_m, w_m = sel(before), sel(want)
            created = len({key(r) for r in w_m} - {key(r) for r in b_m})
            excess = max(0, len(b_m) + created - CAP)
            gone = sorted(key(r) for r in w_m if key(r) not in kept)
            # the rule: untouched entries (not hit: unchanged), earliest
            # refresh first, ties by key bytes
            cand = [r for r in w_m if key(r) in bmap and np.array_equal(r, bmap[key(r)])]
            cand.sort(key=lambda r: (refresh(r, ks), r[4:4 + ks].tobytes()))
            expect = sorted(key(r) for r in cand[:excess])
            assert len(gone) == excess, (owner, m, len(gone), excess)
            assert gone == expect, (owner, m)
            if owner == 0:
                assert excess == 0       # the batch writes no global map
            total += excess
    assert total == st["ct_evicted"], (total, st)


def test_evict_mid_apply_keeps_epoch_and_pending_work(torch):
    """The eviction inside an apply patches only the CT table (patch_ct), it
    does not commit: an earlier device apply's creates and TCP-map log
    entries are still pending (no host sync between the batches), and a
    policy entry added after the evicting batch was classified waits for a
    commit.  The apply stays on the device, keeps the epoch its kernels read,
    leaves the policy change pending for the next classify, and every
    verdict, CT byte and surviving entry matches the oracle's sequential run
    of both batches."""
    from cilium_amd.datapath import Datapath, pack
    from cilium_amd.loader import ct_rows
    t, flows = full_tables(4)
    # (new flows only: a live flow's packet could delete its entry, freeing
    # room the second batch then would not need to evict)
    h1 = S.headers_c5(t, flows, 100, seed=8, new_frac=1.0)
    h2 = S.headers_c5(t, flows, 8000, seed=9, new_frac=0.1)
    dp = Datapath(0)
    pms = load_capped(dp, t)
    dp.set_clock(1003)
    b1, b2 = pack(h1), pack(h2)
    o1 = dp.classify(b1, MODE_INGRESS, 0, want_ct=True)
    dp.ct_apply(b1, o1, MODE_INGRESS, 0)
    o2 = dp.classify(b2, MODE_INGRESS, 0, want_ct=True)
    e0 = dp.stats()["epoch"]
    pms[S.EP_LXC_ID].Allow(4_000_000, 0, 0, 0)   # (an identity no header has)
    dp.ct_apply(b2, o2, MODE_INGRESS, 0)
    torch.cuda.synchronize()
    st = dp.stats()
    assert st["epoch"] == e0, (st["epoch"], e0)
    assert st["ct_evicted"] > 0 and st["ct_apply_host"] == 0, st
    assert st["ct_apply_device"] == 2, st
    ver = np.concatenate([o1.verdict.cpu().numpy(), o2.verdict.cpu().numpy()])
    ctb = np.concatenate([o1.ct.cpu().numpy(), o2.ct.cpu().numpy()])
    dp.counters_sync()
    rows = ct_rows(dp, dp.ct_fds)
    o3 = dp.classify(b1, MODE_INGRESS, 0, want_ct=True)   # commits the policy entry
    torch.cuda.synchronize()
    assert dp.stats()["epoch"] != e0
    assert pms[S.EP_LXC_ID].Exists(4_000_000, 0, 0, 0)
    del o3
    dp.close()
    o = O.Oracle(t)
    o.set_clock(1003)
    _, over, _, _, oct_ = o.run_sequential(S.concat([h1, h2]), MODE_INGRESS, 0, want_ct=True)
    np.testing.assert_array_equal(ver, over)
    np.testing.assert_array_equal(ctb, oct_)
    wmap = {r[:44].tobytes(): r for r in o.ct_dump()}
    for r in rows:
        assert r[:44].tobytes() in wmap
        np.testing.assert_array_equal(r, wmap[r[:44].tobytes()])
