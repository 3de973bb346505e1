"""LXC_NAT46 on the GPU (nat.hip + the classify kernels + cfc_ct_apply): the
NAT64 hop of IPv6 egress headers to v4-mapped peers (bpf_lxc.c:353-360,
tail_ipv6_to_ipv4 :1070-1083, nat46.h:336-420) and the NAT46 hop of IPv4
ingress headers that hit a nat46 CT entry (bpf_lxc.c:939-944,
tail_ipv4_to_ipv6 :1098-1110, nat46.h:236-328), against the oracle's
sequential run (Oracle.run_sequential; its NAT restatement is pinned by the
reference's nat46_egress_v6 / nat46_reply_v4 fixtures, test_oracle_golden):
verdicts, identities, CT bytes, event words and records, every CT entry of
both families, every counter.  The GPU tests run on an MI355X (pytest -m gpu);
the stream checks at the bottom run on the CPU."""
import numpy as np
import pytest

import oracle as O
from cilium_amd import synth as S

MODE_INGRESS, MODE_EGRESS, MODE_FULL = 0, 1, 3
NATLEN = 1 << 24


def nat_tables(seed=61, n_hist=1200, clock=1000):
    """config_nat's tables with the CT state of a NAT64 history (the oracle
    runs it: its entries carry nat46) -> (tables, ipc4, history, forwarded)"""
    t, ipc4 = S.config_nat(seed)
    rng = np.random.default_rng(seed + 9)
    hist = S.nat64_flows(rng, ipc4, n_hist, 20000)
    o = O.Oracle(t)
    o.set_clock(clock)
    act, ver, ide, words = o.run_sequential(hist, MODE_EGRESS, S.EP_LXC_ID)
    t.ct = S.ct_from_rows(o.ct_dump())
    return t, ipc4, hist, np.flatnonzero(act != 2)


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [1, 3])
def test_nat64_egress_vs_oracle(torch, chunks):
    from test_gpu_ctorder import check, run_both
    t, ipc4, hist, ok = nat_tables()
    h = S.headers_nat64(t, ipc4, hist, 30_000)
    g, want = run_both(torch, t, h, MODE_EGRESS, S.EP_LXC_ID, clock=1003, chunks=chunks)
    check(g, want)
    assert g["stats"]["nat_hops"] > 5000, g["stats"]
    assert (want["nt"] & NATLEN).any()


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [1, 2])
def test_nat64_local_delivery_vs_oracle(torch, chunks):
    """NAT64 to an endpoint of this node: the hop's IPv4 egress delivers
    locally (l3.h:103-131) and the destination's ipv4_policy runs a third CT
    stage in its CT maps — its creates without nat46 (conntrack.h:714-716),
    its deletes at that stage.  The nat64_local_v6 fixture's tables (the
    reference's run pins the oracle there, test_oracle_golden) and its
    stream three times over, shuffled, against the sequential oracle."""
    import golden_io as G
    from test_gpu_ctorder import check, run_both
    g = G.Golden("nat64_local_v6")
    rng = np.random.default_rng(7)
    h = S.concat([g.headers] * 3)
    h = S.take(h, rng.permutation(len(h)))
    gg, want = run_both(torch, g.tables, h, MODE_EGRESS, S.EP_LXC_ID, clock=1003,
                        chunks=chunks)
    check(gg, want)
    assert gg["stats"]["nat_hops"] > 3000, gg["stats"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [MODE_INGRESS, MODE_FULL])
def test_nat46_reply_vs_oracle(torch, mode):
    from test_gpu_ctorder import check, run_both
    t, ipc4, hist, ok = nat_tables(seed=63)
    h = S.headers_nat46(t, ipc4, hist, ok, 30_000)
    g, want = run_both(torch, t, h, mode, 0, clock=1003, chunks=2)
    check(g, want)
    assert g["stats"]["nat_hops"] > 5000, g["stats"]


@pytest.mark.gpu
def test_nat_round_trip_vs_oracle(torch):
    """NAT64 flows opened in one IPv6 egress batch, their replies (NAT46)
    in the next IPv4 ingress batch: the entries the device apply created
    carry nat46 into the next classify"""
    from test_gpu_ctorder import check, run_both
    from cilium_amd.datapath import Datapath, pack
    from cilium_amd.loader import ct_rows, load_tables
    t, ipc4 = S.config_nat(65)
    t.ct = np.zeros(0, S.CT_DT)   # (empty CT maps: the first batch opens the flows)
    rng = np.random.default_rng(66)
    out6 = S.nat64_flows(rng, ipc4, 20_000, 20000)
    dp = Datapath(0)
    load_tables(dp, t)
    dp.set_clock(1000)
    b6 = pack(out6)
    o6 = dp.classify(b6, MODE_EGRESS, S.EP_LXC_ID, want_ct=True)
    dp.ct_apply(b6, o6, MODE_EGRESS, S.EP_LXC_ID)
    torch.cuda.synchronize()
    act6 = o6.action.cpu().numpy()
    # the replies of the forwarded ones
    ok = np.flatnonzero(act6 != 2)
    rep = S.headers_nat46(t, ipc4, out6, ok, 20_000, seed=67)
    b4 = pack(rep)
    o4 = dp.classify(b4, MODE_INGRESS, 0, want_ct=True, want_notify=True)
    dp.ct_apply(b4, o4, MODE_INGRESS, 0)
    torch.cuda.synchronize()
    g = dict(act=o4.action.cpu().numpy(), ver=o4.verdict.cpu().numpy(),
             ide=o4.identity.cpu().numpy().view(np.uint32), ct=o4.ct.cpu().numpy(),
             nt=o4.notify.cpu().numpy().view(np.uint32))
    dp.counters_sync()   # (the CT accounting into the maps)
    rows = ct_rows(dp, dp.ct_fds)
    st = dp.stats()
    dp.close()
    o = O.Oracle(t)
    o.set_clock(1000)
    o.run_sequential(out6, MODE_EGRESS, S.EP_LXC_ID)
    act, ver, ide, words, ct = o.run_sequential(rep, MODE_INGRESS, 0, want_ct=True)
    for k, w in (("act", act), ("ver", ver), ("ide", ide), ("ct", ct), ("nt", words)):
        bad = np.nonzero(g[k] != w)[0]
        assert len(bad) == 0, f"{k}: {len(bad)} differ, first {bad[:6]}"
    want = o.ct_dump()
    if rows.shape == want.shape:
        for r in np.nonzero((rows != want).any(1))[0][:6]:
            cols = np.nonzero(rows[r] != want[r])[0]
            print("ct row", r, cols, rows[r][cols], want[r][cols], rows[r].tobytes().hex())
    else:
        print("ct rows", rows.shape, want.shape)
    np.testing.assert_array_equal(rows, want)
    assert st["nat_hops"] > 20_000 and st["ct_apply_host"] == 0, st


# ---- the streams (CPU: the oracle only) -----------------------------------

def test_nat_streams_exercise_the_hops():
    """the generated streams reach every NAT outcome the GPU tests compare"""
    t, ipc4, hist, ok = nat_tables(n_hist=600)
    o = O.Oracle(t)
    o.set_clock(1003)
    h = S.headers_nat64(t, ipc4, hist, 6000)
    act, ver, ide, words, ct = o.run_sequential(h, MODE_EGRESS, S.EP_LXC_ID, want_ct=True)
    nat = (words & NATLEN) != 0
    assert nat.sum() > 1000
    assert (ver == -156).any()                       # ipv6_to_ipv4's exthdr drop
    assert ((ct >> 4) & 0xC).tolist().count(0xC) > 50  # hop creates
    assert ((ct >> 4) & 7).tolist().count(5) > 100     # hop ESTABLISHED
    rows = S.ct_from_rows(o.ct_dump())
    assert len(rows)
    o2 = O.Oracle(t)
    o2.set_clock(1003)
    h4 = S.headers_nat46(t, ipc4, hist, ok, 6000)
    act, ver, ide, words, ct = o2.run_sequential(h4, MODE_INGRESS, 0, want_ct=True)
    nat = (words & NATLEN) != 0
    assert nat.sum() > 1000
    assert ((ct >> 4) & 0xC).tolist().count(0xC) > 50  # ipv6_policy creates
    assert (ver == -133).any() and (ver == 0).any()
