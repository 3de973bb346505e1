"""Packet-order conntrack on the GPU (ctorder.hip + the device apply): a
batch classified and folded by cfc_ct_apply gives, header by header, what the
reference gives running the batch one packet at a time — each packet's
ct_lookup sees the ct_create / ct_delete of the packets before it
(conntrack.h:221-285, 615-772; bpf_lxc.c:963-970).  Compared with the
oracle's sequential run (Oracle.run_sequential, pinned to the reference's
BPF by the ct_seq_* fixtures: test_oracle_golden) on streams full of such
dependencies: verdicts, identities, CT bytes, every CT entry, every counter,
every monitor record.  Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import oracle as O
from cilium_amd import synth as S
from cilium_amd import metricsmap
from cilium_amd.datapath import Datapath, pack
from cilium_amd.loader import ct_rows, load_tables, policy_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def run_both(torch, t, h, mode, ep_lxc=0, clock=1003, chunks=3, notify=True):
    """the engine, batch by batch (classify, cfc_ct_apply, monitor records),
    and the oracle one header at a time over the same stream.  notify=False:
    no event words (the apply then folds a hot slot's plain hits by
    reduction, ctapply.hip k_cta_fold_long)"""
    dp = Datapath(0)
    pms = load_tables(dp, t)
    dp.set_clock(clock)
    b = pack(h)
    n = len(h)
    step = (n + chunks - 1) // chunks
    g = {k: [] for k in ("act", "ver", "ide", "ct", "nt", "rec", "idx")}
    for a in range(0, n, step):
        sub = b.slice(a, a + step)
        out = dp.classify(sub, mode, ep_lxc, want_ct=True, want_notify=notify)
        dp.ct_apply(sub, out, mode, ep_lxc)
        if notify:
            rec, idx, total = dp.monitor_events(sub, out, mode, ep_lxc)
        torch.cuda.synchronize()
        g["act"].append(out.action.cpu().numpy())
        g["ver"].append(out.verdict.cpu().numpy())
        g["ide"].append(out.identity.cpu().numpy().view(np.uint32))
        g["ct"].append(out.ct.cpu().numpy())
        if notify:
            g["nt"].append(out.notify.cpu().numpy().view(np.uint32))
            g["rec"].append(np.ascontiguousarray(rec.cpu().numpy()).view(O.EVENT_DT)
                            .reshape(-1))
            g["idx"].append(idx.cpu().numpy().astype(np.uint64) + a)
    g = {k: np.concatenate(v) for k, v in g.items() if v}
    dp.counters_sync()
    g["counters"] = {lxc: np.array(policy_rows(pm), np.uint64).reshape(-1, 7)
                     for lxc, pm in pms.items()}
    g["metrics"] = np.array(metricsmap.dump_rows(dp), np.uint64).reshape(-1, 4)
    g["identity"] = dp.identity_counters()
    g["rows"] = ct_rows(dp, dp.ct_fds)
    g["stats"] = dp.stats()
    dp.close()
    o = O.Oracle(t)
    o.set_clock(clock)
    act, ver, ide, words, ct = o.run_sequential(h, mode, ep_lxc, want_ct=True)
    rec, idx = o.events(h, mode, ep_lxc, ver, ide, words)
    want = dict(act=act, ver=ver, ide=ide, ct=ct, nt=words, rec=rec, idx=idx,
                rows=o.ct_dump(), metrics=o.metrics(), identity=o.identity_counters(),
                counters={lxc: o.policy_counters(lxc) for lxc in t.policy})
    return g, want


def check(g, want):
    for k in ("act", "ver", "ide", "ct", "nt", "idx"):
        if k not in g:
            continue
        bad = np.nonzero(g[k] != want[k])[0]
        assert len(bad) == 0, f"{k}: {len(bad)} differ, first {bad[:6]} " \
                              f"{g[k][bad[:6]]} vs {want[k][bad[:6]]}"
    if "rec" in g:
        np.testing.assert_array_equal(g["rec"].view(np.uint8), want["rec"].view(np.uint8))
    a, b = g["rows"], want["rows"]
    if a.shape == b.shape:
        for r in np.nonzero((a != b).any(1))[0][:4]:
            cols = np.nonzero(a[r] != b[r])[0]
            print("ct row", r, cols, a[r][cols], b[r][cols], a[r].tobytes().hex())
    else:
        print("ct rows", a.shape, b.shape)
    np.testing.assert_array_equal(a, b)
    for lxc, exp in want["counters"].items():
        np.testing.assert_array_equal(g["counters"][lxc], exp)
    np.testing.assert_array_equal(g["metrics"], want["metrics"])
    np.testing.assert_array_equal(g["identity"], want["identity"])
    assert g["stats"]["ct_apply_host"] == 0, g["stats"]


@pytest.mark.parametrize("clock", [1003, 2000])
def test_c5_packet_order(torch, clock):
    """C5 tables and live flows; a stream whose new flows have several
    packets (SYN, ACK, data, ICMP error, FIN/RST, a packet after the close)
    and whose denied flows lose their entry to their first packet.  Clock
    1003: the flows' report interval still running (only new TCP flags and
    closes report); 2000: past it (each flow's first hit per direction
    reports, its later hits in the batch do not)."""
    t, flows = S.config_c5(5, n_flows=200_000, n_prefixes=50_000, n_policy=8000, now=1000)
    h = S.headers_c5_seq(t, flows, 900_000, seed=11)
    g, want = run_both(torch, t, h, 3, clock=clock)
    check(g, want)
    # the stream holds what it is about
    assert g["stats"]["ct_order_changed"] > 10_000, g["stats"]
    ct = want["ct"]
    assert ((ct & 7) == 5).sum() > 1000 and ((ct & 0xF) == 0xC).sum() > 1000
    caps = np.unique(want["rec"]["len_cap"][want["rec"]["type"] == 4])
    assert 128 in caps, caps


def test_c5_packet_order_one_batch(torch):
    """The same, the whole stream one batch (every dependency inside it)."""
    t, flows = S.config_c5(5, n_flows=50_000, n_prefixes=20_000, n_policy=4000, now=1000)
    h = S.headers_c5_seq(t, flows, 400_000, seed=12)
    g, want = run_both(torch, t, h, 0, clock=1010, chunks=1)
    check(g, want)
    assert g["stats"]["ct_order_changed"] > 1000, g["stats"]


@pytest.mark.parametrize("clock", [1003, 2000])
def test_c5_packet_order_hot_flows(torch, clock):
    """Without event words: a Zipf stream's hottest flows, ordered by their
    closes, hold tens of thousands of ops on one slot each — their final
    state comes from a reduction over the run (k_cta_fold_long), every CT
    entry byte for byte against the sequential oracle."""
    t, flows = S.config_c5(5, n_flows=50_000, n_prefixes=50_000, n_policy=8000, now=1000)
    h = S.headers_c5_seq(t, flows, 1_200_000, seed=13)
    g, want = run_both(torch, t, h, 3, clock=clock, chunks=2, notify=False)
    check(g, want)
    # hot slots: some flow has more than FOLD_LONG (512) packets per batch
    key = h.saddr.astype(np.uint64) << 32 | h.daddr.astype(np.uint64)
    _, cnt = np.unique(key, return_counts=True)
    assert cnt.max() > 4 * 512, cnt.max()


@pytest.mark.parametrize("mode", [0, 3])
def test_sparse_apply_packet_order(torch, mode, monkeypatch):
    """The apply's sparse passes — ordering and scan over the classify
    launch's work list (kern_common.hpp wl_want) instead of the whole batch —
    on a stream without deletes (the headers of denied live flows taken out;
    test_sparse_apply_with_deletes keeps them): multi-packet new flows,
    closes, ICMP errors, hot flows.  Every output, CT entry and counter
    against the sequential oracle, and the dense passes (CFC_DENSE_APPLY)
    give the same."""
    t, flows = S.config_c5(5, n_flows=100_000, n_prefixes=50_000, n_policy=8000, now=1000)
    h = S.headers_c5_seq(t, flows, 600_000, seed=17)
    o = O.Oracle(t)
    o.set_clock(1003)
    _, ov, _, oct_ = o.classify(h, mode, 0, nthreads=16, want_ct=True)
    est_drop = ((oct_ & 0xF) == (1 | 4)) & (ov == -133)   # ESTABLISHED, DROP_POLICY
    h = S.take(h, np.flatnonzero(~est_drop))
    g, want = run_both(torch, t, h, mode, chunks=3, notify=False)
    check(g, want)
    # (a batch whose sequential run still deletes — a new flow's later packet
    # the policy drops — takes the dense passes)
    assert g["stats"]["ct_apply_sparse"] >= 2, g["stats"]
    assert g["stats"]["ct_order_changed"] > 1000, g["stats"]
    monkeypatch.setenv("CFC_DENSE_APPLY", "1")
    gd, _ = run_both(torch, t, h, mode, chunks=3, notify=False)
    assert gd["stats"]["ct_apply_sparse"] == 0, gd["stats"]
    for k in ("act", "ver", "ide", "ct"):
        np.testing.assert_array_equal(g[k], gd[k])
    np.testing.assert_array_equal(g["rows"], gd["rows"])


@pytest.mark.parametrize("mode", [0, 3])
def test_sparse_apply_with_deletes(torch, mode, monkeypatch):
    """Batches that delete stay on the sparse passes (round 6: the deleted
    slots' mixed hits join the work list, ctorder.hip k_ord_mixed /
    k_ord_collect_mix / k_ord_write): the dependency stream with its denied
    live flows (each loses its entry to its first packet, the later packets
    of the batch find none), closes, multi-packet new flows, ICMP errors.
    Every output, CT entry and counter against the sequential oracle, every
    batch sparse, and the dense passes give the same."""
    t, flows = S.config_c5(5, n_flows=100_000, n_prefixes=50_000, n_policy=8000, now=1000)
    h = S.headers_c5_seq(t, flows, 600_000, seed=19)
    o = O.Oracle(t)
    o.set_clock(1003)
    _, ov, _, oct_ = o.classify(h, mode, 0, nthreads=16, want_ct=True)
    est_drop = ((oct_ & 0xF) == (1 | 4)) & (ov == -133)   # ESTABLISHED, DROP_POLICY
    assert est_drop.sum() > 1000
    g, want = run_both(torch, t, h, mode, chunks=3, notify=False)
    check(g, want)
    monkeypatch.setenv("CFC_DENSE_APPLY", "1")
    gd, _ = run_both(torch, t, h, mode, chunks=3, notify=False)
    assert gd["stats"]["ct_apply_sparse"] == 0, gd["stats"]
    for k in ("act", "ver", "ide", "ct"):
        np.testing.assert_array_equal(g[k], gd[k])
    np.testing.assert_array_equal(g["rows"], gd["rows"])
    assert g["stats"]["ct_apply_sparse"] == 3, g["stats"]
