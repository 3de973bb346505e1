"""The BASELINE.json configurations at their full size on the GPU, every
output of every header and every counter compared with the oracle:
  C2  configs[1]: 100k IPv4 prefixes, 16k-entry policymap, 25k prefilter,
      one 64M-header batch (the bench's batch);
  C3  configs[2]: 1M IPv6 + 100k IPv4 prefixes, 50k-entry prefilter;
  C5  configs[4]: C2 + 10M live flows (16M CT entries, a 32M-slot device
      table) with Zipf traffic, two batches folded into CT in between — the
      CT accounting pass overflows its LDS table here; and its IPv6 shape
      (10M live CT6 flows, two batches, the GC's expiry on the device).
Run on an MI355X: pytest -m gpu."""
import time

import numpy as np
import pytest

import oracle as O
from cilium_amd import metricsmap
from cilium_amd import synth as S
from cilium_amd.datapath import Datapath, HeaderBatchV4, pack
from cilium_amd.loader import ct_rows, load_tables, policy_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def log(*a):
    print(*a, flush=True)


def compare_counters(dp, pms, o):
    dp.counters_sync()
    for lxc, pm in pms.items():
        np.testing.assert_array_equal(np.array(policy_rows(pm), np.uint64).reshape(-1, 7),
                                      o.policy_counters(lxc))
    np.testing.assert_array_equal(
        np.array(metricsmap.dump_rows(dp), np.uint64).reshape(-1, 4), o.metrics())
    np.testing.assert_array_equal(dp.identity_counters(), o.identity_counters())


def compare_outputs(out, oa, ov, oi):
    for name, a, b in (("action", out.action.cpu().numpy().astype(np.int32), oa),
                       ("verdict", out.verdict.cpu().numpy(), ov),
                       ("identity", out.identity.cpu().numpy().view(np.uint32), oi)):
        bad = np.flatnonzero(a != b)
        assert len(bad) == 0, f"{name}: {len(bad)} of {len(a)} differ, first {bad[:8]}"


def test_c2_full_64M_batch(torch):
    t0 = time.time()
    t = S.config_c2_bench(2)
    dp = Datapath(0)
    pms = load_tables(dp, t)
    n = 64 << 20
    s, d, p, m = S.gen_batch_v4_torch(t, n, 2000, "cuda:0")
    out = dp.classify_v4(HeaderBatchV4(s, d, p, m), 3)
    torch.cuda.synchronize()
    h = S.unpack_v4(s.cpu().numpy(), d.cpu().numpy(), p.cpu().numpy(), m.cpu().numpy())
    log(f"C2 64M: engine done {time.time() - t0:.1f}s")
    o = O.Oracle(t)
    oa, ov, oi = o.classify(h, 3, 0, nthreads=16)
    log(f"C2 64M: oracle done {time.time() - t0:.1f}s")
    compare_outputs(out, oa, ov, oi)
    compare_counters(dp, pms, o)
    assert len(np.unique(ov)) >= 4
    dp.close()


def test_c3_full_tables(torch):
    t0 = time.time()
    t = S.config_c3(3)
    dp = Datapath(0)
    pms = load_tables(dp, t)
    st = dp.stats()
    assert st["ipcache_v6_prefixes"] >= 1_000_000 and st["ipcache_v4_prefixes"] >= 100_000
    assert st["prefilter_v4_fix"] + st["prefilter_v6_fix"] >= 50_000
    log(f"C3: tables {time.time() - t0:.1f}s, lpm6 {st['lpm6_kib']} KiB")
    o = O.Oracle(t)
    h6 = S.headers_c3(t, 4_000_000, seed=33)
    rng = np.random.default_rng(34)
    h4 = S.gen_headers_v4(rng, 4_000_000, t.ipcache[t.ipcache["family"] == 1],
                          S.local_v4_addrs(t), proxy_ident=S.proxy_identities(t))
    for h in (h6, h4):
        out = dp.classify(pack(h), 3)
        torch.cuda.synchronize()
        oa, ov, oi = o.classify(h, 3, 0, nthreads=16)
        compare_outputs(out, oa, ov, oi)
    log(f"C3: compared {time.time() - t0:.1f}s")
    compare_counters(dp, pms, o)
    dp.close()


def test_c5_full_flows(torch):
    t0 = time.time()
    t, flows = S.config_c5(5, n_flows=10_000_000, now=1000)
    log(f"C5: {len(t.ct)} CT entries generated {time.time() - t0:.1f}s")
    dp = Datapath(0)
    pms = load_tables(dp, t)
    st = dp.stats()
    # ICMP 'related' entries in the TCP maps are unreachable by a lookup and
    # stay host-side (layout.h); the rest is the device table (> 8M -> 32M slots)
    assert st["ct4_entries"] >= 10_000_000, st
    log(f"C5: engine tables {time.time() - t0:.1f}s")
    o = O.Oracle(t)
    log(f"C5: oracle tables {time.time() - t0:.1f}s")
    h = S.headers_c5(t, flows, 8_000_000, seed=55)
    rng = np.random.default_rng(55)
    h.tcpflags = np.where(h.proto == 6, rng.choice(np.array([0x10, 0x18, 0x02], np.uint8),
                                                   size=len(h)), 0).astype(np.uint8)
    b = pack(h)
    for k, clock in enumerate((1003, 1010)):
        dp.set_clock(clock)
        o.set_clock(clock)
        a, e = k * len(h) // 2, (k + 1) * len(h) // 2
        sub = b.slice(a, e)
        out = dp.classify(sub, 3, want_ct=True, want_notify=True)
        # (the events after the apply: it rewrites the CT results and monitor
        # lengths into packet order, DESIGN.md §4 "Packet order")
        dp.ct_apply(sub, out, 3)
        rec, idx, total = dp.monitor_events(sub, out, 3)
        part = h.slice(a, e)
        oa, ov, oi, oct_, ow = o.classify(part, 3, 0, nthreads=16, want_ct=True,
                                          want_notify=True, apply_ct=True)
        compare_outputs(out, oa, ov, oi)
        np.testing.assert_array_equal(out.ct.cpu().numpy(), oct_)
        orec, oidx = o.events(part, 3, 0, ov, oi, ow)
        assert total == len(orec)
        np.testing.assert_array_equal(idx.cpu().numpy().astype(np.uint64), oidx)
        np.testing.assert_array_equal(
            np.ascontiguousarray(rec.cpu().numpy()).view(O.EVENT_DT).reshape(-1), orec)
        log(f"C5: batch {k} compared {time.time() - t0:.1f}s")
    st = dp.stats()
    assert (st["ct_apply_device"], st["ct_apply_host"]) == (2, 0), st
    compare_counters(dp, pms, o)
    got, want = ct_rows(dp, dp.ct_fds), o.ct_dump()
    assert got.shape == want.shape
    np.testing.assert_array_equal(got, want)
    log(f"C5: CT maps compared ({len(got)} entries) {time.time() - t0:.1f}s")
    dp.close()


def test_c5_v6_full_flows(torch):
    """The C5 shape in IPv6 at full size: C3-shaped tables (100k IPv6
    prefixes) + 10M live flows in the global CT6 maps (a 32M-slot device
    table of 48-byte keys), two Zipf batches classified, applied on the
    device in packet order, then the CT GC's expiry on the device
    (k_ct_gc<true>): verdicts, CT bytes, counters, the GC's deletes and every
    CT6 entry against the oracle."""
    from cilium_amd import ctmap
    t0 = time.time()
    t, flows = S.config_c5_v6(6, n_flows=10_000_000, n_prefixes=100_000, now=1000)
    log(f"C5v6: {len(t.ct)} CT entries generated {time.time() - t0:.1f}s")
    dp = Datapath(0)
    pms = load_tables(dp, t)
    st = dp.stats()
    assert st["ct6_entries"] >= 10_000_000 and st["ct_slots"] >= 32 << 20, st
    log(f"C5v6: engine tables {time.time() - t0:.1f}s")
    o = O.Oracle(t)
    h = S.headers_c5_v6(t, flows, 4_000_000, seed=66)
    rng = np.random.default_rng(66)
    h.tcpflags = np.where(h.proto == 6, rng.choice(np.array([0x10, 0x18, 0x02], np.uint8),
                                                   size=len(h)), 0).astype(np.uint8)
    b = pack(h)
    for k, clock in enumerate((1003, 1010)):
        dp.set_clock(clock)
        o.set_clock(clock)
        a, e = k * len(h) // 2, (k + 1) * len(h) // 2
        sub = b.slice(a, e)
        out = dp.classify(sub, 0, want_ct=True)
        dp.ct_apply(sub, out, 0)
        oa, ov, oi, oct_ = o.classify(h.slice(a, e), 0, 0, nthreads=16, want_ct=True,
                                      apply_ct=True)
        compare_outputs(out, oa, ov, oi)
        np.testing.assert_array_equal(out.ct.cpu().numpy(), oct_)
        log(f"C5v6: batch {k} compared {time.time() - t0:.1f}s")
    st = dp.stats()
    assert (st["ct_apply_device"], st["ct_apply_host"]) == (2, 0), st
    # the GC at a clock past the UDP lifetime of the flows the batches missed
    f = ctmap.GCFilter(remove_expired=True)
    ctmap.GC(dp, -1, f, now=1070)
    n = o.ct_gc(time=1070)
    st = f.stats   # (test_gpu_ctgc.same_count: a twice-written pending entry counts twice)
    assert st["device_deleted"] + st["host_deleted"] <= n <= st["deleted"], (st, n)
    assert st["device_deleted"] > 0, st
    compare_counters(dp, pms, o)
    got, want = ct_rows(dp, dp.ct_fds), o.ct_dump()
    assert got.shape == want.shape
    np.testing.assert_array_equal(got, want)
    log(f"C5v6: CT maps compared ({len(got)} entries) {time.time() - t0:.1f}s")
    dp.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_c1_million(torch, mode):
    """C1 (configs[0]): the example policies' MapState over 11 endpoints,
    1M headers: ingress to every endpoint, or egress from app=myService
    (L4 + CIDR rules), every output and counter against the oracle."""
    t, _ = S.config_c1(1)
    if mode == 0:
        ep, h = 0, S.headers_c1(t, 1_000_000, seed=11)
    else:
        ep = [x for x in t.policy if t.seclabel[x] == 257][0]
        addr = t.endpoints["addr"][t.endpoints["lxc_id"] == ep][0, :4].copy().view("<u4")[0]
        rng = np.random.default_rng(12)
        h = S.gen_headers_v4(rng, 1_000_000, t.ipcache, S.local_v4_addrs(t),
                             local_frac=0.2, src_fixed=addr, ports=S.C1_PORTS,
                             other_proto=0.0)
    dp = Datapath(0)
    pms = load_tables(dp, t)
    out = dp.classify(pack(h), mode, ep)
    torch.cuda.synchronize()
    o = O.Oracle(t)
    oa, ov, oi = o.classify(h, mode, ep, nthreads=16)
    compare_outputs(out, oa, ov, oi)
    compare_counters(dp, pms, o)
    assert len(np.unique(ov)) >= 2
    dp.close()
