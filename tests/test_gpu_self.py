"""Traffic to itself on the GPU (cfc_api.cpp self_cuts, selfseg.hip): an
endpoint's flows to its own address and the flows a service loops back into
it, inside the egress batches that create their entries.  A later header of
such a flow finds, as k1, the entry an earlier header's other stage wrote
(conntrack.h:487-494, 725-748), so the engine cuts the batch there and
classifies each segment after the ones before it were folded into CT.
Compared with the oracle's packet order (Oracle.run_sequential), which the
self_egress_v4 / self_egress_v6 fixtures pin to the reference."""
import numpy as np
import pytest

import golden_io as G
from cilium_amd import synth as S
from test_gpu_parity import compare_with_oracle, run_gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def _self_stream(g, seed, n):
    """The fixture's tables; a stream of n headers: self TCP / UDP flows
    (opening packet, answer, more packets, some closes), pings and ICMP
    errors to itself, the fixture's own packets (service flows, their
    answers), and the fixture's plain traffic, shuffled flow-wise so each
    flow keeps its packet order"""
    rng = np.random.default_rng(seed)
    h0 = g.headers
    v6 = h0.family == 6
    A = np.asarray(S.LXC_IPV6, np.uint8) if v6 else np.uint32(S.LXC_IPV4)
    nf = n // 10
    x = rng.integers(1024, 65535, size=nf)
    y = rng.choice(np.array([80, 53, 8080, 5353, 443]), size=nf)
    proto = np.where(np.isin(y, [53, 5353]), S.IPPROTO_UDP, S.IPPROTO_TCP)
    pos, rows = [], []
    t0 = rng.random(nf)
    for j, (a, b, f) in enumerate([(x, y, 0x02), (y, x, 0x12), (x, y, 0x10), (y, x, 0x18),
                                   (x, y, 0x11)]):
        sel = rng.random(nf) < (1.0 if j < 2 else 0.6)
        for i in np.flatnonzero(sel):
            rows.append((int(a[i]), int(b[i]), int(proto[i]), f))
            pos.append(t0[i] + 0.002 * j + rng.random() * 0.001)
    icmp = S.IPPROTO_ICMPV6 if v6 else S.IPPROTO_ICMP
    echo, reply, errs = (128, 129, [1, 3]) if v6 else (8, 0, [3, 11])
    for _ in range(n // 40):
        p = rng.random()
        rows.append((echo, 0, icmp, 0))
        pos.append(p)
        rows.append((reply, 0, icmp, 0))
        pos.append(p + 0.001)
    for _ in range(n // 100):
        rows.append((int(rng.choice(errs)), 0, icmp, 0))
        pos.append(rng.random())
    m = len(rows)
    r = np.array(rows, np.int64)
    sa = np.tile(A, (m, 1)) if v6 else np.full(m, A, np.uint32)
    h = S.Headers(h0.family, sa, sa.copy(), S.htons(r[:, 0]), S.htons(r[:, 1]),
                  r[:, 2].astype(np.uint8), np.zeros(m, np.uint8),
                  rng.integers(100, 1500, size=m).astype(np.uint16), np.zeros(m, np.uint32),
                  np.where(r[:, 2] == S.IPPROTO_TCP, r[:, 3], 0).astype(np.uint8))
    h.flags[(h.proto == S.IPPROTO_TCP) & ((h.tcpflags & 0x05) != 0)] = S.HF_TCP_CLOSE
    # the fixture's stream (service flows and their answers, plain traffic)
    # keeps its own order, spread through the stream
    p0 = np.sort(rng.random(len(h0)))
    h0 = S.Headers(h0.family, h0.saddr, h0.daddr, h0.sport, h0.dport, h0.proto, h0.flags,
                   h0.length, h0.mark, S.tcp_flags_of(h0), None)
    out = S.concat([h, h0])
    out = S.take(out, np.argsort(np.concatenate([np.array(pos), p0]), kind="stable"))
    out.hash = None
    return out


@pytest.mark.parametrize("name", ["self_egress_v4", "self_egress_v6"])
def test_self_stream_vs_oracle(torch, name):
    """Verdicts, identities, CT bytes, counters and every CT entry against
    the oracle's packet order, in two batches each folded before the next;
    the batch-start view differs on many headers, and the batches were cut"""
    g = G.Golden(name)
    h = _self_stream(g, 5 if name.endswith("v4") else 6, 40_000)
    compare_with_oracle(torch, g.tables, h, g.mode, g.ep_lxc, chunks=2)
    assert run_gpu.stats["ct_self_segments"] > 0
    assert run_gpu.stats["ct_apply_host"] == 0
    import oracle as O
    oa, ov, oi = O.Oracle(g.tables).classify(h, g.mode, g.ep_lxc, nthreads=8)
    o = O.Oracle(g.tables)
    sa, sv, si, _ = o.classify(h, g.mode, g.ep_lxc, nthreads=8, want_ct=True, apply_ct=True)
    assert ((oa != sa) | (ov != sv)).sum() > 100


def test_self_cuts_off_without_self_traffic(torch):
    """A batch with no header to the sender's own addresses is one launch"""
    g = G.Golden("ct_seq_egress_v4")
    h = S.take(g.headers, np.flatnonzero(g.headers.daddr != S.LXC_IPV4))
    run_gpu(torch, g.tables, h, g.mode, g.ep_lxc)
    assert run_gpu.stats["ct_self_segments"] == 0
