"""The engine's side of the multi-GPU counter exchange, on one
GPU: two contexts stand in for two ranks, each classifies its contiguous shard
of the stream against the same tables, their counter blocks are exported
(cfc_counters_export), summed as the RCCL all-reduce would, imported into one
(cfc_counters_import) and folded (cfc_counters_sync).  The totals — policy
entries, cilium_metrics and the per-identity forward/drop counters — equal
the oracle's over the whole stream.  Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import oracle as O
from cilium_amd import metricsmap
from cilium_amd import synth as S
from cilium_amd.datapath import Datapath, pack_v4
from cilium_amd.distributed import shard_range
from cilium_amd.loader import load_tables, policy_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


@pytest.mark.parametrize("mode", [0, 1, 3])
def test_export_sum_import_equals_whole_stream(torch, mode):
    t = S.config_c2(7, n_prefixes=50_000, n_policy=8000, n_endpoints=2)
    if mode == 1:
        rng = np.random.default_rng(7)
        h = S.gen_headers_v4(rng, 1_000_000, t.ipcache, S.local_v4_addrs(t),
                             local_frac=0.2, src_fixed=S.LXC_IPV4)
    else:
        h = S.headers_c2(t, 1_000_000, seed=7)
    ep = S.EP_LXC_ID if mode == 1 else 0
    world = 2
    ranks, blocks = [], []
    for r in range(world):
        dp = Datapath(0)
        pms = load_tables(dp, t)
        a, b = shard_range(len(h), r, world)
        dp.classify_v4(pack_v4(h.slice(a, b)), mode, ep)
        _, n = dp.counters_device()
        blk = torch.empty(n, dtype=torch.int64, device="cuda:0")
        dp.counters_export(blk)
        ranks.append((dp, pms))
        blocks.append(blk)
    total = blocks[0] + blocks[1]          # the all-reduce (SUM, int64 = u64)
    for dp, _ in ranks:
        dp.counters_import(total)
        dp.counters_sync()
    torch.cuda.synchronize()
    o = O.Oracle(t)
    o.classify(h, mode, ep, nthreads=16)
    for dp, pms in ranks:
        for lxc, pm in pms.items():
            np.testing.assert_array_equal(np.array(policy_rows(pm), np.uint64),
                                          o.policy_counters(lxc))
        np.testing.assert_array_equal(
            np.array(metricsmap.dump_rows(dp), np.uint64).reshape(-1, 4), o.metrics())
        ident = dp.identity_counters()
        np.testing.assert_array_equal(ident, o.identity_counters())
        assert ident[:, 2].sum() > 0 and ident[:, 4].sum() > 0
    # export zeroed the blocks: another sync adds nothing
    dp, pms = ranks[0]
    dp.counters_sync()
    np.testing.assert_array_equal(dp.identity_counters(), o.identity_counters())
    for dp, _ in ranks:
        dp.close()
