"""Device-side growth of the CT table (cfc_api.cpp ct_grow, ctapply.hip
k_ct_rehash).  The reference's CT maps are fixed-size LRU hashes
(bpf_lxc.c:53-89) whose inserts never stop; the engine's device table is
open-addressed and sized at commit, so a batch that would take it past 3/4
load moves it into a table of more slots on the device, inside
cfc_ct_apply_*, and folds the batch there — no host rebuild.  A stream whose
new flows outgrow a small starting table, in packet order, compared with the
oracle's sequential run (Oracle.run_sequential, pinned to the reference's
BPF by the ct_seq_* fixtures): verdicts, identities, CT bytes, monitor
records, every CT entry, every counter — and the growth really happened.
Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import oracle as O
from cilium_amd import synth as S
from cilium_amd import _lib as L
from cilium_amd.datapath import Datapath
from cilium_amd.loader import load_tables

from test_gpu_ctorder import check, run_both
from test_gpu_parity import compare_with_oracle, run_gpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def slots_at_load(t):
    dp = Datapath(0)
    load_tables(dp, t)
    st = dp.stats()
    dp.close()
    return st["ct_slots"]


@pytest.mark.parametrize("mode", [0, 3])
def test_ct_table_grows_inside_a_batch(torch, mode):
    """5k live flows (10k entries: a 32k-slot table), then a 600k-header packet-order
    stream with 30% new-flow headers in two batches: the first batch alone
    adds more keys than 3/4 of the table holds, so its apply grows the table
    on the device (with the batch's ordering already resolved) and folds it
    there; the second batch runs on the grown table."""
    t, flows = S.config_c5(5, n_flows=5_000, n_prefixes=20_000, n_policy=4000, now=1000)
    t.ct_max_entries = 1 << 20   # (the maps have room: only the device table is small)
    h = S.headers_c5_seq(t, flows, 600_000, seed=21, new_frac=0.3)
    before = slots_at_load(t)
    g, want = run_both(torch, t, h, mode, clock=1003, chunks=2, notify=True)
    check(g, want)
    st = g["stats"]
    assert st["ct_grown"] >= 1, st
    assert st["ct_slots"] > before, (st, before)
    assert st["ct_apply_host"] == 0, st


def test_ct_table_grows_twice_before_a_sync(torch):
    """Three batches that each outgrow the table: the growths stack their
    slot maps before anything reads the host mirror (one remap, composed on
    the device, taken at the final dump)."""
    t, flows = S.config_c5(5, n_flows=2_000, n_prefixes=20_000, n_policy=4000, now=1000)
    t.ct_max_entries = 1 << 20
    h = S.headers_c5_seq(t, flows, 900_000, seed=22, new_frac=0.4)
    g, want = run_both(torch, t, h, 3, clock=1003, chunks=3, notify=False)
    check(g, want)
    assert g["stats"]["ct_grown"] >= 2, g["stats"]


def test_ct6_table_grows_inside_a_batch(torch):
    """IPv6: 5k live flows, 40% new-flow headers, three batches folded on
    the device; every CT6 entry and counter against the oracle."""
    t, flows = S.config_c5_v6(6, n_flows=5_000, n_prefixes=20_000)
    t.ct_max_entries = 1 << 20
    h = S.headers_c5_v6(t, flows, 300_000, seed=43, new_frac=0.4)
    before = slots_at_load(t)
    compare_with_oracle(torch, t, h, 0, chunks=3, ct_apply=L.CT_APPLY_DEVICE)
    st = run_gpu.stats
    assert st["ct_grown"] >= 1 and st["ct_slots"] > before, (st, before)
    assert (st["ct_apply_device"], st["ct_apply_host"]) == (3, 0), st
