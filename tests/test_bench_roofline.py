"""The bench line's roofline from the committed PMC records
(profiles/pmc_traffic.json, written by scripts/pmc_summary.py --record) and
the random-access ceilings (profiles/ubench/): every recorded kernel prices
below its ceiling (frac <= 1) under the slowest row its misses can be
priced at, and the headline C2 kernel sits at >= 0.5 of it.  CPU only: the
records carry each kernel's average launch time from the same profile."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

DB = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))["entries"]


def test_ceilings_measured():
    rows = bench.ubench_ceilings()
    assert rows, "profiles/ubench has no random-access rows"
    mibs = [m for m, _ in rows]
    assert mibs == sorted(mibs)
    # the L2-resident rows are the fastest, the largest tables the slowest
    assert rows[0][1] > rows[-1][1]


@pytest.mark.parametrize("e", DB, ids=[x["workload"] for x in DB])
def test_recorded_kernels_below_ceiling(e):
    rows = bench.ubench_ceilings()
    assert os.path.isdir(os.path.join(ROOT, e["source"])), e["source"]
    for k, pk in e["kernels"].items():
        for field in ("headers", "l2_requests_per_launch", "hbm_bytes_per_launch", "avg_ms"):
            assert field in pk, (k, field)
        if not pk["headers"]:
            # (a CT apply or GC kernel: priced per launch against HBM in the
            # bench line's ct_apply section, not on the request roofline)
            assert pk["hbm_bytes_per_launch"] > 0 and pk["avg_ms"] > 0, (k, pk)
            continue
        # (the requests and the hit / miss split come from separate counter
        # passes over the same bench run: equal to a few in 10^4)
        assert pk["l2_hits_per_launch"] + pk["l2_misses_per_launch"] == pytest.approx(
            pk["l2_requests_per_launch"], rel=1e-3)
        # a small working set prices misses at the HBM row, the slowest
        d, t_ideal, _ = bench.kernel_roofline(k, pk["headers"], pk["avg_ms"], 1 << 20, pk, rows)
        assert 0 < d["frac"] <= 1.0, (e["workload"], k, d["frac"])
        assert t_ideal > 0


def test_headline_c2_at_half_of_its_ceiling():
    e = next(x for x in DB if x["workload"] == "c2")
    pk = e["kernels"]["k_classify_v4"]
    d, _, _ = bench.kernel_roofline("k_classify_v4", pk["headers"], pk["avg_ms"],
                                    3 << 20, pk, bench.ubench_ceilings())
    assert d["frac"] >= 0.5, d
    assert pk["headers"] == 64 << 20


def test_stream_ceiling_measured_and_monotone():
    """The stream-miss ceiling (scripts/ubench_mix.hip stream mode): more
    L2 probes per 32-byte stream item, fewer items per second, and a
    probe-free item runs at a streaming rate."""
    rates = [bench.stream_ceiling(p) for p in (0.0, 0.5, 1.0, 1.63, 2.0, 4.0, 16.0)]
    assert all(r for r in rates), rates
    assert all(a >= b for a, b in zip(rates, rates[1:])), rates
    assert rates[0] * 32 > 3000   # GB/s of stream with no probes


def test_headline_c2_priced_with_its_own_misses():
    """k_classify_v4 at C2 is priced with its misses as the coalesced header
    stream they are (33 B per header), its L2 hits spread over it: the
    stream model is what the line's frac uses, and the kernel sits below
    that ceiling."""
    e = next(x for x in DB if x["workload"] == "c2")
    pk = e["kernels"]["k_classify_v4"]
    d, t_ideal, _ = bench.kernel_roofline("k_classify_v4", pk["headers"], pk["avg_ms"],
                                          3 << 20, pk, bench.ubench_ceilings(),
                                          bench.STREAM_V4)
    st = d["stream_model"]
    assert st and st["random_misses_per_launch"] < 0.2 * st["stream_lines_per_launch"], d
    assert 0.5 <= d["frac"] <= 1.0, d
