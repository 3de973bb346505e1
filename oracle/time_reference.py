"""Time the reference's own BPF datapath on this container's cores.

TEST INFRASTRUCTURE ONLY (build container; the GPU box has no reference).
Runs the C2 bench workload's tables (100k IPv4 prefixes, 16k-entry
policymap, 25k /32 prefilter) through the compiled reference programs
(oracle/_ref: bpf_xdp.o, bpf_netdev.o -> bpf_lxc.o tail calls) with
BPF_PROG_TEST_RUN, one distinct header per run (repeat 1), FULL mode (XDP,
then netdev ingress for XDP_PASS), and sums the kernel-reported in-program
durations.

SURVEY.md §8d (1): one process per core, each pinned to its core
(sched_setaffinity) with its own loaded programs and maps, all running at
once on disjoint slices of the header stream; a process's rate is its
headers over its summed in-program time, and the node figure is the sum of
the per-core rates measured side by side (so contention between the cores
is in it, not extrapolated from one core).

usage: python3 oracle/time_reference.py [n_headers [processes]] > profiles/r06/cpu_reference_bpf.json
"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

from cilium_amd import synth as S   # noqa: E402
import bpf_harness as H             # noqa: E402
import gen_golden as GG             # noqa: E402


def worker(core, lo, hi, n, start, q):
    """one pinned process: its own reference datapath, headers [lo, hi)"""
    os.sched_setaffinity(0, {core})
    t = S.config_c2_bench(2)
    h = S.headers_c2(t, n, seed=2)
    dp = GG.RefDatapath(t)
    try:
        start.wait()   # (every process loaded: they run side by side)
        tot_xdp = tot_tc = passed = 0
        w0 = time.perf_counter()
        for i in range(lo, hi):
            ret, d = H.test_run_duration(dp.xdp, GG.build_packet_v4(h, i), xdp=True)
            tot_xdp += d
            if ret == GG.XDP_PASS:
                passed += 1
                _, d2 = H.test_run_duration(dp.netdev, GG.build_packet_v4(h, i),
                                            mark=int(h.mark[i]))
                tot_tc += d2
        wall = time.perf_counter() - w0
    finally:
        dp.close()
    q.put(dict(core=core, headers=hi - lo, xdp_ns=tot_xdp, tc_ns=tot_tc, passed=passed,
               wall_s=wall))


def main(n=80000, procs=None):
    cores = sorted(os.sched_getaffinity(0))
    procs = min(procs or len(cores), len(cores))
    ctx = mp.get_context("fork")
    q, start = ctx.Queue(), ctx.Barrier(procs)
    per = (n + procs - 1) // procs
    ps = [ctx.Process(target=worker,
                      args=(cores[k], k * per, min(n, (k + 1) * per), n, start, q))
          for k in range(procs)]
    for p in ps:
        p.start()
    res = sorted((q.get() for _ in ps), key=lambda r: r["core"])
    for p in ps:
        p.join()
    rates = [r["headers"] / ((r["xdp_ns"] + r["tc_ns"]) * 1e-9) / 1e6 for r in res]
    ns = sum(r["xdp_ns"] + r["tc_ns"] for r in res)
    passed = sum(r["passed"] for r in res)
    wall = max(r["wall_s"] for r in res)
    print(json.dumps({
        "what": "reference BPF datapath (bpf_xdp.c + bpf_netdev.c -> bpf_lxc.c, "
                "compiled from /root/reference by oracle/Makefile) under "
                "BPF_PROG_TEST_RUN, C2 tables, FULL mode, one distinct header "
                "per run; one pinned process per core, all cores at once",
        "headers": n, "xdp_pass": passed,
        "cores": procs,
        "in_program_ns_per_header": round(ns / n, 1),
        "xdp_ns_per_header": round(sum(r["xdp_ns"] for r in res) / n, 1),
        "tc_ns_per_passed_header": round(sum(r["tc_ns"] for r in res) / max(1, passed), 1),
        "mpps_per_core": [round(x, 3) for x in rates],
        "mpps_node": round(sum(rates), 3),
        "mpps_node_wall_incl_syscalls": round(n / wall / 1e6, 3),
        "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" \t:"),
        "kernel": os.uname().release,
        "wall_s_incl_syscalls": round(wall, 2),
    }))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
