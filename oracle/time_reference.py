"""Time the reference's own BPF datapath on this container's cores.

TEST INFRASTRUCTURE ONLY (build container; the GPU box has no reference).
Runs the C2 bench workload's tables (100k IPv4 prefixes, 16k-entry
policymap, 25k /32 prefilter) through the compiled reference programs
(oracle/_ref: bpf_xdp.o, bpf_netdev.o -> bpf_lxc.o tail calls) with
BPF_PROG_TEST_RUN, one distinct header per run (repeat 1), FULL mode (XDP,
then netdev ingress for XDP_PASS), and sums the kernel-reported in-program
durations.  Per-core rate = headers / sum(duration); the node figure scales
it by the cores the kernel can run programs on in parallel (stated).

usage: python3 oracle/time_reference.py [n_headers] > profiles/cpu_reference_bpf_r01.json
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

from cilium_amd import synth as S   # noqa: E402
import bpf_harness as H             # noqa: E402
import gen_golden as GG             # noqa: E402


def main(n=20000):
    t = S.config_c2_bench(2)
    h = S.headers_c2(t, n, seed=2)
    dp = GG.RefDatapath(t)
    try:
        tot_xdp = tot_tc = 0
        passed = 0
        w0 = time.perf_counter()
        for i in range(n):
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
    ns = tot_xdp + tot_tc
    cores = len(os.sched_getaffinity(0))
    per_core = n / (ns * 1e-9) / 1e6
    print(json.dumps({
        "what": "reference BPF datapath (bpf_xdp.c + bpf_netdev.c -> bpf_lxc.c, "
                "compiled from /root/reference by oracle/Makefile) under "
                "BPF_PROG_TEST_RUN, C2 tables, FULL mode, one distinct header "
                "per run",
        "headers": n, "xdp_pass": passed,
        "in_program_ns_per_header": round(ns / n, 1),
        "xdp_ns_per_header": round(tot_xdp / n, 1),
        "tc_ns_per_passed_header": round(tot_tc / max(1, passed), 1),
        "mpps_per_core": round(per_core, 3),
        "cores": cores,
        "mpps_node_extrapolated": round(per_core * cores, 3),
        "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" \t:"),
        "kernel": os.uname().release,
        "wall_s_incl_syscalls": round(wall, 2),
    }))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
