"""Benchmark: classified headers/s (Mpps, whole node) of the MI355X verdict
engine at the C2 configuration (100k-prefix IPv4 ipcache + 16k-entry
policymap, 64M-header batches; BASELINE.json configs[1]).

A step = one cfc_classify_v4 launch over one resident 64M-header batch in
FULL mode: XDP prefilter (25k-entry /32 deny-list) -> ipcache LPM -> endpoint
-> policymap with L3/wildcard fallbacks -> verdicts + counters.  With
--gpus N (torchrun, one rank per GPU) each rank classifies its own 64M shard
of the stream (weak scaling, tables replicated) and the counters are
all-reduced over RCCL once at the end of the timed region.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
S_IN, S_OUT = 16, 8        # SoA bytes per header in (saddr,daddr,ports,meta) / out
# bytes the classify kernel streams per header through HBM: the SoA input,
# verdict + identity + action, and the two counter-key arrays k_hist reads
STREAM_V4 = S_IN + 4 + 4 + 1 + 4 + 4
STREAM_V6 = 40 + 4 + 4 + 1 + 4 + 4


def ubench_ceilings():
    """Measured chip-wide random-load rate (G loads/s, best over load width
    and loads in flight) per table size in MiB: scripts/ubench_random.hip,
    committed under profiles/ubench/.  One L2 request per load (TCC_REQ of
    the same kernel, profiles/ubench/README)."""
    import glob
    best = {}
    for f in glob.glob(os.path.join(ROOT, "profiles", "ubench", "random_access_*.jsonl")):
        for line in open(f):
            r = json.loads(line)
            best[r["table_mib"]] = max(best.get(r["table_mib"], 0.0), r["gloads_per_s"])
    return sorted(best.items())


def mix_ceiling(p):
    """The chip's measured rate (G loads/s) of independent random 16-byte
    loads when a fraction p hits a 2 MiB (L2-resident) table and the rest a
    4 GiB (HBM) one (scripts/ubench_mix.hip, profiles/r04/ubench_mix.jsonl),
    interpolated in p; None without the measurement.  The measurement shows
    that hits and misses of one kernel do not overlap: at p >= 0.75 the mix
    runs below even the additive model (a wave waits for its slowest load)."""
    try:
        pts = sorted((r["p"], r["gloads_per_s"]) for r in
                     map(json.loads, open(os.path.join(ROOT, "profiles", "r04",
                                                       "ubench_mix.jsonl"))))
    except (OSError, ValueError):
        return None
    for (p0, r0), (p1, r1) in zip(pts, pts[1:]):
        if p0 <= p <= p1:
            return r0 + (r1 - r0) * (p - p0) / max(p1 - p0, 1e-9)
    return pts[-1][1] if p > pts[-1][0] else pts[0][1]


def stream_ceiling(probes_per_item):
    """The chip's measured rate (G items/s) of a kernel whose misses are a
    coalesced stream: per item (a lane-iteration) P random 16-byte probes of
    a 2 MiB (L2-resident) table, 16 bytes read one iteration ahead from a
    4 GiB input stream and 16 bytes written (scripts/ubench_mix.hip stream
    mode, profiles/r05/ubench_stream.jsonl), interpolated in P; None without
    the measurement."""
    try:
        pts = sorted((r["probes_per_item"], r["gitems_per_s"]) for r in
                     map(json.loads, open(os.path.join(ROOT, "profiles", "r05",
                                                       "ubench_stream.jsonl"))))
    except (OSError, ValueError):
        return None
    for (p0, r0), (p1, r1) in zip(pts, pts[1:]):
        if p0 <= probes_per_item <= p1:
            # (time per item is what adds up linearly in P)
            t = 1 / r0 + (1 / r1 - 1 / r0) * (probes_per_item - p0) / max(p1 - p0, 1e-9)
            return 1 / t
    p_last, r_last = pts[-1]
    return r_last * p_last / probes_per_item if probes_per_item > p_last else pts[0][1]


def ceiling_for(ws_bytes, rows):
    """(table MiB, G loads/s) of the smallest measured table holding ws_bytes."""
    for mib, rate in rows:
        if mib * (1 << 20) >= ws_bytes:
            return mib, rate
    return rows[-1]


def pmc_entry(workload, mode, layout, kernels, variant="lookup"):
    """This configuration's per-kernel PMC record (scripts/pmc_summary.py
    --record) for this kernel variant (lookup, ct_apply, notify), or None
    when absent or made for other batch sizes."""
    try:
        db = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    except (OSError, ValueError):
        return None
    for e in db.get("entries", []):
        if (e["workload"], e["mode"], e["lpm4_layout"], e.get("variant", "lookup")) != \
                (workload, mode, layout, variant):
            continue
        if all(k in e["kernels"] and e["kernels"][k]["headers"] == n for k, n in kernels):
            return e
    return None


def kernel_roofline(k, hn, ms, ws, pk, rows, stream_bph=None):
    """One kernel's roofline entry: the launch's L2 hits priced at the L2
    ceiling, its misses (TCC_MISS: the header stream, the output stores, and
    table lines past L2) at the row of the memory that serves them — the
    Infinity-Cache row of a kernel whose tables outgrow L2, else the HBM row
    (the largest table measured) — over its live duration ms; pk: its PMC
    record (profiles/pmc_traffic.json) or None.  Returns (entry, ideal
    seconds, uniform-model seconds)."""
    l2_peak = ceiling_for(1, rows)[1]
    mib, peak_k = ceiling_for(ws, rows)
    miss_mib, miss_peak = (mib, peak_k) if ws > 6 * (1 << 20) else rows[-1]
    d = {"kernel": k, "headers": hn, "ms_per_launch": round(ms, 4),
         "working_set_mib": round(ws / (1 << 20), 2),
         "ceiling_table_mib": mib, "ceiling_greq_s": peak_k}
    if not pk:
        return d, 0.0, 0.0
    req = pk["l2_requests_per_launch"]
    hits, miss = pk.get("l2_hits_per_launch"), pk.get("l2_misses_per_launch")
    if hits is None or miss is None:
        hits, miss = req, 0.0
    t_add = hits / (l2_peak * 1e9) + miss / (miss_peak * 1e9)
    t_unif = req / (peak_k * 1e9)
    # the bound: the measured rate of this kernel's hit/miss mix (the
    # additive model is optimistic for mixes, profiles/r04/ubench_mix.jsonl:
    # L2 hits mixed with HBM misses); a kernel whose misses the Infinity
    # Cache serves keeps the additive model
    p = hits / req if req else 1.0
    mixr = mix_ceiling(p) if miss_mib >= 4096 else None
    t_mix = req / (mixr * 1e9) if mixr else t_add
    t_ideal = t_mix
    # the kernel's own miss type: its header stream and output stores are
    # coalesced and read an iteration ahead (the stream model: items of 32
    # stream bytes, the L2 hits spread over them); the misses beyond the
    # stream's lines (a table past L2, C5's CT slots) at the random row
    st = None
    if stream_bph:
        items = hn * stream_bph / 32.0
        rate = stream_ceiling(hits / items) if items else None
        lines = hn * stream_bph / 128.0
        rand = max(0.0, miss - lines)
        # (a kernel whose misses are mostly table lines past L2 — C5's CT
        # slots, the IPv6 tables in the Infinity Cache — keeps the
        # random-miss mix: its stream is the smaller part)
        if rate and rand <= 0.2 * lines:
            t_ideal = items / (rate * 1e9) + rand / (miss_peak * 1e9)
            st = {"items_per_launch": items, "probes_per_item": round(hits / items, 3),
                  "stream_ceiling_gitems_s": round(rate, 3),
                  "stream_lines_per_launch": lines, "random_misses_per_launch": rand}
    d.update({"l2_requests_per_launch": req,
              "l2_requests_per_header": round(req / hn, 3),
              "l2_hits_per_launch": hits, "l2_misses_per_launch": miss,
              "hit_fraction": round(p, 4),
              "mix_ceiling_greq_s": round(mixr, 1) if mixr else None,
              "stream_model": st,
              "frac_random_mix": round(t_mix / (ms * 1e-3), 4),
              "hit_ceiling_greq_s": l2_peak,
              "miss_ceiling_greq_s": miss_peak, "miss_ceiling_table_mib": miss_mib,
              "achieved_greq_s": round(req / (ms * 1e-3) / 1e9, 1),
              "frac": round(t_ideal / (ms * 1e-3), 4),
              "frac_additive": round(t_add / (ms * 1e-3), 4),
              "frac_uniform": round(t_unif / (ms * 1e-3), 4),
              "hbm_bytes_per_launch": pk["hbm_bytes_per_launch"]})
    return d, t_ideal, t_unif


def reference_bpf_baseline():
    """The reference's own BPF datapath timed under BPF_PROG_TEST_RUN in the
    build container (oracle/time_reference.py; the GPU box has no reference
    and no BPF objects), newest committed measurement."""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "cpu_reference_bpf_*.json")))
    if not fs:
        return None
    fs.sort(key=lambda f: os.path.basename(os.path.dirname(f)))
    r = json.load(open(fs[-1]))
    if "mpps_node" in r:   # (round 6 on: one pinned process per core, all at once)
        return {"value": r["mpps_node"], "unit": "Mpps (node)",
                "cores": r["cores"], "kind": "reference",
                "mpps_per_core": r["mpps_per_core"],
                "where": f"build container ({r['cpu']}, kernel {r['kernel']}), not the GPU box",
                "sample": f"{r['headers']} distinct C2 headers over {r['cores']} pinned "
                          f"processes (one per core, side by side), FULL mode (bpf_xdp -> "
                          f"bpf_netdev -> bpf_lxc tail calls), in-program time summed per "
                          f"process, one header per BPF_PROG_TEST_RUN",
                "source": os.path.relpath(fs[-1], ROOT)}
    return {"value": r["mpps_per_core"], "unit": "Mpps per core",
            "cores": 1, "kind": "reference",
            "where": f"build container ({r['cpu']}, kernel {r['kernel']}), not the GPU box",
            "sample": f"{r['headers']} distinct C2 headers, FULL mode (bpf_xdp -> "
                      f"bpf_netdev -> bpf_lxc tail calls), in-program time summed, "
                      f"one header per BPF_PROG_TEST_RUN",
            "source": os.path.relpath(fs[-1], ROOT)}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--headers", type=int, default=64 << 20)
    ap.add_argument("--mode", default="full",
                    choices=["ingress", "egress", "xdp", "full"])
    ap.add_argument("--cpu-sample", type=int, default=2_000_000,
                    help="headers timed on the host-core oracle (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--notify", action="store_true",
                    help="also produce every monitor record — drop_notify and "
                         "trace_notify (cfc_monitor_events_v4) — inside the timed step")
    ap.add_argument("--lpm4", default="auto", choices=["auto", "dir24_8", "trie"],
                    help="IPv4 ipcache device layout (cfc_set_option CFC_OPT_LPM4)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c5"],
                    help="c2: BASELINE.json configs[1] (the metric's config); "
                         "c3: configs[2], dual stack: 1M IPv6 + 100k IPv4 "
                         "prefixes, 50k prefilter, half the batch each family; "
                         "c5: configs[4], + conntrack with --flows live flows "
                         "and Zipf(1.1) traffic (side measurements)")
    ap.add_argument("--flows", type=int, default=10_000_000)
    ap.add_argument("--ct-apply", action="store_true",
                    help="c5: every step is classify + cfc_ct_apply_v4 (the batch's CT "
                         "creates, deletes and timeouts written into the device CT "
                         "table) + the CT garbage collector when its interval has "
                         "passed; the new flows' source ports are re-drawn on the "
                         "device at the start of each step, so every step creates")
    ap.add_argument("--family", type=int, default=4, choices=[4, 6],
                    help="c5: the IPv4 (default) or the IPv6 shape — config_c5_v6's C3 "
                         "tables (100k IPv6 prefixes) and --flows live CT6 flows, every "
                         "header IPv6 (cfc_classify_v6 + cfc_ct_apply_v6)")
    ap.add_argument("--stream", default="spec", choices=["spec", "seq"],
                    help="c5: spec = SURVEY.md §8d's C5 stream (new flows whose "
                         "reverse is not in the batch); seq = synth.headers_c5_seq, "
                         "the dependency-heavy stream of the packet-order tests "
                         "(new flows of several packets, closes, deletes, ICMP errors)")
    ap.add_argument("--step-seconds", type=int, default=61,
                    help="--ct-apply: datapath clock advance per step (cfc_set_clock)")
    ap.add_argument("--gc-interval", type=int, default=60,
                    help="--ct-apply: conntrack-garbage-collector-interval "
                         "(daemon/main.go:367, default 60 s): cfc_ct_gc with "
                         "RemoveExpired at the step's clock once this much clock "
                         "has passed since the last one (0: no GC)")
    args = ap.parse_args()
    if args.ct_apply and args.workload != "c5":
        ap.error("--ct-apply needs --workload c5")
    if args.notify and (args.workload == "c3" or args.family == 6):
        ap.error("--notify covers IPv4 batches (c2, c5)")
    if args.family == 6 and (args.workload != "c5" or args.stream != "spec"):
        ap.error("--family 6: the c5 workload's spec stream")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the ranks before anything touches the
        # GPU (torchrun on 127.0.0.1), wait for them, exit with their status
        import subprocess
        port = 29500 + os.getpid() % 2000
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
               f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    import torch
    import torch.distributed as dist
    from cilium_amd import synth as S
    from cilium_amd import _lib as LL
    from cilium_amd.datapath import Datapath, HeaderBatchV4, Verdicts
    from cilium_amd.distributed import allreduce_counters, c5_rank_setup, env_rank
    from cilium_amd.loader import load_tables

    rank, local_rank, world = env_rank()
    assert world == args.gpus, f"WORLD_SIZE {world} != --gpus {args.gpus}"
    # (the rank's GPU first: RCCL's communicator binds to the current device)
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local_rank)
    mode = {"ingress": 0, "egress": 1, "xdp": 2, "full": 3}[args.mode]
    ep_lxc = S.EP_LXC_ID if mode == 1 else 0

    t0 = time.time()
    v6c5 = args.workload == "c5" and args.family == 6
    if v6c5:
        assert world == 1, "--family 6: one GPU"
        tables, flows = S.config_c5_v6(args.seed, n_flows=args.flows)
        log(f"[rank {rank}] C5 IPv6 tables: {len(tables.ct)} CT6 entries for "
            f"{len(flows)} flows ({time.time() - t0:.1f}s)")
    elif args.workload == "c5":
        tables, flows = S.config_c5(args.seed, n_flows=args.flows)
        # several GPUs: flow affinity — each rank holds the CT
        # entries and draws the traffic of the address pairs it owns; no CT
        # collective
        tables.ct, flows = c5_rank_setup(tables, flows, rank, world)
        log(f"[rank {rank}] C5 tables: {len(tables.ct)} CT entries for "
            f"{len(flows)} of {args.flows} flows ({time.time() - t0:.1f}s)")
    elif args.workload == "c3":
        tables = S.config_c3(3)
    else:
        tables = S.config_c2_bench(args.seed)
    dp = Datapath(local_rank)
    dp.set_option(LL.OPT_LPM4, {"auto": LL.LPM4_AUTO, "dir24_8": LL.LPM4_DIR24_8,
                                "trie": LL.LPM4_TRIE}[args.lpm4])
    load_tables(dp, tables)
    st = dp.stats()
    log(f"[rank {rank}] tables loaded+committed in {time.time() - t0:.1f}s: {st}")

    n = args.headers
    batch6, h6 = None, None
    # each rank owns its shard of the stream: seed differs per rank
    if args.workload == "c3":
        from cilium_amd.datapath import pack_v6
        h6 = S.headers_c3(tables, n // 2, seed=args.seed * 1000 + rank)
        batch6 = pack_v6(h6, dev)
        n = n - n // 2
        s, d, p, m = S.gen_batch_v4_torch(tables, n, args.seed * 1000 + rank, dev)
    elif v6c5:   # every header IPv6: the v4 batch is empty
        from cilium_amd.datapath import pack_v6
        h6, new6 = S.headers_c5_v6(tables, flows, n, seed=args.seed * 1000 + rank,
                                   return_new=True)
        new6 &= (h6.proto == S.IPPROTO_TCP) | (h6.proto == S.IPPROTO_UDP)
        batch6 = pack_v6(h6, dev)
        n = 0
        s, d, p, m = (torch.empty(0, dtype=torch.int32, device=dev) for _ in range(4))
        tf = torch.empty(0, dtype=torch.uint8, device=dev)
        new_idx = torch.from_numpy(np.flatnonzero(new6)).to(dev)
        new_ports = batch6.ports[new_idx].clone()
        h6 = S.take(h6, slice(0, min(len(h6), args.cpu_sample)))   # (the CPU sample)
    elif args.workload == "c5":
        from cilium_amd.datapath import pack_v4
        if args.stream == "seq":
            assert world == 1, "--stream seq: one GPU"
            h5, new5 = S.headers_c5_seq(tables, flows, n, seed=args.seed * 1000 + rank,
                                        return_new=True)
            # (the ports of TCP / UDP new flows are re-drawn per step; ICMP
            # keeps its type: an error stays related to its flow's pair)
            new5 &= (h5.proto == S.IPPROTO_TCP) | (h5.proto == S.IPPROTO_UDP)
        else:
            h5, new5 = S.headers_c5(tables, flows, n, seed=args.seed * 1000 + rank,
                                    return_new=True, owner=(rank, world))
        hb = pack_v4(h5, dev)
        s, d, p, m, tf = hb.saddr, hb.daddr, hb.ports, hb.meta, hb.tcp_flags
        del hb, h5
        new_idx = torch.from_numpy(np.flatnonzero(new5)).to(dev)
        new_ports = p[new_idx].clone()
    else:
        s, d, p, m = S.gen_batch_v4_torch(tables, n, args.seed * 1000 + rank, dev)
    if mode == 1:
        s.fill_(S.LXC_IPV4 - (1 << 32) if S.LXC_IPV4 >= 1 << 31 else S.LXC_IPV4)
    if args.workload != "c5":
        tf = None    # no TCP flag bytes in the C2/C3 streams (all CT_NEW)
    batch = HeaderBatchV4(s, d, p, m, None, tf)
    out = Verdicts(torch.empty(n, dtype=torch.int32, device=dev),
                   torch.empty(n, dtype=torch.int32, device=dev), None,
                   torch.empty(n, dtype=torch.uint8, device=dev) if args.ct_apply else None)
    salt = [0]
    clock = {"now": 0, "last_gc": 0, "gcs": 0, "gc_deleted": 0, "alive": None}
    n6 = len(batch6) if batch6 is not None else 0
    out6 = Verdicts(torch.empty(n6, dtype=torch.int32, device=dev),
                    torch.empty(n6, dtype=torch.int32, device=dev), None,
                    torch.empty(n6, dtype=torch.uint8, device=dev) if v6c5 and args.ct_apply
                    else None)
    # the batch the CT apply folds (IPv6 with --family 6)
    ct_batch, ct_out = (batch6, out6) if v6c5 else (batch, out)

    nt_rec = nt_idx = nt_cnt = None
    if args.notify:
        import ctypes
        from cilium_amd.datapath import _ptr
        out.notify = torch.empty(n, dtype=torch.int32, device=dev)
        nt_rec = torch.empty((n, 8), dtype=torch.int32, device=dev)
        nt_idx = torch.empty(n, dtype=torch.int64, device=dev)
        nt_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        from cilium_amd.datapath import hdr_struct, out_struct
        nt_hdr = hdr_struct(batch)
        nt_out = out_struct(out)
        nt_stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    # --ct-apply: HIP events around the apply and the GC of each timed step
    # (both synchronise with the host inside: the events bracket that too)
    ct_ev = []

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    def step(timed=False):
        if args.ct_apply:   # fresh new flows: their source ports re-drawn
            salt[0] += 1
            ct_batch.ports[new_idx] = new_ports ^ ((salt[0] * 0x9E37) & 0xFFFF)
            clock["now"] += args.step_seconds
            dp.set_clock(clock["now"])
        if n:
            dp.classify_v4(batch, mode, ep_lxc, out=out)
        if v6c5:
            dp.classify_v6(batch6, mode, ep_lxc, out=out6)
        if args.ct_apply:
            e0 = ev() if timed else None
            dp.ct_apply(ct_batch, ct_out, mode, ep_lxc)
            e1 = ev() if timed else None
            e2 = None
            # EnableConntrackGC's loop (pkg/endpointmanager/conntrack.go:96-125)
            if args.gc_interval and clock["now"] - clock["last_gc"] >= args.gc_interval:
                g = dp.ct_gc(-1, clock["now"])
                e2 = ev() if timed else None
                clock["last_gc"] = clock["now"]
                clock["gcs"] += 1
                clock["gc_deleted"] += g["deleted"]
                clock["alive"] = g["alive"]
            if timed:
                ct_ev.append((e0, e1, e2))
        if args.notify:   # records stay on the device (no sync in the step)
            LL.check(dp.L.cfc_monitor_events_v4(
                dp.h, ctypes.byref(nt_hdr), ctypes.byref(nt_out), mode, ep_lxc,
                _ptr(nt_rec), _ptr(nt_idx), n, _ptr(nt_cnt), nt_stream),
                "monitor events")
        if n6 and not v6c5:
            dp.classify_v6(batch6, mode, ep_lxc, out=out6)
    torch.cuda.synchronize()
    log(f"[rank {rank}] batch of {n} headers generated ({(n * S_IN) >> 20} MiB)")

    ord0 = None
    for w in range(args.warmup):
        step()
        if args.ct_apply:   # each step creates its new flows, the GC drops old ones
            torch.cuda.synchronize()
            sw = dp.stats()
            log(f"[rank {rank}] warmup {w}: clock {clock['now']} s, apply device "
                f"{sw['ct_apply_device']} host {sw['ct_apply_host']}, GC runs "
                f"{clock['gcs']} deleted {clock['gc_deleted']}")
    torch.cuda.synchronize()
    dp.counters_clear()
    # HIP events recorded by the library on the launch stream around the
    # classify kernel and the counter kernels of every timed call
    dp.set_option(LL.OPT_TIMING, 1)
    dp.timing_collect()
    if args.ct_apply:
        ord0 = dp.stats()["ct_order_changed"]

    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step(timed=True)
        evs[i][1].record(stream)
    if world > 1:
        allreduce_counters(dp)   # the only collective: counter SUM over RCCL
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - w0
    call_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    tm = dp.timing_collect()
    assert tm["launches"] == args.steps * ((1 if n else 0) + (1 if n6 else 0)), tm
    kern_ms = tm["classify_ms"] / args.steps        # classify kernel(s) per step
    count_ms = tm["count_ms"] / args.steps          # counter kernels per step
    kern6_ms = tm["classify_v6_ms"] / args.steps    # the IPv6 kernel's share
    if world > 1:
        tw = torch.tensor([wall], device=dev, dtype=torch.float64)
        dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        wall = float(tw.item())
    if world == 1 and not args.ct_apply:
        dp.counters_sync()
    # (with --ct-apply the counters stay on the device: folding them brings
    # the host mirror of the CT maps up to date first, untimed host work in
    # proportion to the run's CT changes — minutes after a long dependency
    # stream — that no figure of this line reads)
    total = (n + n6) * world * args.steps
    mpps = total / wall / 1e6
    log(f"[rank {rank}] {args.steps} steps in {wall * 1e3:.2f} ms; per call "
        f"{call_ms:.3f} ms = classify {kern_ms:.3f} + counters {count_ms:.3f}; "
        f"{mpps:.0f} Mpps")

    if rank != 0:
        dist.destroy_process_group()
        return

    # ---- algorithmic bytes per header from the oracle's lookup counts (L),
    #      and the host-core baseline + a parity check on the same sample
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    samp = args.cpu_sample if (world == 1 and not args.no_cpu) else 200_000
    samp6 = samp
    samp = min(samp, n)
    hs = S.unpack_v4(s[:samp].cpu().numpy(), d[:samp].cpu().numpy(),
                     p[:samp].cpu().numpy(), m[:samp].cpu().numpy())
    hs.tcpflags = (tf[:samp].cpu().numpy() if tf is not None
                   else np.zeros(samp, np.uint8))
    orc = O.Oracle(tables)
    # every core this process may use: the GPU pool gives a one-GPU box a
    # 16-core share and says so in OMP_NUM_THREADS (nproc shows the whole
    # machine there); elsewhere the affinity mask
    cores = int(os.environ.get("OMP_NUM_THREADS", 0)) or len(os.sched_getaffinity(0))
    # the timed run computes what the engine computes (no lookup counting);
    # the lookup counts for the §8d bytes come from a second, untimed run
    c0 = time.perf_counter()
    if n:
        oa, ov, oi = orc.classify(hs, mode, ep_lxc, nthreads=cores)
    cpu_s = time.perf_counter() - c0
    lk = orc.classify(hs, mode, ep_lxc, nthreads=cores, want_lookups=True)[3] if n \
        else np.zeros(1)
    # the timed region's last launch wrote `out` for this same batch
    # (with --ct-apply the tables moved on during the timed steps: the CT
    # parity of classify + apply is tests/test_gpu_fullsize.py's)
    parity = None if (args.ct_apply or not n) else bool(np.array_equal(out.verdict[:samp].cpu().numpy(), ov) and
                  np.array_equal(out.identity[:samp].cpu().numpy().view(np.uint32), oi))
    if v6c5:
        # the IPv6 sample's tuples as the last step classified them (its new
        # flows' ports re-drawn per step)
        pp = batch6.ports[:len(h6)].cpu().numpy().view(np.uint32)
        h6.sport, h6.dport = (pp & 0xFFFF).astype(np.uint16), (pp >> 16).astype(np.uint16)
    if args.notify:   # the sample's monitor records, every field
        _, ov2, oi2, ow = orc.classify(hs, mode, ep_lxc, nthreads=cores,
                                       want_notify=True)
        orec, oidx = orc.events(hs, mode, ep_lxc, ov2, oi2, ow)
        k = len(oidx)
        grec = nt_rec[:k].cpu().numpy()
        gidx = nt_idx[:k].cpu().numpy().astype(np.uint64)
        parity = parity and bool(np.array_equal(gidx, oidx) and np.array_equal(
            np.ascontiguousarray(grec).view(np.uint8).reshape(-1),
            np.ascontiguousarray(orec).view(np.uint8).reshape(-1)))
    mean_l = float(lk.mean())
    b_hdr = S_IN + S_OUT + 64.0 * mean_l
    algo_bytes = n * b_hdr
    if n6:   # the IPv6 half: 40 B in per header, its own lookup counts
        s6 = min(samp6, n6, len(h6))
        hs6 = S.take(h6, slice(0, s6))
        c1 = time.perf_counter()
        o6a, o6v, o6i = orc.classify(hs6, mode, ep_lxc, nthreads=cores)
        cpu_s += time.perf_counter() - c1
        lk6 = orc.classify(hs6, mode, ep_lxc, nthreads=cores, want_lookups=True)[3]
        parity = parity and bool(
            np.array_equal(out6.verdict[:s6].cpu().numpy(), o6v) and
            np.array_equal(out6.identity[:s6].cpu().numpy().view(np.uint32), o6i))
        b6 = 40 + S_OUT + 64.0 * float(lk6.mean())
        algo_bytes += n6 * b6
        mean_l = (n * mean_l + n6 * float(lk6.mean())) / (n + n6)
        b_hdr = algo_bytes / (n + n6)
        samp += s6
    algo_gbs = algo_bytes / (kern_ms * 1e-3) / 1e9
    layout = {1: "dir24_8", 2: "trie"}.get(st["lpm4_layout"], "none")
    # ---- the bound: the chip's random-request rate for the tables' size.
    # Per kernel: its working set (device tables; CT slots with their timer
    # and accounting words), the measured random-load ceiling for that size,
    # and its L2 requests per launch (TCC_REQ, committed PMC pass of this
    # configuration) over its live HIP-event duration.
    ws_ct4 = 64 * (1 << max(0, 2 * st["ct4_entries"] - 1).bit_length()) if st["ct4_entries"] else 0
    ws_ct6 = 96 * (1 << max(0, 2 * st["ct6_entries"] - 1).bit_length()) if st["ct6_entries"] else 0
    ws4 = st["device_bytes"] - 1024 * st["lpm6_kib"] + ws_ct4
    ws6 = st["device_bytes"] - 1024 * st["lpm4_kib"] + ws_ct6
    kernels = [("k_classify_v4", n, kern_ms - kern6_ms, ws4)] if n else []
    if n6:
        kernels.append(("k_classify_v6", n6, kern6_ms, ws6))
    rows = ubench_ceilings()
    # L2 hits at the L2 ceiling; misses (TCC_MISS: the header stream, the
    # output stores, and table lines past L2) at the row of the memory that
    # serves them: the Infinity-Cache row of a kernel whose tables outgrow
    # L2, else the HBM row (the largest table measured)
    variant = "ct_apply" if args.ct_apply else "notify" if args.notify else "lookup"
    pe = pmc_entry("c5v6" if v6c5 else args.workload, args.mode, layout,
                   [(k, hn) for k, hn, _, _ in kernels], variant)
    per_kernel = []
    req_tot = ideal_s = ideal_u = traffic = 0.0
    for k, hn, ms, ws in kernels:
        d, t_ideal, t_unif = kernel_roofline(k, hn, ms, ws, pe["kernels"][k] if pe else None,
                                             rows, STREAM_V6 if k.endswith("v6") else STREAM_V4)
        if pe:
            req_tot += d["l2_requests_per_launch"]
            ideal_s += t_ideal
            ideal_u += t_unif
            traffic += d["hbm_bytes_per_launch"]
        per_kernel.append(d)
    stream_b = n * STREAM_V4 + n6 * STREAM_V6
    bound = ("l2" if all(d["ceiling_table_mib"] <= 6 for d in per_kernel)
             else "infinity-cache" if all(d["ceiling_table_mib"] <= 256 for d in per_kernel)
             else "hbm-random")
    res = {
        "metric": "classified headers/sec (Mpps, whole node) at 100k-prefix "
                  "ipcache + 16k-ID policy",
        "value": round(mpps, 1),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": f"synthetic (seeded {args.workload.upper()} generator, SURVEY.md §8d)",
        "config": {
            "workload": ("C2: 100k IPv4 /8-/32 ipcache prefixes + 16384-entry "
                         "policymap + 25k /32 prefilter deny-list, "
                         if args.workload == "c2" else
                         f"C3: dual stack, {st['ipcache_v6_prefixes']} IPv6 /32-/128 + "
                         f"{st['ipcache_v4_prefixes']} IPv4 prefixes, "
                         f"{st['prefilter_v4_fix'] + st['prefilter_v6_fix']}-entry "
                         f"prefilter, {n6} IPv6 + {n} IPv4 headers per step, "
                         if args.workload == "c3" else
                         f"C5 IPv6: C3 tables ({st['ipcache_v6_prefixes']} IPv6 prefixes) + "
                         f"{st['ct6_entries']} reachable CT6 entries ({args.flows} live "
                         f"flows, global CT6 maps), 95% Zipf(1.1) packets of live flows + "
                         f"5% new (synth.headers_c5_v6), "
                         if v6c5 else
                         f"C5: C2 tables + {st['ct4_entries']} reachable CT4 "
                         f"entries ({args.flows} live flows, global CT maps), "
                         + ("95% Zipf(1.1) packets of live flows + 5% new, "
                            if args.stream == "spec" else
                            "92% Zipf(1.1) packets of live flows (2% closing, denied "
                            "flows deleted) + 8% new flows of several packets "
                            "(synth.headers_c5_seq), "))
                        + f"{n + n6}-header batch per GPU, mode {args.mode}",
            "headers_per_step_per_gpu": n + n6,
            "ipcache_prefixes": st["ipcache_v4_prefixes"],
            "policy_entries": st["policy_entries"],
            "prefilter_v4_fix": st["prefilter_v4_fix"],
            "mode": args.mode,
            "lpm4_layout": {1: "dir24_8", 2: "trie"}.get(st["lpm4_layout"], "none"),
            "parallelism": (f"flow-affinity shards x{world} (address-pair owner: CT "
                            f"entries and traffic per rank, no CT collective)"
                            if args.workload == "c5" and world > 1 else
                            f"header-stream shards x{world}, tables replicated"),
            "drop_notify": bool(args.notify),
            "ct_apply": bool(args.ct_apply),
            "family": 6 if v6c5 else 4,
        },
        "roofline": {
            "kernel": " + ".join(k for k, _, _, _ in kernels),
            # random L2 (or Infinity-Cache) requests: the measured request-rate
            # ceiling for the tables' size is the bound
            "bound": bound,
            "achieved": round(req_tot / (kern_ms * 1e-3) / 1e9, 1) if pe else None,
            "peak": round(req_tot / ideal_s / 1e9, 1) if pe else None,
            "unit": "Greq/s",
            "frac": round(ideal_s / (kern_ms * 1e-3), 4) if pe else None,
            # every request at the ceiling row of its kernel's working set
            # (round 2's model: it overprices IC-resident tables' L2 hits)
            "frac_uniform": round(ideal_u / (kern_ms * 1e-3), 4) if pe else None,
            "traffic": traffic if pe else None,
            "pmc_source": pe["source"] if pe else None,
            "kernels": per_kernel,
            "hbm_stream": {
                "bytes_per_header": round(stream_b / (n + n6), 2),
                "achieved_gbs": round(stream_b / (kern_ms * 1e-3) / 1e9, 1),
                "peak_gbs": HBM_PEAK_GBS,
                "frac": round(stream_b / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            },
            # SURVEY.md §8d's accounting — 24 B of header I/O + a 64 B line per
            # map lookup — is not a bound here: the tables are cache-resident,
            # so most lookups never reach HBM ("frac" above prices them at
            # the cache that serves them).  Kept as the §8d bytes per header
            # only; its rate is labelled as what it is
            "algorithmic": {
                "bytes_per_header": round(b_hdr, 2),
                "mean_lookups_per_header": round(mean_l, 4),
                "sec8d_equivalent_gbs_not_a_bound": round(algo_gbs, 1),
            },
            "kernel_ms_per_launch": round(kern_ms, 4),
            "count_kernels_ms_per_launch": round(count_ms, 4),
            "call_ms_per_launch": round(call_ms, 4),
        },
        "cpu_baseline": None if (world > 1 or args.no_cpu) else {
            "value": round(samp / cpu_s / 1e6, 3),
            "unit": "Mpps",
            "cores": cores,
            "kind": "port",
            "sample": f"first {samp} headers of the same stream through the C "
                      f"restatement (oracle/cfc_oracle.c), {cores} OpenMP threads",
            # the reference itself, measured where it can run
            "reference_bpf": reference_bpf_baseline(),
        },
        "parity_sample_ok": parity,
        "monitor_records_per_step_per_gpu": int(nt_cnt.item()) if args.notify else None,
    }
    if args.ct_apply:   # the step is classify + cfc_ct_apply_v4 (+ cfc_ct_gc)
        st2 = dp.stats()
        # the host fallback (table past 3/4 load) is not the measured path
        if st2["ct_apply_host"]:
            log(f"[rank {rank}] CT apply left the device path: {st2}")
            sys.exit(3)
        res["ct_apply"] = {
            "path_device_calls": st2["ct_apply_device"],
            "path_host_calls": st2["ct_apply_host"],
            "apply_and_gc_ms_per_step": round(call_ms - tm["classify_ms"] / args.steps
                                              - count_ms, 4),
            # HIP events around cfc_ct_apply_v4 and cfc_ct_gc of each step
            "apply_ms_per_step": round(float(np.mean([a.elapsed_time(b)
                                                      for a, b, _ in ct_ev])), 4),
            "gc_ms_per_run": round(float(np.mean([b.elapsed_time(c) for _, b, c in ct_ev
                                                  if c is not None])), 4)
            if any(c is not None for _, _, c in ct_ev) else None,
            "stream": args.stream,
            # CT stages per step whose packet-order result differs from the
            # batch-start lookup (ctorder.hip), and their share of the stages
            "ct_order_changed_per_step": (st2["ct_order_changed"] - ord0) / args.steps,
            "clock_s_per_step": args.step_seconds,
            "gc_interval_s": args.gc_interval,
            "gc_runs": clock["gcs"],
            "gc_deleted": clock["gc_deleted"],
            "ct_entries_after_last_gc": clock["alive"],
            # every timed step's call time (HIP events around classify +
            # apply + GC), and the device table's growths inside the run
            # (cfc_stats.ct_grown: the table moved into one of more slots on
            # the device, no host rebuild) and its slots at the end
            "step_ms": [round(a.elapsed_time(b), 3) for a, b in evs],
            "step_ms_max_over_median": round(max(a.elapsed_time(b) for a, b in evs) /
                                             float(np.median([a.elapsed_time(b)
                                                              for a, b in evs])), 3),
            "ct_grown": st2["ct_grown"],
            "ct_slots_end": st2["ct_slots"],
        }
        if pe:   # the apply's and GC's kernels from the same PMC record
            ck = []
            for k, d in sorted(pe["kernels"].items(), key=lambda kv: -kv[1]["avg_ms"]
                               * kv[1].get("calls", 1)):
                if k.startswith("k_classify"):
                    continue
                ms = d["avg_ms"]
                # FETCH_SIZE counts a wide streaming read at 1/2 on gfx950
                # (MI355X_MICROARCH.md); the random reads at their size: the
                # kernel's HBM bytes lie between FETCH + WRITE and 2 FETCH + WRITE
                lo = d["hbm_bytes_per_launch"]
                fetch = lo - (d.get("write_bytes_per_launch") or 0.0)
                hi = lo + fetch
                ck.append({"kernel": k, "ms_per_launch": round(ms, 4),
                           "launches": d.get("calls"),
                           "hbm_bytes_per_launch": [round(lo), round(hi)],
                           "achieved_gbs": [round(lo / (ms * 1e-3) / 1e9, 1),
                                            round(hi / (ms * 1e-3) / 1e9, 1)],
                           "frac_hbm": [round(lo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                        round(hi / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)],
                           "l2_requests_per_launch": d["l2_requests_per_launch"]})
            res["ct_apply"]["kernels"] = ck
            res["ct_apply"]["pmc_source"] = pe["source"]
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
