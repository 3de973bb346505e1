"""Cost of drop notifications at C2 scale (GPU box): the classify kernel with
and without the per-header notify store, and cfc_drop_notify_v4 (count +
scan + write kernels) over the same 64M-header batch.  Prints one JSON line.

  python3 scripts/bench_notify.py [--headers N] [--mode full|ingress|egress]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--headers", type=int, default=64 << 20)
    ap.add_argument("--mode", default="full")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    from cilium_amd import synth as S
    from cilium_amd.datapath import Datapath, HeaderBatchV4, Verdicts
    from cilium_amd.loader import load_tables

    mode = {"ingress": 0, "egress": 1, "full": 3}[a.mode]
    ep = S.EP_LXC_ID if mode == 1 else 0
    dev = torch.device("cuda", 0)
    t = S.config_c2_bench(2)
    dp = Datapath(0)
    load_tables(dp, t)
    n = a.headers
    s, d, p, m = S.gen_batch_v4_torch(t, n, 2000, dev)
    if mode == 1:
        s.fill_(S.LXC_IPV4 - (1 << 32) if S.LXC_IPV4 >= 1 << 31 else S.LXC_IPV4)
    b = HeaderBatchV4(s, d, p, m, None)
    mk = lambda nt: Verdicts(torch.empty(n, dtype=torch.int32, device=dev),   # noqa: E731
                             torch.empty(n, dtype=torch.int32, device=dev), None,
                             None, torch.empty(n, dtype=torch.int32, device=dev) if nt else None)
    o0, o1 = mk(False), mk(True)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            r = fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps, r

    ms_plain, _ = timed(lambda: dp.classify_v4(b, mode, ep, out=o0))
    ms_nt, _ = timed(lambda: dp.classify_v4(b, mode, ep, out=o1))
    # drop_notify synchronises to read the total: time it with one sync per
    # call included (a lower bound on the kernels' rate)
    ms_dn, (rec, idx, total) = timed(lambda: dp.drop_notify(b, o1, mode, ep))
    # algorithmic bytes: notify word read twice (count, write) per header;
    # per record the verdict, identity, meta, ports, saddr, daddr reads and
    # the 32-byte record + 8-byte index writes
    bytes_dn = 8 * n + total * (6 * 4 + 32 + 8)
    print(json.dumps({
        "workload": f"C2 bench tables, {n} headers, mode {a.mode}",
        "classify_ms": round(ms_plain, 4), "classify_notify_ms": round(ms_nt, 4),
        "drop_notify_ms": round(ms_dn, 4), "records": int(total),
        "drop_notify_GBps": round(bytes_dn / ms_dn / 1e6, 1),
        "drop_notify_bytes": int(bytes_dn)}))
    dp.close()


if __name__ == "__main__":
    main()
