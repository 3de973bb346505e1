"""Add the kernel's own ipcache longest-prefix match to every golden fixture.

TEST INFRASTRUCTURE ONLY (build container: needs bpf(2) and the reference
objects under oracle/_ref).  For each tests/golden/*.npz it creates
cilium_ipcache exactly as the reference's bpf_lxc.o defines it (LPM trie,
struct ipcache_key -> struct remote_endpoint_info, bpf/lib/maps.h:152-159),
fills it with the fixture's ipcache rows as the harness does
(gen_golden.RefDatapath), and stores, per header, the kernel's
BPF_MAP_LOOKUP_ELEM result for the header's source and destination address
(and, with services, the packet's translated addresses): x_lpm (n, 4) labels
and x_lpm_hit (n, 4).  The same lookup runs inside gen_golden.save() for
fixtures generated from now on; this script brings the existing ones up to
date without re-running their streams.

usage: python3 oracle/pin_lpm.py [fixture ...]
"""
import glob
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import bpf_harness as H   # noqa: E402
import gen_golden as GG   # noqa: E402


def pin(path):
    z = dict(np.load(path, allow_pickle=False))
    ipc = z["ipcache"]
    L = H.Loader({"cilium_ipcache": max(512000, len(ipc) + 16)})
    try:
        m = L.map_from_elf("bpf_lxc.o", "cilium_ipcache")
        for e in ipc:
            m.update(GG.ipcache_key(e), struct.pack("<II", int(e["label"]), int(e["tunnel"])))
        n = len(z["h_saddr"])
        h = _Hdr(int(z["h_family"]), z["h_saddr"], z["h_daddr"], n)
        lab, hit = GG.lpm_pin(m, h, z.get("x_pkt") if "lb4" in z else None)
    finally:
        L.close()
    z["x_lpm"], z["x_lpm_hit"] = lab, hit
    np.savez_compressed(path, **z)
    return n, hit.mean(axis=0)


class _Hdr:
    def __init__(self, family, saddr, daddr, n):
        self.family, self.saddr, self.daddr, self._n = family, saddr, daddr, n

    def __len__(self):
        return self._n


def main(names):
    paths = ([os.path.join(GG.GOLDEN, f"{x}.npz") for x in names] if names
             else sorted(glob.glob(os.path.join(GG.GOLDEN, "*.npz"))))
    for p in paths:
        n, rate = pin(p)
        print(f"{os.path.basename(p)}: {n} headers, hit rate per column "
              f"{np.round(rate, 3).tolist()}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
