"""The global loads and waits of one kernel in a hipcc -S listing, in
order: a quick check that a kernel issues its loads together (one
s_waitcnt vmcnt per batch) rather than one wait per load.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S \\
        -o /tmp/x.s cilium_amd/csrc/ctapply.hip
    python scripts/isa_loads.py /tmp/x.s k_ct_gc4 [N]
"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    for m in re.finditer(r"^(_Z\S*" + re.escape(sys.argv[2]) + r"\S*):", s, re.M):
        st = m.end()
        body = s[st:s.index(".Lfunc_end", st)].splitlines()
        seq = []
        for ln in body:
            t = ln.strip()
            if t.startswith(("global_load", "global_atomic", "s_waitcnt vmcnt", "global_store")):
                seq.append(t.split()[0] + (t[t.index("("):t.index(")") + 1] if "vmcnt" in t else ""))
        print(m.group(1)[:90], f"({len(body)} lines)")
        print(" ".join(seq[:n]))


if __name__ == "__main__":
    main()
