"""Run the reference's own BPF datapath with BPF_PROG_TEST_RUN.

TEST INFRASTRUCTURE ONLY (golden-vector generation in this container).
Nothing in cilium_amd/ imports this; it never runs on the GPU box.

It loads the objects built by oracle/Makefile from the reference sources
(bpf/bpf_xdp.c, bpf/bpf_netdev.c, bpf/bpf_lxc.c) into the running kernel:

* ELF maps section entries are `struct bpf_elf_map`
  (reference bpf/include/iproute2/bpf_elf.h): type, size_key, size_value,
  max_elem, flags, ... -> BPF_MAP_CREATE.  Maps are shared by name across
  programs (the pinning the reference relies on, bpf/lib/maps.h:31), except
  for per-endpoint maps that are renamed per endpoint instance.
* R_BPF_64_64 relocations against map symbols are patched to
  BPF_PSEUDO_MAP_FD ld_imm64 instructions.
* Tail calls are wired by filling the prog-array maps exactly as the agent
  does: cilium_calls_<id>[CILIUM_CALL_*] (bpf/lib/common.h:45-57) and
  cilium_policy[LXC_ID] (bpf/lib/maps.h, bpf/lib/l3.h:130).
"""
import ctypes
import os
import struct

_libc = ctypes.CDLL(None, use_errno=True)
_NR_bpf = 321

BPF_MAP_CREATE, BPF_MAP_LOOKUP_ELEM, BPF_MAP_UPDATE_ELEM = 0, 1, 2
BPF_MAP_DELETE_ELEM, BPF_MAP_GET_NEXT_KEY, BPF_PROG_LOAD = 3, 4, 5
BPF_PROG_TEST_RUN = 10

PROG_SCHED_CLS, PROG_XDP = 3, 6
MAP_PERCPU_HASH = 5
SKB_CTX_SIZE = 192          # sizeof(struct __sk_buff) on 6.x kernels
SKB_OFF_MARK, SKB_OFF_CB = 8, 48

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")


class BpfError(OSError):
    pass


def _bpf(cmd, attr: bytes, size=144):
    buf = ctypes.create_string_buffer(attr, size)
    r = _libc.syscall(_NR_bpf, cmd, buf, size)
    if r < 0:
        e = ctypes.get_errno()
        raise BpfError(e, f"bpf cmd {cmd}: {os.strerror(e)}")
    return r, buf


def ncpus_possible():
    txt = open("/sys/devices/system/cpu/possible").read().strip()
    hi = int(txt.split("-")[-1]) if "-" in txt else int(txt)
    return hi + 1


class Map:
    def __init__(self, name, mtype, ksz, vsz, max_elem, flags):
        self.name, self.type, self.ksz, self.vsz = name, mtype, ksz, vsz
        attr = struct.pack("<IIIII", mtype, ksz, vsz, max_elem, flags)
        self.fd, _ = _bpf(BPF_MAP_CREATE, attr)

    @property
    def percpu(self):
        return self.type == MAP_PERCPU_HASH

    def _vlen(self):
        if self.percpu:
            return ((self.vsz + 7) // 8) * 8 * ncpus_possible()
        return self.vsz

    def update(self, key: bytes, value: bytes, flags=0):
        assert len(key) == self.ksz, (self.name, len(key), self.ksz)
        assert len(value) == self.vsz or self.percpu, (self.name, len(value))
        kb = ctypes.create_string_buffer(key, len(key))
        vb = ctypes.create_string_buffer(value, max(len(value), self._vlen()))
        _bpf(BPF_MAP_UPDATE_ELEM, struct.pack(
            "<IIQQQ", self.fd, 0, ctypes.addressof(kb), ctypes.addressof(vb),
            flags))

    def delete(self, key: bytes):
        kb = ctypes.create_string_buffer(key, len(key))
        _bpf(BPF_MAP_DELETE_ELEM, struct.pack("<IIQ", self.fd, 0,
                                              ctypes.addressof(kb)))

    def lookup(self, key: bytes):
        kb = ctypes.create_string_buffer(key, len(key))
        vb = ctypes.create_string_buffer(self._vlen())
        try:
            _bpf(BPF_MAP_LOOKUP_ELEM, struct.pack(
                "<IIQQQ", self.fd, 0, ctypes.addressof(kb),
                ctypes.addressof(vb), 0))
        except BpfError:
            return None
        return vb.raw

    def keys(self):
        out, prev = [], None
        nk = ctypes.create_string_buffer(self.ksz)
        while True:
            if prev is None:
                pk = 0
            else:
                pkb = ctypes.create_string_buffer(prev, self.ksz)
                pk = ctypes.addressof(pkb)
            try:
                _bpf(BPF_MAP_GET_NEXT_KEY, struct.pack(
                    "<IIQQ", self.fd, 0, pk, ctypes.addressof(nk)))
            except BpfError:
                return out
            prev = nk.raw
            out.append(prev)

    def close(self):
        if self.fd >= 0:
            os.close(self.fd)
            self.fd = -1


class _Elf:
    def __init__(self, path):
        self.d = d = open(path, "rb").read()
        shoff, = struct.unpack_from("<Q", d, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, 0x3A)
        self.secs = []
        for i in range(shnum):
            f = struct.unpack_from("<IIQQQQIIQQ", d, shoff + i * shentsize)
            self.secs.append(dict(name=f[0], type=f[1], off=f[4], size=f[5],
                                  link=f[6], info=f[7]))
        strtab = self.secs[shstrndx]
        for s in self.secs:
            s["nm"] = self._str(strtab, s["name"])
        symtab = [s for s in self.secs if s["type"] == 2][0]
        strs = self.secs[symtab["link"]]
        self.syms = []
        for i in range(symtab["size"] // 24):
            n, _, _, shndx, val, _ = struct.unpack_from(
                "<IBBHQQ", d, symtab["off"] + i * 24)
            self.syms.append((self._str(strs, n), shndx, val))
        self.maps_sec = [i for i, s in enumerate(self.secs)
                         if s["nm"] == "maps"][0]

    def _str(self, tab, off):
        s = self.d[tab["off"] + off:]
        return s[:s.index(b"\0")].decode()

    def section(self, name):
        for i, s in enumerate(self.secs):
            if s["nm"] == name:
                return i, s
        raise KeyError(name)

    def mapdef(self, sym_val):
        off = self.secs[self.maps_sec]["off"] + sym_val
        return struct.unpack_from("<IIIII", self.d, off)


class Loader:
    """Loads programs, sharing maps by (renamed) name in `self.maps`."""

    def __init__(self, max_elem_override=None):
        self.maps = {}
        self.max_elem = dict(max_elem_override or {})
        self._keep = []
        self.progs = []
        self._elf_cache = {}

    def _elf(self, obj):
        if obj not in self._elf_cache:
            self._elf_cache[obj] = _Elf(os.path.join(REF_DIR, obj))
        return self._elf_cache[obj]

    def map_from_elf(self, obj, name):
        """Create (or return) map `name` exactly as obj's maps section
        defines it (struct bpf_elf_map), without loading any program."""
        if name not in self.maps:
            elf = self._elf(obj)
            val = next(v for n, sh, v in elf.syms if n == name and sh == elf.maps_sec)
            t, ks, vs, me, fl = elf.mapdef(val)
            self.maps[name] = Map(name, t, ks, vs, self.max_elem.get(name, me), fl)
        return self.maps[name]

    def load(self, obj, section, prog_type, rename=None):
        rename = rename or {}
        elf = self._elf(obj)
        idx, sec = elf.section(section)
        insns = bytearray(elf.d[sec["off"]:sec["off"] + sec["size"]])
        for rs in (s for s in elf.secs if s["type"] == 9 and s["info"] == idx):
            for i in range(rs["size"] // 16):
                off, info = struct.unpack_from("<QQ", elf.d, rs["off"] + i * 16)
                name, shndx, val = elf.syms[info >> 32]
                if shndx != elf.maps_sec:
                    raise RuntimeError(f"unexpected relocation to {name}")
                mname = rename.get(name, name)
                if mname not in self.maps:
                    t, ks, vs, me, fl = elf.mapdef(val)
                    me = self.max_elem.get(name, me)
                    self.maps[mname] = Map(mname, t, ks, vs, me, fl)
                ins = bytearray(insns[off:off + 8])
                ins[1] = (ins[1] & 0x0F) | (1 << 4)     # src_reg = PSEUDO_MAP_FD
                insns[off:off + 8] = ins
                struct.pack_into("<i", insns, off + 4, self.maps[mname].fd)
        log = ctypes.create_string_buffer(1 << 22)
        ib = ctypes.create_string_buffer(bytes(insns))
        lic = ctypes.create_string_buffer(b"GPL")
        attr = struct.pack("<IIQQIIQI", prog_type, len(insns) // 8,
                           ctypes.addressof(ib), ctypes.addressof(lic), 1,
                           1 << 22, ctypes.addressof(log), 0)
        try:
            fd, _ = _bpf(BPF_PROG_LOAD, attr)
        except BpfError as e:
            raise BpfError(e.errno, f"load {obj}:{section}: "
                           + log.value.decode(errors="replace")[-2000:])
        self._keep.append((ib, lic))
        self.progs.append(fd)
        return fd

    def close(self):
        for m in self.maps.values():
            m.close()
        for fd in self.progs:
            os.close(fd)
        self.maps.clear()
        self.progs.clear()


# ------------------------------------------------------------ perf ring
# The datapath's notifications go to the perf event array cilium_events
# (bpf/lib/events.h:23-29) through skb_event_output(..., BPF_F_CURRENT_CPU):
# send_trace_notify (trace.h:97-155) and __send_drop_notify (drop.h:50-78).
# PerfRing opens a PERF_COUNT_SW_BPF_OUTPUT event on one CPU, maps its ring
# and hands out the raw samples; the caller pins itself to that CPU so every
# BPF_PROG_TEST_RUN lands there.
_NR_perf_event_open = 298
PERF_TYPE_SOFTWARE, PERF_COUNT_SW_BPF_OUTPUT = 1, 10
PERF_SAMPLE_RAW = 1 << 10
PERF_RECORD_LOST, PERF_RECORD_SAMPLE = 2, 9
PERF_FLAG_FD_CLOEXEC = 8


def pin_cpu():
    """Pin this process to its first allowed CPU (< __NR_CPUS__ 8, the size
    of cilium_events) and return it."""
    cpu = min(c for c in os.sched_getaffinity(0) if c < 8)
    os.sched_setaffinity(0, {cpu})
    return cpu


class PerfRing:
    def __init__(self, cpu, pages=256):
        import mmap
        self.cpu = cpu
        attr = bytearray(128)
        struct.pack_into("<IIQQQ", attr, 0, PERF_TYPE_SOFTWARE, 128,
                         PERF_COUNT_SW_BPF_OUTPUT, 1, PERF_SAMPLE_RAW)
        struct.pack_into("<I", attr, 48, 1)        # wakeup_events
        ab = ctypes.create_string_buffer(bytes(attr), 128)
        fd = _libc.syscall(_NR_perf_event_open, ab, -1, cpu, -1,
                           PERF_FLAG_FD_CLOEXEC)
        if fd < 0:
            e = ctypes.get_errno()
            raise BpfError(e, f"perf_event_open: {os.strerror(e)}")
        self.fd = fd
        self.psz = mmap.PAGESIZE
        self.size = pages * self.psz
        self.mm = mmap.mmap(fd, self.psz + self.size, mmap.MAP_SHARED,
                            mmap.PROT_READ | mmap.PROT_WRITE)
        self.lost = 0

    def read(self):
        """-> list of raw sample payloads (bytes) since the last read."""
        mm = self.mm
        head, = struct.unpack_from("<Q", mm, 1024)
        tail, = struct.unpack_from("<Q", mm, 1032)
        out = []
        base = self.psz
        while tail < head:
            off = tail % self.size
            hdr = self._bytes(base, off, 8)
            typ, misc, sz = struct.unpack("<IHH", hdr)
            rec = self._bytes(base, off, sz)
            if typ == PERF_RECORD_SAMPLE:
                n, = struct.unpack_from("<I", rec, 8)
                out.append(rec[12:12 + n])
            elif typ == PERF_RECORD_LOST:
                self.lost += struct.unpack_from("<Q", rec, 16)[0]
            tail += sz
        struct.pack_into("<Q", mm, 1032, tail)
        return out

    def _bytes(self, base, off, n):
        a = self.mm[base + off: base + min(off + n, self.size)]
        if len(a) < n:
            a += self.mm[base: base + n - len(a)]
        return bytes(a)

    def close(self):
        self.mm.close()
        os.close(self.fd)


def test_run_skb(prog_fd, pkt: bytes, mark=0, cb=(0, 0, 0, 0, 0)):
    """One BPF_PROG_TEST_RUN of a tc program. Returns (retval, cb_out, pkt_out)."""
    pin = ctypes.create_string_buffer(pkt, len(pkt))
    pout = ctypes.create_string_buffer(len(pkt) + 512)
    ctx = bytearray(SKB_CTX_SIZE)
    struct.pack_into("<I", ctx, SKB_OFF_MARK, mark)
    struct.pack_into("<5I", ctx, SKB_OFF_CB, *cb)
    cin = ctypes.create_string_buffer(bytes(ctx), SKB_CTX_SIZE)
    cout = ctypes.create_string_buffer(SKB_CTX_SIZE)
    attr = struct.pack("<IIIIQQIIIIQQ", prog_fd, 0, len(pkt), len(pout),
                       ctypes.addressof(pin), ctypes.addressof(pout), 1, 0,
                       SKB_CTX_SIZE, SKB_CTX_SIZE, ctypes.addressof(cin),
                       ctypes.addressof(cout))
    _, b = _bpf(BPF_PROG_TEST_RUN, attr)
    f = struct.unpack_from("<IIIIQQIIIIQQ", b.raw, 0)
    retval, out_size = f[1], f[3]
    cbo = struct.unpack_from("<5i", cout.raw, SKB_OFF_CB)
    return retval, cbo, pout.raw[:out_size]


def test_run_xdp(prog_fd, pkt: bytes):
    pin = ctypes.create_string_buffer(pkt, len(pkt))
    pout = ctypes.create_string_buffer(len(pkt) + 512)
    attr = struct.pack("<IIIIQQII", prog_fd, 0, len(pkt), len(pout),
                       ctypes.addressof(pin), ctypes.addressof(pout), 1, 0)
    _, b = _bpf(BPF_PROG_TEST_RUN, attr)
    return struct.unpack_from("<IIIIQQII", b.raw, 0)[1]


def test_run_duration(prog_fd, pkt: bytes, mark=0, xdp=False):
    """One BPF_PROG_TEST_RUN (repeat 1) -> (retval, in-kernel ns).  The
    kernel's `duration` covers the program and its tail calls, not the
    syscall around them."""
    pin = ctypes.create_string_buffer(pkt, len(pkt))
    pout = ctypes.create_string_buffer(len(pkt) + 512)
    if xdp:
        attr = struct.pack("<IIIIQQII", prog_fd, 0, len(pkt), len(pout),
                           ctypes.addressof(pin), ctypes.addressof(pout), 1, 0)
        _, b = _bpf(BPF_PROG_TEST_RUN, attr)
        f = struct.unpack_from("<IIIIQQII", b.raw, 0)
        return f[1], f[7]
    ctx = bytearray(SKB_CTX_SIZE)
    struct.pack_into("<I", ctx, SKB_OFF_MARK, mark)
    cin = ctypes.create_string_buffer(bytes(ctx), SKB_CTX_SIZE)
    cout = ctypes.create_string_buffer(SKB_CTX_SIZE)
    attr = struct.pack("<IIIIQQIIIIQQ", prog_fd, 0, len(pkt), len(pout),
                       ctypes.addressof(pin), ctypes.addressof(pout), 1, 0,
                       SKB_CTX_SIZE, SKB_CTX_SIZE, ctypes.addressof(cin),
                       ctypes.addressof(cout))
    _, b = _bpf(BPF_PROG_TEST_RUN, attr)
    f = struct.unpack_from("<IIIIQQIIIIQQ", b.raw, 0)
    return f[1], f[7]
