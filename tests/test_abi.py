"""The C ABI library: loads, exports every symbol include/cfc.h declares, and
its map half behaves like the kernel BPF maps pkg/bpf drives (host-only
context, no GPU needed)."""
import ctypes
import errno
import os
import re
import struct

import numpy as np
import pytest

import cilium_amd as C
from cilium_amd import _lib, cidrmap, ipcache, lxcmap, metricsmap, policymap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "cfc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(cfc_\w+)\s*\(",
                                 txt, flags=re.M)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    fns = header_functions()
    assert len(fns) >= 18
    for f in fns:
        assert hasattr(L, f), f
    assert sorted(_lib.EXPORTS) == fns
    assert L.cfc_abi_version() == 13
    assert L.cfc_num_possible_cpus() == 1


def test_no_gpu_means_no_datapath():
    dp = C.host_only()
    with pytest.raises(OSError) as e:
        dp.commit()
    assert e.value.errno == errno.ENODEV


def test_stats_layout():
    """cfc_stats as the binding lays it out: cfc.h's fields in order, the
    ABI-13 field (ct_self_segments) last, the u64 totals 8-byte aligned;
    before the first commit (a host-only context never has one) the call
    returns -ENOENT"""
    txt = open(os.path.join(ROOT, "include", "cfc.h")).read()
    body = txt[txt.index("uint64_t epoch;"):txt.index("} cfc_stats;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"^\s*u?int\d+_t\s+(\w+);", body, flags=re.M)
    assert [f for f, _ in _lib.Stats._fields_] == names
    assert names[-1] == "ct_self_segments"
    for f, t in _lib.Stats._fields_:
        if t is ctypes.c_uint64:
            assert getattr(_lib.Stats, f).offset % 8 == 0, f
    assert errno_of(C.host_only().stats) == errno.ENOENT


def test_options_on_host_only_context():
    """The ipcache layout is a table option (it applies at the next commit);
    timing needs a device."""
    dp = C.host_only()
    for v in (_lib.LPM4_AUTO, _lib.LPM4_DIR24_8, _lib.LPM4_TRIE):
        dp.set_option(_lib.OPT_LPM4, v)
    assert errno_of(lambda: dp.set_option(_lib.OPT_LPM4, 3)) == errno.EINVAL
    assert errno_of(lambda: dp.set_option(99, 0)) == errno.EINVAL
    assert errno_of(lambda: dp.set_option(_lib.OPT_TIMING, 1)) == errno.ENODEV
    assert errno_of(dp.timing_collect) == errno.ENODEV


def test_node_config_on_host_only_context():
    """cfc_set/get_node_config: starts at bpf/node_config.h's values
    (IPV4_CLUSTER_RANGE 0x100000, MASK 0xff0000, ROUTER_IP beef::1:0:1:0:0)."""
    dp = C.host_only()
    rng, mask, router, hif = dp.node_config()
    assert (rng, mask, hif) == (0x100000, 0xFF0000, 1)
    assert router == bytes([0xbe, 0xef] + [0] * 9 + [1, 0, 1, 0, 0])
    dp.set_node_config(0x0A, 0xFF, bytes(range(16)), 7)
    assert dp.node_config() == (0x0A, 0xFF, bytes(range(16)), 7)
    dp.set_clock(12345)


def errno_of(fn):
    with pytest.raises(OSError) as e:
        fn()
    return e.value.errno


def test_hash_map_semantics():
    dp = C.host_only()
    fd, new = dp.open_or_create_map("/sys/fs/bpf/tc/globals/test_hash", 1, 4, 8, 2)
    assert new
    k1, k2, k3 = (struct.pack("<I", i) for i in (1, 2, 3))
    dp.update_element(fd, k1, b"a" * 8)
    assert errno_of(lambda: dp.update_element(fd, k1, b"b" * 8, 1)) == errno.EEXIST
    assert errno_of(lambda: dp.update_element(fd, k2, b"b" * 8, 2)) == errno.ENOENT
    dp.update_element(fd, k2, b"b" * 8, 1)
    assert errno_of(lambda: dp.update_element(fd, k3, b"c" * 8)) == errno.E2BIG
    dp.update_element(fd, k1, b"z" * 8, 2)                 # replace in place
    assert dp.lookup_element(fd, k1) == b"z" * 8
    assert dp.lookup_element(fd, k3) is None
    assert sorted(dp.keys(fd)) == [k1, k2]
    assert dp.get_next_key(fd, k3) in (k1, k2)              # unknown -> first
    dp.delete_element(fd, k1)
    assert errno_of(lambda: dp.delete_element(fd, k1)) == errno.ENOENT
    # reopen with a different geometry: objCheck refuses (bpf.go:306)
    assert errno_of(lambda: dp.open_or_create_map(
        "/sys/fs/bpf/tc/globals/test_hash", 1, 4, 16, 2)) == errno.EINVAL
    fd2, new2 = dp.open_or_create_map("/sys/fs/bpf/tc/globals/test_hash", 1, 4, 8, 2)
    assert not new2 and dp.lookup_element(fd2, k2) == b"b" * 8
    dp.obj_close(fd2)
    assert errno_of(lambda: dp.obj_close(fd2)) == errno.EBADF


def test_lpm_map_semantics():
    dp = C.host_only()
    fd, _ = dp.open_or_create_map("lpm_test", 11, 8, 1, 3, 1)

    def key(cidr):
        a, p = cidr.split("/")
        return struct.pack("<I", int(p)) + bytes(int(x) for x in a.split("."))
    dp.update_element(fd, key("10.0.0.0/8"), b"\x08")
    dp.update_element(fd, key("10.1.0.0/16"), b"\x10")
    dp.update_element(fd, key("10.1.2.3/16"), b"\x11")    # same prefix: replace
    assert len(dp.keys(fd)) == 2
    assert dp.lookup_element(fd, key("10.1.9.9/32")) == b"\x11"
    assert dp.lookup_element(fd, key("10.2.9.9/32")) == b"\x08"
    assert dp.lookup_element(fd, key("10.1.9.9/12")) == b"\x08"  # bounded by key len
    assert dp.lookup_element(fd, key("11.0.0.1/32")) is None
    assert errno_of(lambda: dp.update_element(fd, key("1.2.3.4/33"), b"\x00")) == errno.EINVAL
    dp.update_element(fd, key("0.0.0.0/0"), b"\x00")
    assert errno_of(lambda: dp.update_element(fd, key("9.0.0.0/8"), b"\x00")) == errno.ENOSPC
    assert dp.lookup_element(fd, key("11.0.0.1/32")) == b"\x00"
    assert errno_of(lambda: dp.delete_element(fd, key("10.0.0.0/9"))) == errno.ENOENT


def test_role_geometry_is_checked():
    dp = C.host_only()
    assert errno_of(lambda: dp.open_or_create_map("cilium_policy_7", 1, 8, 16, 10)) == errno.EINVAL
    assert errno_of(lambda: dp.open_or_create_map("cilium_ipcache", 1, 24, 8, 10)) == errno.EINVAL
    dp.open_or_create_map("cilium_policy_7", 1, 8, 24, 16384)


def test_policymap_mirror():
    dp = C.host_only()
    pm, new = policymap.OpenMap(dp, policymap.path_for(4112))
    assert new
    pm.Allow(1000, 80, 6, policymap.Ingress, 0)
    pm.Allow(1000, 0, 0, policymap.Ingress)
    pm.Allow(0, 53, 17, policymap.Egress, 10001)
    assert pm.Exists(1000, 80, 6, 0) and not pm.Exists(1000, 81, 6, 0)
    d = {x.Key.ToHost(): x.PolicyEntry for x in pm.DumpToSlice()}
    k = policymap.PolicyKey(0, 53, 17, 1)
    assert d[k].ProxyPort == 0x1127        # htons(10001), network order
    # raw layout: identity LE, port network order, proto, direction
    raw = policymap.PolicyKey(1000, 80, 6, 0).ToNetwork().pack()
    assert raw == struct.pack("<I", 1000) + b"\x00\x50" + b"\x06\x00"
    # PolicyKey.String (policymap.go:108-115), on the stored (network) key
    assert policymap.PolicyKey(1000, 0x5000, 6, 0).String() == "Ingress: 1000 80/6"
    assert policymap.PolicyKey(2, 0, 0, 1).String() == "Egress: 2"
    # the display order (policymap_test.go:31-108): direction, then identity
    E = policymap.PolicyEntry()

    def dump(*keys):
        return policymap.PolicyEntriesDump(policymap.PolicyEntryDump(
            policymap.PolicyKey(i, 0, 0, d), E) for i, d in keys)
    assert not dump((0, 0)).Less(0, 0)
    assert dump((0, 0), (1, 0)).Less(0, 1)
    assert dump((0, 0), (1, 1)).Less(0, 1)
    assert not dump((1, 1), (0, 1)).Less(0, 1)
    ds = policymap.PolicyEntriesDump(pm.DumpToSlice())
    ds.Sort()
    assert [(e.Key.TrafficDirection, e.Key.Identity) for e in ds] == [(0, 1000), (0, 1000), (1, 0)]
    pm.Delete(1000, 80, 6, 0)
    assert not pm.Exists(1000, 80, 6, 0)
    pm.Flush()
    assert pm.DumpToSlice() == []


def test_ipcache_and_lxc_mirrors():
    dp = C.host_only()
    m = ipcache.Map(dp)
    m.Update(ipcache.NewKey("10.0.0.0/8"), ipcache.RemoteEndpointInfo(42))
    m.Update(ipcache.NewKey("10.1.0.0/16"), ipcache.RemoteEndpointInfo(43))
    m.Update(ipcache.NewKey("f00d::/64"), ipcache.RemoteEndpointInfo(44))
    assert m.Lookup(ipcache.NewKey("10.1.2.3/32")).SecurityIdentity == 43
    assert m.Lookup(ipcache.NewKey("10.9.2.3/32")).SecurityIdentity == 42
    assert m.Lookup(ipcache.NewKey("f00d::1/128")).SecurityIdentity == 44
    assert m.Lookup(ipcache.NewKey("11.0.0.1/32")) is None
    k = ipcache.NewKey("10.1.0.0/16")
    assert k.Prefixlen == 48 and k.pack()[:8] == struct.pack("<IHBB", 48, 0, 0, 1)
    assert sorted(x.String() for x in m.Dump()) == ["10.0.0.0/8", "10.1.0.0/16",
                                                     "f00d::/64"]
    lx = lxcmap.LXCMap(dp)
    lx.WriteEndpoint([lxcmap.NewEndpointKey("10.0.0.1"),
                      lxcmap.NewEndpointKey("f00d::1")],
                     lxcmap.EndpointInfo(IfIndex=5, LxcID=0x1010))
    lx.AddHostEntry("10.0.255.254")
    assert lx.Lookup("f00d::1").LxcID == 0x1010
    assert lx.Lookup("10.0.255.254").IsHost()
    assert len(lxcmap.EndpointInfo().pack()) == 48


def test_prefilter_revisions_and_rollback():
    dp = C.host_only()
    pf = cidrmap.PreFilter(dp)
    pf.Insert(1, ["1.2.3.4/32", "::1/128"])
    cidrs, rev = pf.Dump()
    assert rev == 2 and sorted(cidrs) == ["1.2.3.4/32", "::1/128"]
    with pytest.raises(ValueError):
        pf.Insert(1, ["5.5.5.5/32"])                     # stale revision
    with pytest.raises(ValueError):
        pf.Insert(2, ["6.6.6.6/32", "7.7.7.0/24"])       # dyn map disabled
    assert sorted(pf.Dump()[0]) == ["1.2.3.4/32", "::1/128"]   # rolled back
    with pytest.raises(ValueError):
        pf.Delete(2, ["1.2.3.4/32", "8.8.8.8/32"])       # all-or-nothing
    pf.Delete(2, ["1.2.3.4/32"])
    assert pf.Dump() == (["::1/128"], 3)


def test_metrics_map_owned_by_datapath():
    dp = C.host_only()
    fd = metricsmap.open_map(dp)
    assert metricsmap.dump(dp, fd) == {}
    # geometry of the datapath-owned map is fixed
    with pytest.raises(OSError):
        dp.open_or_create_map("cilium_metrics", 1, 8, 16, 65536)


def test_flattener_selftest():
    """The IPv6 LPM image (Bloom groups, hash slots) answers like a brute-force
    longest-prefix match, the self-traffic cut rule, and the prefix masks
    against test/bpf/unit-test.c's ipv6_addr_clear_suffix known answers, and
    the host map store (HASH, LPM_TRIE) against a model under random
    operations, and both IPv4 LPM layouts (DIR-24-8, the compact multibit
    trie) through host restatements of the device lookups against a
    brute-force longest-prefix match (cilium_amd/csrc/selftest.cpp, host
    only)."""
    import subprocess
    csrc = os.path.join(ROOT, "cilium_amd", "csrc")
    exe = os.path.join(csrc, "build", "selftest")
    # (make is incremental: a binary older than its sources is rebuilt)
    subprocess.run(["make", "-C", csrc, "-s", "selftest"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok") == 16 and "FAIL" not in r.stdout, r.stdout


def test_ct_maps_host_only():
    """pkg/maps/ctmap names and geometry; bulk load; the oracle-format dump
    returns what was loaded (golden fixture CT state)."""
    import golden_io as G
    from cilium_amd import loader
    g = G.Golden("ct_ingress_v4")
    dp = C.host_only()
    fds = loader.load_ct(dp, g.tables)
    rows = loader.ct_rows(dp, fds)
    want = np.zeros((len(g.tables.ct), 104), np.uint8)
    ct = g.tables.ct
    want[:, 0:2] = np.stack([(ct["lxc"] + 1) & 0xFF, (ct["lxc"] + 1) >> 8], 1)
    want[:, 2] = ct["any"]
    want[:, 3] = ct["family"]
    want[:, 4:42] = ct["tuple"]
    want[:, 44:100] = ct["entry"]
    want = want[np.lexsort(want[:, :44].T[::-1])]
    np.testing.assert_array_equal(rows, want)
    # wrong geometry for a CT role
    with pytest.raises(OSError) as e:
        dp.open_or_create_map("cilium_ct4_global", 9, 16, 56, 1024)
    assert e.value.errno == errno.EINVAL
    fd, new = dp.open_or_create_map("cilium_ct_any6_77", 9, 38, 56, 1024)
    assert new


def test_drop_notify_abi_on_host_only_context():
    """cfc_drop_notify_v4/v6 validate their arguments and need a device; the
    record layout is pkg/monitor's DropNotify (datapath_drop.go:28-40)."""
    import ctypes
    import numpy as np
    import oracle as O
    dp = C.host_only()
    L = dp.L
    hdr = _lib.HdrV4(None, None, None, None, None, None, 0)
    cnt = ctypes.c_uint64(0)
    out = _lib.Out()
    for fn in (L.cfc_drop_notify_v4, L.cfc_drop_notify_v6):
        assert fn(dp.h, ctypes.byref(hdr), ctypes.byref(out), 0, 0, None, None,
                  0, ctypes.byref(cnt), None) == -errno.ENODEV
        assert fn(dp.h, ctypes.byref(hdr), ctypes.byref(out), 0, 0, None, None,
                  0, None, None) == -errno.EINVAL
        assert fn(dp.h, ctypes.byref(hdr), ctypes.byref(out), 9, 0, None, None,
                  0, ctypes.byref(cnt), None) == -errno.EINVAL
    # Out carries eight device pointers (cfc_out, ABI 7: + the packet's
    # rewritten addresses); cfc_hdr_v4 gained skb->hash
    assert ctypes.sizeof(_lib.Out) == 64
    assert ctypes.sizeof(_lib.HdrV4) == 64 and ctypes.sizeof(_lib.HdrV6) == 64
    dt = O.DROP_NOTIFY_DT
    assert dt.itemsize == 32
    assert [dt.fields[k][1] for k in dt.names] == [0, 1, 2, 4, 8, 12, 16, 20, 24, 28]
    assert np.zeros(1, dt).view(np.uint8).size == 32


def test_c_abi_from_c(tmp_path):
    """include/cfc.h under a C11 compiler (-Werror) and the pkg/bpf call
    sequence from C on a host-only context (tests/c/abi_host.c): what a cgo
    shim compiles and calls."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / "abi_host")
    lib = os.path.join(ROOT, "cilium_amd")
    subprocess.run(["gcc", "-std=c11", "-pedantic", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "include"), "-o", exe,
                    os.path.join(ROOT, "tests", "c", "abi_host.c"), "-L", lib, "-lcfc",
                    f"-Wl,-rpath,{lib}"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "abi_host: ok" in r.stdout, r.stdout + r.stderr
    # the header alone under a C++11 compiler too (a C++ host binds it as is)
    if shutil.which("g++"):
        src = tmp_path / "h.cpp"
        src.write_text('#include "cfc.h"\nint main() { return cfc_abi_version() != '
                       'CFC_ABI_VERSION; }\n')
        subprocess.run(["g++", "-std=c++11", "-pedantic", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(ROOT, "include"), "-fsyntax-only", str(src)],
                       check=True)
