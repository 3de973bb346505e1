"""pkg/maps/lbmap mirror (cilium_amd/lbmap.py) on a host-only context: the
reference's Service4Key / Service4Value / RevNat4 layouts and byte order, and
UpdateService's slot layout (lbmap.go:351-427) with bpfservice.go's slot
cache, pinned by bpfservice_test.go."""
import struct

import numpy as np

from cilium_amd import lbmap, synth as S
from cilium_amd.datapath import host_only


def test_update_service_slots_and_byte_order():
    dp = host_only()
    m = lbmap.LBMap(dp)
    fe = lbmap.Service4Key("172.20.0.9", 80)
    bes = [lbmap.Service4Value(target="10.1.0.1", port=8080, rev_nat=7),
           lbmap.Service4Value(target="10.1.0.2", port=8080, rev_nat=7, weight=3)]
    m.UpdateService(fe, bes, add_revnat=True, revnat_id=7)
    k, v = dp.dump(m.svc)
    rows = {bytes(a): bytes(b) for a, b in zip(k, v)}
    assert len(rows) == 3
    vip = S.ip4("172.20.0.9")
    master = struct.pack("<IHH", vip, int(S.htons(80)), 0)
    # master slot: count 2 (host order), one non-zero weight (network order)
    assert struct.unpack("<IHHHH", rows[master]) == (0, 0, 2, 0, int(S.htons(1)))
    b1 = struct.pack("<IHH", vip, int(S.htons(80)), 1)
    t, port, cnt, rev, w = struct.unpack("<IHHHH", rows[b1])
    assert (t, port, cnt, rev) == (S.ip4("10.1.0.1"), int(S.htons(8080)), 0, int(S.htons(7)))
    k, v = dp.dump(m.rnat)
    assert bytes(k[0]) == struct.pack("<H", int(S.htons(7)))
    assert bytes(v[0]) == struct.pack("<IH", vip, int(S.htons(80)))
    # removing a backend keeps the slots: its slot becomes a hole holding
    # the remaining backend (bpfservice.go deleteBackend), the count stays
    m.UpdateService(fe, bes[:1], add_revnat=False)
    k, v = dp.dump(m.svc)
    rows = {bytes(a): bytes(b) for a, b in zip(k, v)}
    assert len(rows) == 3
    b2 = struct.pack("<IHH", vip, int(S.htons(80)), 2)
    assert rows[b2][:4] == struct.pack("<I", S.ip4("10.1.0.1"))
    assert struct.unpack("<IHHHH", rows[master])[2] == 2
    # the last backend gone, the service has no slots: the stale ones go
    m.UpdateService(fe, [], add_revnat=False)
    k, v = dp.dump(m.svc)
    assert len(k) == 1
    m.DeleteService(fe)
    k, v = dp.dump(m.svc)
    assert len(k) == 0
    dp.close()


def test_synth_rows_load():
    """synth.lb4_services rows go in as raw map bytes (loader.load_tables)."""
    rng = np.random.default_rng(3)
    t = S.config_c2(3, n_prefixes=500, n_policy=50, n_endpoints=2)
    lb, rn, vips, ports, protos = S.lb4_services(rng, t, n_services=12)
    dp = host_only()
    m = lbmap.LBMap(dp)
    m.load_rows(lb, rn)
    k, v = dp.dump(m.svc)
    assert len(k) == len(lb)
    got = sorted(bytes(a) + bytes(b) for a, b in zip(k, v))
    want = sorted(r.tobytes() for r in lb)
    assert got == want
    dp.close()


def test_lb_map_geometry_checked():
    """objCheck: the load balancer's maps only with the reference's geometry"""
    import errno
    import pytest
    dp = host_only()
    with pytest.raises(OSError) as e:
        dp.open_or_create_map("cilium_lb4_services", 1, 8, 16, 65536)
    assert e.value.errno == errno.EINVAL
    with pytest.raises(OSError):
        dp.open_or_create_map("cilium_lb4_reverse_nat", 1, 4, 6, 65536)
    dp.close()


def _be(ip):
    return lbmap.Service4Value(target=ip, port=80, rev_nat=1)


def test_scale_service():
    # bpfservice_test.go:41-116 (TestScaleService)
    svc = lbmap.BpfService(lbmap.Service4Key("1.1.1.1", 80))
    b1, b2, b3, b4 = (_be(x) for x in ("2.2.2.2", "3.3.3.3", "4.4.4.4", "5.5.5.5"))

    def slots():
        return {i: (b.bpfValue.String(), b.isHole) for i, b in svc.backendsByMapIndex.items()}
    svc.addBackend(b1)
    assert slots() == {1: (b1.String(), False)} and svc.holes == []
    svc.addBackend(b2)
    assert slots() == {1: (b1.String(), False), 2: (b2.String(), False)}
    svc.deleteBackend(b1)
    assert slots() == {1: (b2.String(), True), 2: (b2.String(), False)} and len(svc.holes) == 1
    svc.addBackend(b3)
    assert slots() == {1: (b3.String(), False), 2: (b2.String(), False)} and svc.holes == []
    svc.addBackend(b4)
    assert slots() == {1: (b3.String(), False), 2: (b2.String(), False),
                       3: (b4.String(), False)}
    svc.deleteBackend(b4)
    assert len(svc.backendsByMapIndex) == 3 and len(svc.holes) == 1
    assert slots()[1][0] == b3.String() and slots()[2][0] == b2.String()
    assert slots()[3][1] and slots()[3][0] in (b3.String(), b2.String())   # either fills
    svc.deleteBackend(b3)
    assert slots() == {1: (b2.String(), True), 2: (b2.String(), False),
                       3: (b2.String(), True)} and len(svc.holes) == 2
    svc.deleteBackend(b2)   # the last backend: every slot goes
    assert svc.backendsByMapIndex == {} and svc.holes == []
    svc.addBackend(b4)
    assert slots() == {1: (b4.String(), False)} and svc.holes == []


def test_prepare_update():
    # bpfservice_test.go:118-181 (TestPrepareUpdate)
    cache = lbmap.LBMapCache()
    fe = lbmap.Service4Key("1.1.1.1", 80)
    b1, b2, b3 = (_be(x) for x in ("2.2.2.2", "3.3.3.3", "4.4.4.4"))

    def ids(svc):
        return [b.String() for b in svc.getBackends()]
    assert ids(cache.prepareUpdate(fe, [b1, b2])) == [b1.String(), b2.String()]
    assert ids(cache.prepareUpdate(fe, [b1, b2, b3])) == [b1.String(), b2.String(), b3.String()]
    got = ids(cache.prepareUpdate(fe, [b2, b3]))
    assert len(got) == 3 and got[0] != b1.String() and got[1:] == [b2.String(), b3.String()]
    assert ids(cache.prepareUpdate(fe, [b1, b2, b3])) == [b1.String(), b2.String(), b3.String()]
    svc = cache.prepareUpdate(fe, [])
    assert svc.backendsByMapIndex == {} and svc.getBackends() == []
