"""Unit tests of the replay building blocks (include/nrgpu_testing.h) against numpy:
the stable LSD radix sort (decoupled look-back, one launch per 8-bit digit) and the
max-scan used by the synthetic replay."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sort(nrg, dev, keys, vals, bits):
    import torch

    n = len(keys)
    dk = torch.from_numpy(keys.view(np.int32).copy()).cuda()
    dv = torch.from_numpy(vals.view(np.int32).copy()).cuda() if vals is not None else None
    ok = torch.empty(n, dtype=torch.int32, device="cuda")
    ov = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    nrg._lib.check(nrg.load().nrg_test_sort_pairs(dev.handle, dk.data_ptr(), dv.data_ptr() if dv is not None else None,
                                                  n, bits, ok.data_ptr(), ov.data_ptr()))
    return ok.cpu().numpy().view(np.uint32), ov.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,bits,span", [(1, 8, 5), (2047, 8, 3), (2048, 12, 4000), (6000, 18, 7),
                                         (100_000, 19, 300_000), (300_001, 24, 1 << 24), (50_000, 32, 1 << 32),
                                         (70_000, 18, 1)])
def test_radix_sort_stable(nrg, orc, n, bits, span):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1 << 19)
    keys = (orc.gen_uniform(n, n + bits, span) & ((1 << bits) - 1)).astype(np.uint32)
    vals = orc.gen_raw(n, 5).astype(np.uint32)
    sk, sv = _sort(nrg, dev, keys, vals, bits)
    o = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(sk, keys[o])
    np.testing.assert_array_equal(sv, vals[o])
    sk, sv = _sort(nrg, dev, keys, None, bits)
    np.testing.assert_array_equal(sk, keys[o])
    np.testing.assert_array_equal(sv, o.astype(np.uint32))


def test_radix_sort_synthetic_pattern(nrg, orc):
    """The key pattern of the synthetic replay at tid = 0 (every op's first cold touch on word 2)."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1 << 16)
    n, T = 1000, 6
    raw = orc.gen_raw(4 * n, 900)
    keys = []
    for i in range(n):
        keys.append(int(raw[4 * i + 2]) % 2)
        b = 0
        for k in range(5):
            keys.append(b % 199998 + 2)
            b = (b + int(raw[4 * i + 2])) & ((1 << 64) - 1)
    keys = np.array(keys, np.uint32)
    vals = np.arange(n * T, dtype=np.uint32)
    sk, sv = _sort(nrg, dev, keys, vals, 18)
    o = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(sk, keys[o])
    np.testing.assert_array_equal(sv, vals[o])


@pytest.mark.parametrize("n,span,setfrac", [(10, 3, 0), (6000, 7, 0), (6000, 7, 10), (100_000, 50, 5),
                                            (200_000, 100_000, 1)])
def test_maxscan(nrg, orc, n, span, setfrac):
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, max_batch=1 << 16)
    keys = np.sort(orc.gen_uniform(n, 3, span)).astype(np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    if setfrac:
        vals[orc.gen_uniform(n, 4, 100) < setfrac] |= np.uint32(0x80000000)
    head = np.ones(n, bool)
    head[1:] = keys[1:] != keys[:-1]
    mark = np.where(head | (vals >= 0x80000000), np.arange(n), 0)
    want = np.maximum.accumulate(mark).astype(np.uint32)
    dk = torch.from_numpy(keys.view(np.int32)).cuda()
    dv = torch.from_numpy(vals.view(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    nrg._lib.check(nrg.load().nrg_test_maxscan(dev.handle, dk.data_ptr(), dv.data_ptr(), n, out.data_ptr()))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("keys", [1, 2, 8, 64, 512])
def test_lds_add_lane_order(nrg, keys):
    """The hardware property the synthetic replay's rankings rest on (synthetic.hip):
    the lanes of one returning LDS add that hit the same count get their old values in lane
    order, so a wave's ranks follow log order."""
    import ctypes as C

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, max_batch=1 << 12)
    out = (C.c_uint64 * 2)()
    nrg._lib.check(nrg.load().nrg_test_lds_add_order(dev.handle, keys, 40, 512, out), "nrg_test_lds_add_order")
    assert out[0] == 512 * 8 * 64 * 40 * 5
    assert out[1] == 0, f"{out[1]} of {out[0]} lanes out of lane order"


def test_device_stack_and_zipf_generators(nrg, orc):
    """Device generators used by bench.py: stack ops bit-exact with the oracle; Zipf keys equal
    to the oracle's except where device pow and glibc pow round differently (rare, +-1 rank)."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1024)
    dev.use_torch_stream()
    n = 200_000
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    dev.gen_stack_ops_device(d, n, 77)
    torch.cuda.synchronize()
    ops = d.cpu().numpy().view("u8")
    vals, opc = orc.gen_stack_ops(n, 77)
    assert ((ops & 0xFFFFFFFF).astype("u4") == vals).all()
    assert ((ops >> 32).astype("u4") == opc).all()
    for scramble in (False, True):
        dev.gen_zipf_device(d, n, 91, 1_000_000, 0.99, scramble)
        torch.cuda.synchronize()
        got = d.cpu().numpy().view("u8")
        want = orc.gen_zipf(n, 91, 1_000_000, 0.99, scramble)
        assert (got < 1_000_000).all()
        assert (got != want).mean() < 1e-3
    dev.close()
