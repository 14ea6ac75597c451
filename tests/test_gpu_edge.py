"""Edge cases of the hashmap replay through the C ABI: empty and one-sided rounds, the whole u64
key domain (key 0, u64::MAX - 1, and u64::MAX which lives in the side slot), a table that runs
out of slots (NRG_E_TABLE_FULL, where std::HashMap would grow), an append larger than the ring
(NRG_E_RING_FULL, where Log::append would spin, nr/src/log.rs:368-380), and errors reported by
the next synchronising call."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MAXU = 0xFFFFFFFFFFFFFFFF


def _puts(nrg, keys, vals):
    r = np.zeros(len(keys), nrg.PUT_DTYPE)
    r["key"] = keys
    r["val"] = vals
    return r


@pytest.mark.parametrize("pipeline", [0, 1])
def test_empty_and_one_sided_rounds(nrg, orc, pipeline):
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=12, max_batch=1024, pipeline=pipeline)
    dev.use_torch_stream()
    om = orc.HashMap()
    e64 = torch.empty(0, dtype=torch.int64, device="cuda")
    e8 = torch.empty(0, dtype=torch.uint8, device="cuda")
    dev.hm_round_device(e64, 0, 1, e64, 0, e64, e8)  # nothing at all
    keys = np.array([5, 6, 7], np.uint64)
    vals = np.array([50, 60, 70], np.uint64)
    d_p = torch.from_numpy(_puts(nrg, keys, vals).view(np.int64).copy()).cuda()
    dev.hm_round_device(d_p, 3, 1, e64, 0, e64, e8)  # writes only
    om.replay(keys, vals)
    gk = np.array([5, 8, 7], np.uint64)
    d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
    gv = torch.full((3,), -1, dtype=torch.int64, device="cuda")
    gf = torch.full((3,), 9, dtype=torch.uint8, device="cuda")
    dev.hm_round_device(e64, 0, 1, d_gk, 3, gv, gf)  # reads only
    dev.join()
    torch.cuda.synchronize()
    ov, of = om.get_batch(gk)
    np.testing.assert_array_equal(gf.cpu().numpy(), of)
    np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), ov)
    dev.log_exec()  # nothing left to replay: a no-op
    v, f = dev.hm_get(np.zeros(0, np.uint64))
    assert len(v) == 0 and len(f) == 0
    assert dev.hm_size() == len(om) == 3
    dev.close()


def test_full_key_domain(nrg, orc):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=12, max_batch=1024)
    om = orc.HashMap()
    keys = np.array([0, MAXU, MAXU - 1, 1, MAXU, 0, 1 << 63, MAXU], np.uint64)
    vals = np.array([1, 2, 3, 4, 5, 6, 7, MAXU], np.uint64)
    first = dev.log_append(_puts(nrg, keys, vals), 1)
    prev, pf = dev.log_exec(first, first + len(keys))
    oprev, opf = om.replay(keys, vals)
    np.testing.assert_array_equal(pf, opf)
    np.testing.assert_array_equal(prev, oprev)
    q = np.array([0, MAXU, MAXU - 1, 1, 2, 1 << 63], np.uint64)
    v, f = dev.hm_get(q)
    ov, of = om.get_batch(q)
    np.testing.assert_array_equal(f, of)
    np.testing.assert_array_equal(v, ov)
    k, vv = dev.hm_dump()
    ok_, ov_ = om.dump_sorted()
    np.testing.assert_array_equal(k, ok_)
    np.testing.assert_array_equal(vv, ov_)
    assert dev.hm_digest() == om.digest()
    dev.close()


def test_table_full_is_an_error(nrg):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=4, max_batch=64)  # 16 slots
    keys = np.arange(100, 120, dtype=np.uint64)  # 20 distinct keys
    dev.log_append(_puts(nrg, keys, keys), 1)
    with pytest.raises(nrg.NrgError) as e:
        dev.log_exec()
    assert e.value.code == nrg._lib.NRG_E_TABLE_FULL
    # the error is latched once: the replica stays usable for keys it holds
    v, f = dev.hm_get(np.array([100], np.uint64))
    assert f[0] in (0, 1)
    dev.close()


def test_ring_full_is_an_error(nrg):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=1 << 15, log_bytes=1024)
    size = dev.log_state()["size"]  # minimum ring: 2 * GC_FROM_HEAD entries
    n = size - 8192 + 1  # more than a ring can ever hold ahead of head
    keys = np.arange(n, dtype=np.uint64)
    with pytest.raises(nrg.NrgError) as e:
        dev.log_append(_puts(nrg, keys, keys), 1)
    assert e.value.code == nrg._lib.NRG_E_RING_FULL
    st = dev.log_state()
    assert st["tail"] == 0  # nothing was appended
    dev.close()
