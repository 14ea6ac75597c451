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


def _round(nrg, dev, keys, vals, gk):
    import torch

    d_p = torch.from_numpy(_puts(nrg, keys, vals).view(np.int64).copy()).cuda()
    d_gk = torch.from_numpy(np.ascontiguousarray(gk).view(np.int64)).cuda()
    gv = torch.full((len(gk),), -1, dtype=torch.int64, device="cuda")
    gf = torch.full((len(gk),), 9, dtype=torch.uint8, device="cuda")
    dev.hm_round_device(d_p, len(keys), 1, d_gk, len(gk), gv, gf)
    return d_p, d_gk, gv, gf


def test_log_reset_with_a_deferred_round(nrg, orc):
    """pipeline=1: round, Log::reset, round. The first round's deferred half (apply + reads)
    must run before the reset lets the next round reuse log positions 0.. (advisor finding on
    nrg_log_reset); every read and the final digest against the oracle."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=14, max_batch=4096, pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    outs, want = [], []
    for r in range(4):
        keys = orc.gen_uniform(2000, 40 + r, 3000)
        vals = orc.gen_raw(2000, 50 + r)
        gk = orc.gen_uniform(1500, 60 + r, 3500)
        outs.append(_round(nrg, dev, keys, vals, gk))
        om.replay(keys, vals)
        want.append(om.get_batch(gk))
        if r % 2 == 0:
            dev.log_reset()
            st = dev.log_state()
            assert st["tail"] == st["head"] == st["ltail"] == 0
    dev.join()
    torch.cuda.synchronize()
    for r, (_, _, gv, gf) in enumerate(outs):
        np.testing.assert_array_equal(gf.cpu().numpy(), want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), want[r][0], err_msg=f"round {r} vals")
    assert dev.hm_digest() == om.digest()
    dev.close()


def test_stream_switch_between_async_rounds(nrg, orc):
    """nrg_set_stream between async rounds orders everything queued on the old stream before
    the new stream's work (advisor finding): rounds alternate between two torch streams with no
    host synchronisation in between."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=15, max_batch=8192, pipeline=1)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    om = orc.HashMap()
    outs, want = [], []
    for r in range(6):
        s = s1 if r % 2 == 0 else s2
        with torch.cuda.stream(s):
            keys = orc.gen_uniform(6000, 70 + r, 9000)
            vals = orc.gen_raw(6000, 80 + r)
            gk = orc.gen_uniform(5000, 90 + r, 9500)
            dev.set_stream(s.cuda_stream)
            outs.append(_round(nrg, dev, keys, vals, gk))
            om.replay(keys, vals)
            want.append(om.get_batch(gk))
    dev.join()
    torch.cuda.synchronize()
    for r, (_, _, gv, gf) in enumerate(outs):
        np.testing.assert_array_equal(gf.cpu().numpy(), want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), want[r][0], err_msg=f"round {r} vals")
    assert dev.hm_digest() == om.digest()
    dev.close()


def test_stack_overflow_then_dump_and_peek(nrg):
    """A chunk that pushes past stack_capacity latches NRG_E_CAPACITY once; afterwards len,
    dump and peek never report or copy more than the capacity (advisor finding)."""
    cap = 1000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=4096, stack_capacity=cap)
    recs = np.zeros(1500, nrg.STACK_OP_DTYPE)
    recs["val"] = np.arange(1500, dtype=np.uint32)
    recs["op"] = 1
    dev.log_append(recs, 1)
    with pytest.raises(nrg.NrgError) as e:
        dev.log_exec()
    assert e.value.code == nrg._lib.NRG_E_CAPACITY
    n = dev.st_len()
    assert n <= cap
    out = dev.st_dump()
    assert len(out) == n <= cap
    top = dev.st_peek()
    assert top is None or 0 <= top < 1500
    dev.close()
