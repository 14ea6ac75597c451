"""The reference's Log unit tests (nr/src/log.rs:708-1131), run against the PRODUCT Log: the
head/tail/ctail/ltail bookkeeping of libnrgpu.so (runtime.cpp) and its HBM ring, observed
through nrg_log_state and nrg_test_ring_read. The reference manipulates private fields to set
up each case; here every state is reached through the public calls (append, exec) instead.

Each GPU context holds its own copy of the shared log, so the reference's `head = min over
replicas' ltails` (nr/src/log.rs:536-580) is this replica's ltail; the multi-replica forms
(advance_head over four replicas, is_replica_synced_for_reads for two) run through the Python
Log mirror over several device replicas (nrgpu/replica.py).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GC_FROM_HEAD = 8192  # nr/src/log.rs:36
DEFAULT_LOG_BYTES = 32 << 20  # nr/src/log.rs:22


def _stack_dev(nrg, **kw):
    # stack records are the smallest (8 B): the log tests only need records of some kind
    kw.setdefault("max_batch", 1 << 16)
    kw.setdefault("stack_capacity", 1 << 22)
    return nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, **kw)


def _pushes(n, base=0):
    import nrgpu

    r = np.zeros(n, nrgpu.STACK_OP_DTYPE)
    r["val"] = (np.arange(n, dtype=np.uint64) + base).astype(np.uint32)
    r["op"] = 1
    return r


def _append_many(dev, n, base=0, chunk=1 << 16):
    done = 0
    while done < n:
        m = min(chunk, n - done)
        dev.log_append(_pushes(m, base + done), 1)
        done += m


@pytest.mark.parametrize("nbytes,entries", [
    (1024 * 1024, 16384),              # test_log_create: 1 MiB / 64 B entries (:748-767)
    (1024, 2 * GC_FROM_HEAD),          # test_log_min_size: at least 2 * GC_FROM_HEAD (:771-776)
    (524 * 1024, 16384),               # test_log_power_of_two: 8384 -> next power of two (:781-787)
    (DEFAULT_LOG_BYTES, DEFAULT_LOG_BYTES // 64),  # test_log_create_default (:790-808)
])
def test_log_sizing(nrg, nbytes, entries):
    dev = _stack_dev(nrg, log_bytes=nbytes)
    st = dev.log_state()
    assert st["size"] == entries
    assert st["head"] == st["tail"] == st["ctail"] == st["ltail"] == 0
    dev.close()


def test_log_index_in_the_ring(nrg):
    """test_log_index (:812-816): for a 2 MiB log, logical index 99000 lives at entry 696. Here
    99,001 records are appended (GC replays and advances the head on the way) and the record
    appended as number 99000 is read back from physical ring position 696."""
    dev = _stack_dev(nrg, log_bytes=2 * 1024 * 1024)
    assert dev.log_state()["size"] == 32768
    _append_many(dev, 99001, chunk=8192)  # appends of <= size - GC_FROM_HEAD entries
    st = dev.log_state()
    assert st["tail"] == 99001 and st["head"] <= 99000
    rec = np.zeros(1, nrg.STACK_OP_DTYPE)
    nrg.load().nrg_test_ring_read(dev.handle, 696, rec.ctypes.data_as(C.c_void_p))
    assert int(rec["val"][0]) == 99000 and int(rec["op"][0]) == 1
    dev.close()


def test_log_append_and_exec(nrg):
    """test_log_append / _append_multiple (:837-858) and test_log_exec / _exec_multiple
    (:920-994): tail counts appended entries, head stays 0; exec moves ctail and ltail to tail;
    exec of an up-to-date replica replays nothing (:951-968)."""
    dev = _stack_dev(nrg)
    dev.log_append(_pushes(1), 1)
    st = dev.log_state()
    assert (st["head"], st["tail"], st["ltail"]) == (0, 1, 0)
    dev.log_append(_pushes(2, 1), 1)
    assert dev.log_state()["tail"] == 3
    dev.log_exec()
    st = dev.log_state()
    assert st["tail"] == st["ctail"] == st["ltail"] == 3
    dev.log_exec()  # nothing to replay
    st = dev.log_state()
    assert st["tail"] == st["ctail"] == st["ltail"] == 3
    assert dev.st_dump().tolist() == [0, 1, 2]
    dev.close()


def test_log_append_gc_advances_head(nrg):
    """test_log_append_gc (:877-894): with tail = size - GC_FROM_HEAD - 1 and the replica's ltail
    at 1024, appending 4 entries advances head to 1024 and leaves tail = size - GC_FROM_HEAD + 3."""
    dev = _stack_dev(nrg, log_bytes=DEFAULT_LOG_BYTES)
    size = dev.log_state()["size"]
    _append_many(dev, 1024)
    dev.log_exec()  # ltail = 1024
    _append_many(dev, size - GC_FROM_HEAD - 1 - 1024, base=1024)
    st = dev.log_state()
    assert (st["tail"], st["ltail"], st["head"]) == (size - GC_FROM_HEAD - 1, 1024, 0)
    dev.log_append(_pushes(4), 1)
    st = dev.log_state()
    assert st["head"] == 1024
    assert st["tail"] == size - GC_FROM_HEAD + 3
    assert st["ltail"] == 1024  # the head moved without replaying: the room was there
    dev.close()


def test_log_append_wrap(nrg):
    """test_log_append_wrap (:899-916): head at 2 * 8192, tail at size - 10, appending 1024
    entries wraps the ring: tail = size + 1014. Then the wrapped entries replay in order."""
    dev = _stack_dev(nrg, log_bytes=DEFAULT_LOG_BYTES)
    size = dev.log_state()["size"]
    _append_many(dev, 2 * 8192)
    dev.log_exec()
    _append_many(dev, size - 10 - 2 * 8192, base=2 * 8192)
    dev.log_append(_pushes(1024, size - 10), 1)
    st = dev.log_state()
    assert st["tail"] == size + 1014 and st["head"] == 2 * 8192
    dev.log_exec()
    st = dev.log_state()
    assert st["ltail"] == st["ctail"] == size + 1014
    # every push landed, in log order, across the wrap
    assert dev.st_len() == size + 1014
    rec = np.zeros(1, nrg.STACK_OP_DTYPE)
    nrg.load().nrg_test_ring_read(dev.handle, 1013, rec.ctypes.data_as(C.c_void_p))  # logical size + 1013
    assert int(rec["val"][0]) == (size + 1013) & 0xFFFFFFFF
    dev.close()


def test_log_advance_head_min_ltail(nrg):
    """test_log_advance_head (:862-873): with replica ltails 1023, 224, 4096 and 799 the head
    advances to the smallest, 224. Four device replicas share one Log (nrgpu.Log); each replays
    up to its own point, and advance_head takes the minimum over them."""
    import nrgpu

    log = nrgpu.Log(DEFAULT_LOG_BYTES)
    reps = [nrgpu.Replica(log, nrgpu.Stack, device=0, max_batch=1 << 13, stack_capacity=1 << 14) for _ in range(4)]
    assert [r.idx for r in reps] == [1, 2, 3, 4]  # Log::register hands out ids from 1 (:820-825)
    done = 0
    for target, r in sorted(zip([1023, 224, 4096, 799], reps), key=lambda x: x[0]):
        log.append(_pushes(target - done, done), 1)
        done = target
        r.dev.log_exec()
    assert sorted(r.dev.log_state()["ltail"] for r in reps) == [224, 799, 1023, 4096]
    assert log.advance_head() == 224
    for r in reps:
        r.dev.close()


def test_replica_synced_for_reads(nrg):
    """test_replica_synced_for_read (:1108-1130): after one replica replays an entry the other
    has not, reads are allowed on the first and refused on the second until it replays."""
    import nrgpu

    log = nrgpu.Log(DEFAULT_LOG_BYTES)
    one = nrgpu.Replica(log, nrgpu.NrHashMap, device=0, log2_slots=10, max_batch=1024)
    two = nrgpu.Replica(log, nrgpu.NrHashMap, device=0, log2_slots=10, max_batch=1024)
    assert (one.idx, two.idx) == (1, 2)
    log.append(nrgpu.NrHashMap.encode([nrgpu.Put(5, 50)]), one.idx)
    one.dev.log_exec()
    assert log.is_replica_synced_for_reads(one) and not log.is_replica_synced_for_reads(two)
    v, f = one.dev.hm_get(np.array([5], np.uint64))
    assert int(f[0]) == 1 and int(v[0]) == 50
    with pytest.raises(nrgpu.NrgError) as e:
        two.dev.hm_get(np.array([5], np.uint64))
    assert e.value.code == nrgpu._lib.NRG_E_NOT_SYNCED
    two.dev.log_exec()
    assert log.is_replica_synced_for_reads(two)
    one.dev.close()
    two.dev.close()
