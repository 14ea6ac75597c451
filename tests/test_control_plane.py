"""The reference's deterministic unit tests of the NR control plane, ported one-for-one and
run against the C++ restatement in oracle/nr_cpu.cpp (the CPU baseline's Log / Context /
Replica). Each test names the reference test it ports.

Ops on the test log use the reference tests' `Operation` enum (nr/src/log.rs:716-730):
Read = 0, Write(v) = (1 << 63) | v, Invalid = 1.
"""
import ctypes as C

import numpy as np
import pytest

READ = 0
INVALID = 1


def WRITE(v):
    return (1 << 63) | v


# field selectors of the C test API (oracle/nr_cpu.cpp)
SIZE, RAWB, HEAD, TAIL, CTAIL, NEXT, PANICKED = range(7)
C_TAIL, C_HEAD, C_COMB, C_PANICKED = range(4)
R_IDX, R_COMBINER, R_NEXT, R_JUNK = range(4)


class TLog:
    def __init__(self, orc, nbytes=None):
        self.L = orc.lib()
        self.h = self.L.orc_log_default() if nbytes is None else self.L.orc_log_new(nbytes)

    def __del__(self):
        self.L.orc_log_free(self.h)

    def get(self, f):
        return int(self.L.orc_log_get(self.h, f))

    def set(self, f, v):
        self.L.orc_log_set(self.h, f, v)

    def ltail(self, r):
        return int(self.L.orc_log_ltail(self.h, r))

    def set_ltail(self, r, v):
        self.L.orc_log_set_ltail(self.h, r, v)

    def lmask(self, r):
        return bool(self.L.orc_log_lmask(self.h, r))

    def register(self):
        r = int(self.L.orc_log_register(self.h))
        return None if r < 0 else r

    def append(self, ops, idx):
        a = np.ascontiguousarray(np.asarray(ops, np.uint64))
        cap = 1 << 16
        go, gr = np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
        u64p = C.POINTER(C.c_uint64)
        n = self.L.orc_log_append(self.h, a.ctypes.data_as(u64p), len(a), idx, go.ctypes.data_as(u64p),
                                  gr.ctypes.data_as(u64p), cap)
        return list(zip(go[:n].tolist(), gr[:n].tolist()))

    def exec(self, idx):
        cap = 1 << 16
        o, r = np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
        u64p = C.POINTER(C.c_uint64)
        n = self.L.orc_log_exec(self.h, idx, o.ctypes.data_as(u64p), r.ctypes.data_as(u64p), cap)
        return list(zip(o[:n].tolist(), r[:n].tolist()))

    def entry(self, phys):
        op, rep = C.c_uint64(), C.c_uint64()
        has = self.L.orc_log_entry(self.h, phys, C.byref(op), C.byref(rep))
        return (int(op.value) if has else None), int(rep.value)

    def synced(self, idx, ctail):
        return bool(self.L.orc_log_synced(self.h, idx, ctail))

    def ctail(self):
        return int(self.L.orc_log_get_ctail(self.h))


@pytest.fixture
def K(orc):
    L = orc.lib()
    return dict(DEFAULT_LOG_BYTES=int(L.orc_log_const(0)), MAX_REPLICAS=int(L.orc_log_const(1)),
                GC_FROM_HEAD=int(L.orc_log_const(2)), MAX_PENDING_OPS=int(L.orc_log_const(3)),
                MAX_THREADS_PER_REPLICA=int(L.orc_log_const(4)), ENTRY=int(L.orc_log_entry_size()))


# ---- nr/src/log.rs tests ---------------------------------------------------------------
def test_constants(K):
    """nr/src/log.rs:22,26,36 ; context.rs:12 ; replica.rs:56"""
    assert K["DEFAULT_LOG_BYTES"] == 32 * 1024 * 1024
    assert K["MAX_REPLICAS"] == 192
    assert K["MAX_PENDING_OPS"] == 32
    assert K["MAX_THREADS_PER_REPLICA"] == 256
    assert K["GC_FROM_HEAD"] == 8192


def test_log_entry_size(K):
    """log.rs:742-746 test_log_entry_size"""
    assert K["ENTRY"] == 64


def test_log_create(orc, K):
    """log.rs:748-768 test_log_create"""
    lg = TLog(orc, 1024 * 1024)
    n = (1024 * 1024) // K["ENTRY"]
    assert lg.get(RAWB) == 1024 * 1024
    assert lg.get(SIZE) == n
    assert (lg.get(HEAD), lg.get(TAIL), lg.get(NEXT), lg.get(CTAIL)) == (0, 0, 1, 0)
    assert all(lg.ltail(i) == 0 for i in range(K["MAX_REPLICAS"]))
    assert all(lg.lmask(i) for i in range(K["MAX_REPLICAS"]))


def test_log_entry_create_default(orc):
    """log.rs:733-740 test_entry_create_default"""
    lg = TLog(orc, 1024)
    assert lg.entry(0) == (None, 0)


def test_log_min_size(orc, K):
    """log.rs:770-778 test_log_min_size"""
    lg = TLog(orc, 1024)
    assert lg.get(RAWB) == 2 * K["GC_FROM_HEAD"] * K["ENTRY"]
    assert lg.get(SIZE) == 2 * K["GC_FROM_HEAD"]


def test_log_power_of_two(orc, K):
    """log.rs:780-788 test_log_power_of_two"""
    lg = TLog(orc, 524 * 1024)
    n = 1 << ((524 * 1024) // K["ENTRY"] - 1).bit_length()
    assert lg.get(RAWB) == n * K["ENTRY"]
    assert lg.get(SIZE) == n


def test_log_create_default(orc, K):
    """log.rs:790-810 test_log_create_default"""
    lg = TLog(orc)
    assert lg.get(RAWB) == K["DEFAULT_LOG_BYTES"]
    assert lg.get(SIZE) == K["DEFAULT_LOG_BYTES"] // K["ENTRY"]
    assert (lg.get(HEAD), lg.get(TAIL), lg.get(NEXT), lg.get(CTAIL)) == (0, 0, 1, 0)


def test_log_index(orc):
    """log.rs:812-817 test_log_index"""
    lg = TLog(orc, 2 * 1024 * 1024)
    assert int(orc.lib().orc_log_index(lg.h, 99000)) == 696


def test_log_register(orc):
    """log.rs:819-825 test_log_register"""
    lg = TLog(orc, 1024)
    assert lg.register() == 1
    assert lg.get(NEXT) == 2


def test_log_register_none(orc, K):
    """log.rs:827-834 test_log_register_none"""
    lg = TLog(orc, 1024)
    lg.set(NEXT, K["MAX_REPLICAS"])
    assert lg.register() is None
    assert lg.get(NEXT) == K["MAX_REPLICAS"]


def test_log_append(orc):
    """log.rs:836-848 test_log_append"""
    lg = TLog(orc)
    lg.append([READ], 1)
    assert lg.get(HEAD) == 0 and lg.get(TAIL) == 1
    assert lg.entry(0) == (READ, 1)


def test_log_append_multiple(orc):
    """log.rs:850-859 test_log_append_multiple"""
    lg = TLog(orc)
    lg.append([READ, WRITE(119)], 1)
    assert lg.get(HEAD) == 0 and lg.get(TAIL) == 2


def test_log_advance_head(orc):
    """log.rs:861-874 test_log_advance_head"""
    lg = TLog(orc)
    lg.set(NEXT, 5)
    for i, t in enumerate([1023, 224, 4096, 799]):
        lg.set_ltail(i, t)
    orc.lib().orc_log_advance_head(lg.h, 0)
    assert lg.get(HEAD) == 224


def test_log_append_gc(orc, K):
    """log.rs:876-896 test_log_append_gc"""
    lg = TLog(orc)
    size = lg.get(SIZE)
    lg.set(NEXT, 2)
    lg.set(TAIL, size - K["GC_FROM_HEAD"] - 1)
    lg.set_ltail(0, 1024)
    lg.append([READ] * 4, 1)
    assert lg.get(HEAD) == 1024
    assert lg.get(TAIL) == size - K["GC_FROM_HEAD"] + 3


def test_log_append_wrap(orc):
    """log.rs:898-917 test_log_append_wrap"""
    lg = TLog(orc)
    size = lg.get(SIZE)
    lg.set(NEXT, 2)
    lg.set(HEAD, 2 * 8192)
    lg.set(TAIL, size - 10)
    lg.append([READ] * 1024, 1)
    assert lg.lmask(0) is True
    assert lg.get(TAIL) == size + 1014


def test_log_exec(orc):
    """log.rs:919-940 test_log_exec"""
    lg = TLog(orc)
    lg.append([READ], 1)
    assert lg.exec(1) == [(READ, 1)]
    assert lg.get(TAIL) == lg.get(CTAIL) == lg.ltail(0)


def test_log_exec_empty(orc):
    """log.rs:942-951 test_log_exec_empty"""
    lg = TLog(orc)
    assert lg.exec(1) == []


def test_log_exec_zero(orc):
    """log.rs:953-969 test_log_exec_zero"""
    lg = TLog(orc)
    lg.append([READ], 1)
    assert lg.exec(1) == [(READ, 1)]
    assert lg.exec(1) == []


def test_log_exec_multiple(orc):
    """log.rs:971-996 test_log_exec_multiple"""
    lg = TLog(orc)
    lg.append([READ, WRITE(119)], 1)
    s = 0
    for op, _ in lg.exec(1):
        assert op != INVALID
        s += 121 if op == READ else op & ~(1 << 63)
    assert s == 240
    assert lg.get(TAIL) == lg.get(CTAIL) == lg.ltail(0)


def test_log_exec_wrap(orc):
    """log.rs:998-1025 test_log_exec_wrap"""
    lg = TLog(orc)
    size = lg.get(SIZE)
    lg.append([READ] * 1024, 1)  # required for GC to work correctly
    lg.set(NEXT, 2)
    lg.set(HEAD, 2 * 8192)
    lg.set(TAIL, size - 10)
    lg.append([READ] * 1024, 1)
    lg.set_ltail(0, size - 10)
    ran = lg.exec(1)
    assert len(ran) == 1024 and all(x == (READ, 1) for x in ran)
    assert lg.lmask(0) is False
    assert lg.get(TAIL) == size + 1014


def test_exec_panic(orc):
    """log.rs:1027-1048 test_exec_panic (#[should_panic]: local tail below head)"""
    lg = TLog(orc)
    lg.append([READ] * 1024, 1)
    lg.set(HEAD, 8192)
    assert lg.exec(1) == []
    assert lg.get(PANICKED) == 1


def test_log_overwrite_after_reset(orc):
    """log.rs:1050-1076 test_log_change_refcount: entries written after Log::reset replace
    (drop) the old operations in place."""
    lg = TLog(orc)
    lg.append([WRITE(1)], 1)
    lg.append([WRITE(1)], 1)
    assert [lg.entry(i)[0] for i in range(2)] == [WRITE(1)] * 2
    orc.lib().orc_log_reset(lg.h)
    lg.append([WRITE(2)], 1)
    assert [lg.entry(i)[0] for i in range(2)] == [WRITE(2), WRITE(1)]
    lg.append([WRITE(2)], 1)
    assert [lg.entry(i)[0] for i in range(2)] == [WRITE(2)] * 2


def test_log_overwrite_with_gc(orc, K):
    """log.rs:1078-1106 test_log_refcount_change_with_gc: a 16384-entry log filled twice;
    GC lets the second pass overwrite every entry of the first."""
    total = 16384
    lg = TLog(orc, total * K["ENTRY"])
    assert lg.get(SIZE) == total
    for _ in range(total):
        lg.append([WRITE(1)], 1)
    assert all(lg.entry(i)[0] == WRITE(1) for i in range(0, total, 97))
    for i in range(1, total + 1):
        lg.append([WRITE(2)], 1)
        if i in (1, total // 2, total):
            assert lg.entry(i - 1)[0] == WRITE(2)
            if i < total:
                assert lg.entry(i)[0] == WRITE(1)
    assert all(lg.entry(i)[0] == WRITE(2) for i in range(total))
    assert lg.get(TAIL) == 2 * total


def test_replica_synced_for_read(orc):
    """log.rs:1108-1130 test_replica_synced_for_read"""
    lg = TLog(orc)
    one, two = lg.register(), lg.register()
    assert (one, two) == (1, 2)
    lg.append([READ], one)
    assert lg.exec(one) == [(READ, 1)]
    assert lg.synced(one, lg.ctail()) is True
    assert lg.synced(two, lg.ctail()) is False
    assert lg.exec(two) == [(READ, 1)]
    assert lg.synced(two, lg.ctail()) is True


# ---- nr/src/context.rs tests -----------------------------------------------------------
class TCtx:
    def __init__(self, orc):
        self.L = orc.lib()
        self.h = self.L.orc_ctx_new()

    def __del__(self):
        self.L.orc_ctx_free(self.h)

    def get(self, f):
        return int(self.L.orc_ctx_get(self.h, f))

    def set(self, f, v):
        self.L.orc_ctx_set(self.h, f, v)

    def enqueue(self, op):
        return bool(self.L.orc_ctx_enqueue(self.h, op))

    def enqueue_resps(self, rs):
        a = np.ascontiguousarray(np.asarray(rs, np.uint64))
        self.L.orc_ctx_enqueue_resps(self.h, a.ctypes.data_as(C.POINTER(C.c_uint64)), len(a))

    def ops(self):
        out = np.zeros(64, np.uint64)
        n = self.L.orc_ctx_ops(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), 64)
        return out[:n].tolist()

    def res(self):
        v = C.c_uint64()
        return int(v.value) if self.L.orc_ctx_res(self.h, C.byref(v)) else None


def test_context_create_default(orc):
    """context.rs:215-223"""
    c = TCtx(orc)
    assert (c.get(C_TAIL), c.get(C_HEAD), c.get(C_COMB)) == (0, 0, 0)


def test_context_enqueue(orc):
    """context.rs:225-234"""
    c = TCtx(orc)
    assert c.enqueue(121)
    assert (c.get(C_TAIL), c.get(C_HEAD), c.get(C_COMB)) == (1, 0, 0)
    assert c.ops() == [121]


def test_context_enqueue_full(orc, K):
    """context.rs:236-246"""
    c = TCtx(orc)
    c.set(C_TAIL, K["MAX_PENDING_OPS"])
    assert not c.enqueue(100)
    assert (c.get(C_TAIL), c.get(C_HEAD), c.get(C_COMB)) == (K["MAX_PENDING_OPS"], 0, 0)


def test_context_enqueue_resps(orc):
    """context.rs:248-267"""
    c = TCtx(orc)
    c.set(C_TAIL, 16)
    c.set(C_COMB, 12)
    c.enqueue_resps([11, 12, 13, 14])
    assert (c.get(C_TAIL), c.get(C_HEAD), c.get(C_COMB)) == (16, 0, 16)
    c.set(C_HEAD, 12)  # read back batch[12..16] through res()
    assert [c.res() for _ in range(4)] == [11, 12, 13, 14]


def test_context_enqueue_resps_empty(orc):
    """context.rs:269-284"""
    c = TCtx(orc)
    c.set(C_TAIL, 16)
    c.set(C_COMB, 12)
    c.enqueue_resps([])
    assert (c.get(C_TAIL), c.get(C_HEAD), c.get(C_COMB)) == (16, 0, 12)
    c.set(C_HEAD, 12)
    assert c.res() is None


def test_context_ops(orc, K):
    """context.rs:286-305"""
    c = TCtx(orc)
    half = K["MAX_PENDING_OPS"] // 2
    for i in range(half):
        assert c.enqueue(i * i)
    assert c.ops() == [i * i for i in range(half)]
    assert (c.get(C_TAIL), c.get(C_HEAD), c.get(C_COMB)) == (half, 0, 0)


def test_context_ops_empty(orc):
    """context.rs:307-321"""
    c = TCtx(orc)
    c.set(C_TAIL, 8)
    c.set(C_COMB, 8)
    assert c.ops() == []
    assert (c.get(C_TAIL), c.get(C_HEAD), c.get(C_COMB)) == (8, 0, 8)


def test_context_ops_panic(orc):
    """context.rs:323-334 (#[should_panic]: combiner head beyond tail)"""
    c = TCtx(orc)
    c.set(C_TAIL, 6)
    c.set(C_COMB, 9)
    assert c.ops() == []
    assert c.get(C_PANICKED) == 1


def test_context_res(orc):
    """context.rs:336-359"""
    c = TCtx(orc)
    c.set(C_TAIL, 16)
    c.enqueue_resps([11, 12, 13, 14])
    assert (c.get(C_TAIL), c.get(C_COMB)) == (16, 4)
    for i, want in enumerate([11, 12, 13, 14]):
        assert c.res() == want
        assert c.get(C_HEAD) == i + 1


def test_context_res_empty(orc):
    """context.rs:361-373"""
    c = TCtx(orc)
    c.set(C_TAIL, 8)
    assert c.res() is None


def test_context_res_panic(orc):
    """context.rs:375-386 (#[should_panic]: head beyond combiner offset)"""
    c = TCtx(orc)
    c.set(C_TAIL, 8)
    c.set(C_COMB, 4)
    c.set(C_HEAD, 6)
    assert c.res() is None
    assert c.get(C_PANICKED) == 1


def test_context_index_wraps(orc, K):
    """context.rs:388-398 (batch_size / index): slots are reused modulo MAX_PENDING_OPS"""
    c = TCtx(orc)
    for r in range(3):
        for i in range(K["MAX_PENDING_OPS"]):
            assert c.enqueue(r * 1000 + i)
        assert not c.enqueue(1)
        assert c.ops() == [r * 1000 + i for i in range(K["MAX_PENDING_OPS"])]
        c.enqueue_resps([7] * K["MAX_PENDING_OPS"])
        assert [c.res() for _ in range(K["MAX_PENDING_OPS"])] == [7] * K["MAX_PENDING_OPS"]


# ---- nr/src/replica.rs tests (Data{junk}: dispatch_mut -> junk += 1, Ok(107)) ----------------
class TRep:
    def __init__(self, orc, nbytes=0):
        self.L = orc.lib()
        self.h = self.L.orc_rep_new(nbytes)

    def __del__(self):
        self.L.orc_rep_free(self.h)

    def get(self, f):
        return int(self.L.orc_rep_get(self.h, f))

    def set(self, f, v):
        self.L.orc_rep_set(self.h, f, v)

    def register(self):
        r = int(self.L.orc_rep_register(self.h))
        return None if r < 0 else r

    def res(self, tid):
        v = C.c_uint64()
        return int(v.value) if self.L.orc_rep_ctx_res(self.h, tid, C.byref(v)) else None


def test_replica_create(orc):
    """replica.rs:627-646"""
    r = TRep(orc, 1024)
    assert (r.get(R_IDX), r.get(R_COMBINER), r.get(R_NEXT), r.get(R_JUNK)) == (1, 0, 1, 0)


def test_replica_register(orc):
    """replica.rs:648-658"""
    r = TRep(orc, 1024)
    assert r.register() == 1
    assert r.get(R_NEXT) == 2
    r.set(R_NEXT, 17)
    assert r.register() == 17
    assert r.get(R_NEXT) == 18


def test_replica_register_none(orc, K):
    """replica.rs:660-668"""
    r = TRep(orc, 1024)
    r.set(R_NEXT, K["MAX_THREADS_PER_REPLICA"] + 1)
    assert r.register() is None


def test_replica_make_pending(orc):
    """replica.rs:670-681"""
    r = TRep(orc, 1024)
    assert r.L.orc_rep_make_pending(r.h, 121, 8)
    r.set(R_NEXT, 9)
    r.L.orc_rep_try_combine(r.h, 1)  # the pending op of thread 8 is combined
    assert r.get(R_JUNK) == 1
    assert r.res(8) == 107


def test_replica_make_pending_false(orc, K):
    """replica.rs:683-693"""
    r = TRep(orc, 1024)
    for _ in range(K["MAX_PENDING_OPS"]):
        assert r.L.orc_rep_make_pending(r.h, 121, 1)
    assert not r.L.orc_rep_make_pending(r.h, 11, 1)


def test_replica_try_combine(orc):
    """replica.rs:695-708"""
    r = TRep(orc)
    r.register()
    r.L.orc_rep_make_pending(r.h, 121, 1)
    r.L.orc_rep_try_combine(r.h, 1)
    assert r.get(R_COMBINER) == 0
    assert r.get(R_JUNK) == 1
    assert r.res(1) == 107


def test_replica_try_combine_pending(orc):
    """replica.rs:710-722"""
    r = TRep(orc)
    r.set(R_NEXT, 9)
    r.L.orc_rep_make_pending(r.h, 121, 8)
    r.L.orc_rep_try_combine(r.h, 1)
    assert r.get(R_JUNK) == 1
    assert r.res(8) == 107


def test_replica_try_combine_fail(orc):
    """replica.rs:724-737"""
    r = TRep(orc, 1024)
    r.set(R_NEXT, 9)
    r.set(R_COMBINER, 8)
    r.L.orc_rep_make_pending(r.h, 121, 1)
    r.L.orc_rep_try_combine(r.h, 1)
    assert r.get(R_JUNK) == 0
    assert r.res(1) is None


def test_replica_execute_combine(orc):
    """replica.rs:739-749"""
    r = TRep(orc)
    idx = r.register()
    assert int(r.L.orc_rep_execute_mut(r.h, 121, idx)) == 107
    assert r.get(R_JUNK) == 1


def test_replica_get_response(orc):
    """replica.rs:751-761"""
    r = TRep(orc)
    r.register()
    r.L.orc_rep_make_pending(r.h, 121, 1)
    assert int(r.L.orc_rep_get_response(r.h, 1)) == 107


def test_replica_execute(orc):
    """replica.rs:763-773"""
    r = TRep(orc)
    idx = r.register()
    assert int(r.L.orc_rep_execute_mut(r.h, 121, idx)) == 107
    assert int(r.L.orc_rep_execute(r.h, 11, idx)) == 1


def test_replica_execute_not_synced(orc):
    """replica.rs:775-787: ops appended "off the side" by replica 2 are replayed before a read"""
    r = TRep(orc)
    ops = np.array([121, 212], np.uint64)
    r.L.orc_rep_log_append_exec(r.h, ops.ctypes.data_as(C.POINTER(C.c_uint64)), 2, 2)
    t1 = r.register()
    assert int(r.L.orc_rep_execute(r.h, 11, t1)) == 2


# ---- the Stack and AbstractDataStructure plugged into the nr restatement (bench.py's CPU
# baselines for the stack and synthetic lines, benches/stack.rs:115-134,
# benches/synthetic.rs:296-335): one thread's stream through Replica<D> must give exactly the
# sequential oracle's responses and final state ---------------------------------------------
def test_nr_stack_replica_matches_oracle(orc):
    import numpy as np

    vals, kinds = orc.gen_stack_ops(20_000, 0xAB)
    kinds = kinds.copy()
    kinds[:3000] = 0  # drain past empty: Pop on an empty Vec is None
    init = np.arange(1000, dtype=np.uint32)
    resp, fin = orc.nr_stack_run(init, vals, kinds)
    st = orc.Stack(init)
    r_o, s_o = st.replay(vals, kinds)
    assert np.array_equal((resp >> 32).astype(np.uint8), s_o)
    assert np.array_equal((resp & 0xFFFFFFFF).astype(np.uint32)[s_o == 1], r_o[s_o == 1])
    assert np.array_equal(fin, st.dump()[:len(st)])


def test_nr_synth_replica_matches_oracle(orc):
    import numpy as np

    n = 6000
    raw = orc.gen_raw(3 * n, 0x77)
    ops = np.stack([raw[0::3] % 64, raw[1::3], raw[2::3], (raw[0::3] >> 40) & 1], axis=1).astype(np.uint64)
    ops[:50, 2] = np.uint64(2**64 - 1)  # r2 + hot_writes wraps: the hot loop is empty
    reads = np.stack([raw[1::3][:500] % 64, raw[2::3][:500], raw[0::3][:500]], axis=1).astype(np.uint64)
    resp, rresp, fin = orc.nr_synth_run(ops, reads)
    sy = orc.Synthetic()
    assert np.array_equal(resp, sy.replay(ops))
    assert np.array_equal(rresp, sy.read(reads))
    assert np.array_equal(fin, sy.dump())


def test_nr_stack_and_synth_scale_out_run(orc):
    import os

    cpus = sorted(os.sched_getaffinity(0))[:2]
    for fn in (orc.nr_stack_bench, orc.nr_synth_bench):
        r = fn(cpus, [0] * len(cpus), 0.2, 10_000, 0x5A)
        assert r.ops > 0 and r.writes == r.ops and r.seconds > 0.1
