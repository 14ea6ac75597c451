"""Native flat combining (nrg_combiner_*): many client threads, one GPU round per combine,
for the hashmap (per-thread models), the stack and the synthetic structure (the replica's own
log, read back, replayed by the oracle: every call's responses equal the oracle's at the call's
log positions).

Mirrors the reference's multi-threaded replica use (nr/src/replica.rs:345-356 register,
:414-433 execute_mut, :508-595 combine; nr/tests/stack.rs:170-262 threads against one replica):
every thread owns a disjoint key range, so each thread's responses are deterministic whatever
the interleaving -- previous values of its Puts (HashMap::insert, nr/examples/hashmap.rs:46-50)
and values of its Gets follow its own sequential model -- and the final table equals the
oracle's replay of every thread's Puts.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,ITERS,serve", [(8, 40, 1), (64, 12, 1), (256, 5, 1), (8, 40, 0), (64, 12, 0),
                                           (256, 5, 0), (8, 40, 40), (64, 12, 200)])
def test_combiner_threads(nrg, orc, T, ITERS, serve):
    """T client threads; at 64 the rounds are larger, waiters wake through the futex tree and
    rounds of up to 2048 Puts take the one-launch small rounds; at 256 batches pass 512 ops and
    two rounds run in flight, the larger ones as full (not small) rounds. serve: small rounds go
    to the resident round server (NRG_KNOB_COMB_SERVE, the default) or are launched one by one;
    40 / 200: only rounds of at most that many ops are served, so the server is stopped for every
    larger round and restarted after it."""
    SPAN = 5000
    cap = max(1 << 12, T * 32)
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=20, max_batch=cap, max_reads=cap,
                            log_bytes=64 * (1 << 16))
    dev.hm_prefill_range(1000, 1)  # keys 0..999 -> k + 1: thread 0's range starts with them
    dev.set_knob("COMB_SERVE", serve)
    comb = nrg.Combiner(dev, T)
    errors, finals = [], {}

    def client(seed):
        try:
            tok = comb.register()
            rng = np.random.default_rng(seed)
            lo = tok * SPAN
            model = {k: k + 1 for k in range(lo, min(lo + SPAN, 1000))}
            for it in range(ITERS):
                n = int(rng.integers(1, 33))
                keys = rng.integers(lo, lo + SPAN, n, dtype=np.uint64)
                if it % 3 == 0:
                    keys[n // 2:] = keys[0]  # repeated keys inside one batch
                vals = rng.integers(0, 2**63, n, dtype=np.uint64)
                prev, some = comb.put(tok, keys, vals)
                for i in range(n):
                    k = int(keys[i])
                    want = model.get(k)
                    assert bool(some[i]) == (want is not None), (tok, it, i)
                    if want is not None:
                        assert int(prev[i]) == want, (tok, it, i)
                    model[k] = int(vals[i])
                q = rng.integers(lo, lo + SPAN, int(rng.integers(1, 33)), dtype=np.uint64)
                got, found = comb.get(tok, q)
                for i, k in enumerate(q):
                    want = model.get(int(k))
                    assert bool(found[i]) == (want is not None), (tok, it, i)
                    if want is not None:
                        assert int(got[i]) == want, (tok, it, i)
            finals[tok] = model
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=client, args=(100 + i,)) for i in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[0]
    rounds, ops = comb.stats()
    assert ops > 0
    assert rounds <= 2 * T * ITERS  # combining happened: rounds never exceed calls
    comb.close()
    om = orc.HashMap()
    om.prefill_range(1000, 1)
    keys = np.array([k for m in finals.values() for k in m], np.uint64)
    vals = np.array([v for m in finals.values() for v in m.values()], np.uint64)
    om.replay(keys, vals)
    assert dev.hm_digest() == om.digest()
    dev.close()


def test_combiner_server_stops_and_restarts(nrg, orc):
    """The round server around idle gaps and launched rounds: clients pause together (the
    combiner stops the idle server after 1 ms, the next round starts a new one), and a round of
    more Gets than a served round holds (5120 > SERVE_R 4096: 160 clients post 32 Gets at once)
    is launched between served rounds (the server drains and exits first). Every answer follows
    the per-thread models; the table equals the oracle's replay."""
    import time

    T, SPAN = 160, 4000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=20, max_batch=8192, max_reads=8192,
                            log_bytes=64 * (1 << 16))
    comb = nrg.Combiner(dev, T)
    bar = threading.Barrier(T)
    errors, finals = [], {}

    def client(seed):
        try:
            tok = comb.register()
            rng = np.random.default_rng(seed)
            lo = tok * SPAN
            model = {}
            for it in range(6):
                n = 32
                keys = rng.integers(lo, lo + SPAN, n, dtype=np.uint64)
                vals = rng.integers(0, 2**63, n, dtype=np.uint64)
                prev, some = comb.put(tok, keys, vals)
                for i in range(n):
                    want = model.get(int(keys[i]))
                    assert bool(some[i]) == (want is not None) and (want is None or int(prev[i]) == want)
                    model[int(keys[i])] = int(vals[i])
                bar.wait()
                if it % 2 == 0:
                    time.sleep(0.005)  # everyone idle: the server is stopped
                bar.wait()
                q = rng.integers(lo, lo + SPAN, 32, dtype=np.uint64)  # all 160 at once: one big round
                got, found = comb.get(tok, q)
                for i, k in enumerate(q):
                    want = model.get(int(k))
                    assert bool(found[i]) == (want is not None) and (want is None or int(got[i]) == want)
            finals[tok] = model
        except Exception as e:  # noqa: BLE001
            errors.append(e)
            bar.abort()

    th = [threading.Thread(target=client, args=(500 + i,)) for i in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[0]
    comb.close()
    om = orc.HashMap()
    keys = np.array([k for m in finals.values() for k in m], np.uint64)
    vals = np.array([v for m in finals.values() for v in m.values()], np.uint64)
    om.replay(keys, vals)
    assert dev.hm_digest() == om.digest()
    dev.close()


def test_combiner_limits(nrg):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=12, max_batch=64, max_reads=64)
    with pytest.raises(nrg.NrgError):  # 4 threads x 32 ops exceed max_batch
        nrg.Combiner(dev, 4)
    comb = nrg.Combiner(dev, 2)
    a, b = comb.register(), comb.register()
    assert (a, b) == (0, 1)
    with pytest.raises(nrg.NrgError):  # past max_threads
        comb.register()
    with pytest.raises(ValueError):  # more than MAX_PENDING_OPS per call
        comb.put(a, np.arange(33), np.arange(33))
    with pytest.raises(ValueError):  # keys and values of different lengths
        comb.put(a, np.arange(3), np.arange(2))
    recs = np.zeros(33, nrg.PUT_DTYPE)
    with pytest.raises(nrg.NrgError):  # the C ABI refuses it too
        comb.execute_mut(a, recs)
    prev, some = comb.put(a, [7, 7], [1, 2])
    assert list(some) == [0, 1] and int(prev[1]) == 1
    vals, found = comb.get(b, [7, 8])
    assert list(found) == [1, 0] and int(vals[0]) == 2
    comb.close()
    dev.close()


def test_combiner_token_in_use(nrg):
    """One call at a time per token (include/nrgpu.h): two threads driving ONE token. A call that
    finds its token's previous call still waiting for its round is refused with NRG_E_INVAL,
    instead of reserving past the batch's buffers; the calls that were accepted all complete,
    and the final table is the oracle's replay of exactly the accepted Puts."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=4096, max_reads=4096)
    comb = nrg.Combiner(dev, 2)
    tok = comb.register()
    accepted, refused, errors = [[], []], [0, 0], []

    def client(who):
        rng = np.random.default_rng(40 + who)
        # batches made up front, so the two threads' calls follow each other as closely as
        # Python allows; at least 300 calls each, then on until the threads have collided (a
        # round of the resident server takes ~15 us, so a collision can take a while)
        K = rng.integers(0, 3000, (20000, 32), dtype=np.uint64)
        V = rng.integers(0, 2**63, (20000, 32), dtype=np.uint64)
        try:
            for it in range(20000):
                if it >= 300 and refused[0] + refused[1] > 0:
                    break
                keys, vals = K[it], V[it]
                try:
                    comb.put(tok, keys, vals)
                    accepted[who].append((keys, vals))
                except nrg.NrgError as e:
                    if e.code != nrg._lib.NRG_E_INVAL:
                        raise
                    refused[who] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    _run_threads(2, client)
    assert not errors, errors[0]
    assert refused[0] + refused[1] > 0  # the two threads did collide on the token
    comb.close()
    # each thread's accepted calls are in its own order; the two threads' keys interleave, so
    # compare the final table only over keys one thread alone wrote
    only = [set(), set()]
    for w in (0, 1):
        for k, _ in accepted[w]:
            only[w].update(int(x) for x in k)
    mine = [only[0] - only[1], only[1] - only[0]]
    keys, vals = dev.hm_dump()
    table = dict(zip((int(k) for k in keys), (int(v) for v in vals)))
    for w in (0, 1):
        last = {}
        for k, v in accepted[w]:
            for a, b in zip(k, v):
                last[int(a)] = int(b)
        for k in mine[w]:
            assert table[k] == last[k], (w, k)
    dev.close()


def _read_log(nrg, dev, dtype):
    """The replica's log [head, tail) as records (nrgpu_testing.h nrg_test_ring_read)."""
    import ctypes as C

    lib = nrg._lib.load()
    st = dev.log_state()
    out = np.zeros(st["tail"] - st["head"], dtype)
    rec = np.zeros(1, dtype)
    for i in range(st["head"], st["tail"]):
        nrg._lib.check(lib.nrg_test_ring_read(dev.handle, i & (st["size"] - 1), C.c_void_p(rec.ctypes.data)))
        out[i - st["head"]] = rec[0]
    return out


def _run_threads(T, fn):
    errors = []

    def wrap(i):
        try:
            fn(i)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=wrap, args=(i,)) for i in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[0]


def test_combiner_stack_threads(nrg, orc):
    """Stack replica behind the combiner (configs[4]'s data structure, nr/tests/stack.rs):
    phase 1, T threads push and pop concurrently in calls of 1..32 mixed ops; every call's pop
    values equal the oracle's replay of the replica's log at the call's positions. Phase 2
    (parallel_push_sequential_pop, nr/tests/stack.rs:282-343): threads push increasing values,
    then one thread pops everything and each pusher's values come out decreasing (VerifyStack)."""
    T, CALLS = 8, 30
    L = nrg._lib
    dev = nrg.DeviceReplica(L.NRG_DS_STACK, 0, max_batch=1 << 12, stack_capacity=1 << 20, log_bytes=64 * (1 << 17))
    init = np.arange(100, dtype=np.uint32)
    dev.st_init(init)
    comb = nrg.Combiner(dev, T)
    calls = {}

    def client(i):
        tok = comb.register()
        rng = np.random.default_rng(500 + i)
        mine = []
        for c in range(CALLS):
            n = int(rng.integers(1, 33))
            recs = np.zeros(n, nrg.STACK_OP_DTYPE)
            recs["op"] = rng.integers(0, 2, n)
            recs["op"][0] = L.NRG_STACK_PUSH  # every call starts with a unique Push: finds it in the log
            recs["val"] = ((tok + 1) << 24) | (c << 8) | np.arange(n)
            resp, some = comb.execute_mut(tok, recs)
            mine.append((recs, resp, some))
            if c % 7 == 3:
                top, has = comb.execute(tok, n=4)  # Peek
                assert np.all(has == has[0]) and np.all(top == top[0])
        calls[tok] = mine

    _run_threads(T, client)
    log = _read_log(nrg, dev, nrg.STACK_OP_DTYPE)
    ost = orc.Stack(init)
    oresp, osome = ost.replay(log["val"], log["op"])
    pos = {int(v): i for i, (v, o) in enumerate(zip(log["val"], log["op"])) if o == L.NRG_STACK_PUSH}
    for tok, mine in calls.items():
        for recs, resp, some in mine:
            p = pos[int(recs["val"][0])]
            n = len(recs)
            np.testing.assert_array_equal(log[p:p + n], recs)  # a call's ops are contiguous in the log
            np.testing.assert_array_equal(some, osome[p:p + n])
            np.testing.assert_array_equal(resp, oresp[p:p + n])
    rounds, ops = comb.stats()
    assert ops == len(log) + sum(4 for m in calls.values() for c in range(CALLS) if c % 7 == 3)

    # phase 2: parallel pushes, then sequential pops (VerifyStack's invariant)
    base = len(ost.dump())

    def pusher(i):
        tok = i  # tokens 0..T-1 are taken; pushes carry the pusher id in the low byte
        for c in range(20):
            recs = np.zeros(8, nrg.STACK_OP_DTYPE)
            recs["op"] = L.NRG_STACK_PUSH
            recs["val"] = ((c * 8 + np.arange(8)) << 8) | (0x80 | tok)
            comb.execute_mut(tok, recs)

    _run_threads(T, pusher)
    last = {}
    popped = 0
    while True:
        recs = np.zeros(32, nrg.STACK_OP_DTYPE)  # Pops
        resp, some = comb.execute_mut(0, recs)
        for v, s_ in zip(resp, some):
            if not s_:
                continue
            if (int(v) & 0x80) and popped < 20 * 8 * T:
                tid, seq = int(v) & 0x7F, int(v) >> 8
                assert seq < last.get(tid, 1 << 30), "a pusher's values come out decreasing"
                last[tid] = seq
                popped += 1
        if not np.all(some):
            break
    assert popped == 20 * 8 * T and len(last) == T
    assert base > 0
    comb.close()
    assert dev.st_len() == 0
    dev.close()


def test_combiner_synthetic_threads(nrg, orc):
    """AbstractDataStructure behind the combiner: concurrent ReadWrite/WriteOnly calls whose
    sums equal the oracle's replay of the replica's log, then ReadOnly reads against the final
    storage, which equals the oracle's."""
    T, CALLS = 8, 25
    L = nrg._lib
    dev = nrg.DeviceReplica(L.NRG_DS_SYNTHETIC, 0, max_batch=1 << 12, log_bytes=64 * (1 << 17))
    comb = nrg.Combiner(dev, T)
    calls = {}

    def client(i):
        tok = comb.register()
        rng = np.random.default_rng(900 + i)
        mine = []
        for c in range(CALLS):
            n = int(rng.integers(1, 33))
            recs = np.zeros(n, nrg.SYNTH_OP_DTYPE)
            recs["tid"] = tok
            recs["r1"] = rng.integers(0, 2**63, n, dtype=np.uint64)
            recs["r2"] = rng.integers(0, 2**63, n, dtype=np.uint64)
            recs["op"] = (rng.integers(0, 10, n) > 0).astype(np.uint64)
            resp, some = comb.execute_mut(tok, recs)
            assert np.all(some == 1)
            mine.append((recs, resp))
        calls[tok] = mine

    _run_threads(T, client)
    log = _read_log(nrg, dev, nrg.SYNTH_OP_DTYPE)
    os_ = orc.Synthetic()
    oresp = os_.replay(np.stack([log["tid"], log["r1"], log["r2"], log["op"]], axis=1))
    pos = {int(r): i for i, r in enumerate(log["r1"])}
    for tok, mine in calls.items():
        for recs, resp in mine:
            p = pos[int(recs["r1"][0])]
            n = len(recs)
            np.testing.assert_array_equal(log[p:p + n], recs)
            np.testing.assert_array_equal(resp, oresp[p:p + n])
    rd = np.zeros(20, nrg.SYNTH_RD_DTYPE)
    raw = orc.gen_raw(60, 5)
    rd["tid"], rd["r1"], rd["r2"] = raw[0::3] % 8, raw[1::3], raw[2::3]
    got, some = comb.execute(0, rd)
    np.testing.assert_array_equal(got, os_.read(np.stack([rd["tid"], rd["r1"], rd["r2"]], axis=1)))
    assert np.all(some == 1)
    comb.close()
    np.testing.assert_array_equal(dev.sy_dump(), os_.dump())
    dev.close()
