"""The reference's public API (Log / Replica / ReplicaToken / execute / execute_mut / verify)
over GPU replicas, tested the way nr/tests/stack.rs tests it: a sequential run against a
Vec/HashMap model (sequential_test, :102-168) and several replicas driven by concurrent
threads through one shared log ending in identical state (replicas_are_equal, :434-489)."""
import random
import threading

import pytest

pytestmark = pytest.mark.gpu


def test_stack_sequential_against_vec_model(nrg):
    rng = random.Random(0x5EC)
    log = nrg.Log(4 * 1024 * 1024)
    r = nrg.Replica(log, nrg.Stack, 0, stack_push_resp=1)  # Push -> Some(v) as nr/tests/stack.rs:89-92
    tok = r.register()
    model = []
    for _ in range(50):
        e = rng.getrandbits(32)
        assert r.execute_mut(nrg.Push(e), tok) == e
        model.append(e)
    for _ in range(400):
        op = rng.getrandbits(64) % 3
        if op == 0:
            assert r.execute_mut(nrg.Pop(), tok) == (model.pop() if model else None)
        elif op == 1:
            e = rng.getrandbits(32)
            assert r.execute_mut(nrg.Push(e), tok) == e
            model.append(e)
        else:
            assert r.execute(nrg.Peek(), tok) == (model[-1] if model else None)
    seen = []
    r.verify(lambda data: seen.append(list(data)))
    assert seen[0] == model
    r.dev.close()


def test_hashmap_sequential_against_dict_model(nrg):
    rng = random.Random(0xA5)
    log = nrg.Log(1 << 20)
    r = nrg.Replica(log, nrg.NrHashMap, 0, log2_slots=14)
    tok = r.register()
    model = {}
    for _ in range(600):
        k = rng.randrange(300) if rng.random() < 0.95 else (1 << 64) - 1  # side-slot key too
        if rng.random() < 0.5:
            v = rng.getrandbits(64)
            assert r.execute_mut(nrg.Put(k, v), tok) == model.get(k)
            model[k] = v
        else:
            assert r.execute(nrg.Get(k), tok) == model.get(k)
    batch = [nrg.Put(rng.randrange(300), rng.getrandbits(64)) for _ in range(200)]
    got = r.execute_mut_batch(batch, tok)
    for op, g in zip(batch, got):
        assert g == model.get(op.key)
        model[op.key] = op.val
    seen = []
    r.verify(lambda d: seen.append(d))
    assert seen[0] == model
    r.dev.close()


@pytest.mark.parametrize("ds", ["stack", "hashmap"])
def test_replicas_are_equal(nrg, ds):
    nrep, nthr, nop = 2, 4, 60
    log = nrg.Log(1 << 20)
    if ds == "stack":
        reps = [nrg.Replica(log, nrg.Stack, 0) for _ in range(nrep)]
    else:
        reps = [nrg.Replica(log, nrg.NrHashMap, 0, log2_slots=14) for _ in range(nrep)]
    barrier = threading.Barrier(nrep * nthr)
    errors = []

    def worker(rep, seed):
        try:
            tok = rep.register()
            rng = random.Random(seed)
            barrier.wait()
            for _ in range(nop):
                if ds == "stack":
                    op = nrg.Push(rng.getrandbits(32)) if rng.random() < 0.6 else nrg.Pop()
                else:
                    op = nrg.Put(rng.randrange(100), rng.getrandbits(64))
                rep.execute_mut(op, tok)
            barrier.wait()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(reps[i], 100 * i + j)) for i in range(nrep) for j in range(nthr)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errors, errors
    states = []
    for rep in reps:
        rep.verify(lambda d: states.append(d))
    assert states[0] == states[1], "Data-structures don't match."
    for rep in reps:
        rep.dev.close()


@pytest.mark.parametrize("ds", ["stack", "hashmap"])
def test_late_replica_catches_up(nrg, ds):
    """A replica registered after three rounds of writes (nr/src/log.rs:272-292: register at any
    time; the new replica's ltail is 0) replays the live log on its first read (sync to ctail,
    nr/src/replica.rs:469-479, :483-497) and ends equal to the first replica and the model."""
    rng = random.Random(0x1A7E)
    log = nrg.Log(1 << 20)
    mk = (lambda: nrg.Replica(log, nrg.Stack, 0)) if ds == "stack" else (
        lambda: nrg.Replica(log, nrg.NrHashMap, 0, log2_slots=14))
    a = mk()
    ta = a.register()
    model = [] if ds == "stack" else {}
    for _ in range(3):
        if ds == "stack":
            ops = [nrg.Push(rng.getrandbits(32)) if rng.random() < 0.7 else nrg.Pop() for _ in range(150)]
        else:
            ops = [nrg.Put(rng.randrange(400), rng.getrandbits(64)) for _ in range(150)]
        a.execute_mut_batch(ops, ta)
        for op in ops:
            if ds == "stack":
                if isinstance(op, nrg.Push):
                    model.append(op.val)
                elif model:
                    model.pop()
            else:
                model[op.key] = op.val
    b = mk()  # registered after 450 appended entries
    assert b.idx == 2 and b.dev.log_state()["ltail"] == 0
    tb = b.register()
    if ds == "stack":
        assert b.execute(nrg.Peek(), tb) == (model[-1] if model else None)
    else:
        for k in range(0, 400, 7):
            assert b.execute(nrg.Get(k), tb) == model.get(k)
    # both keep going on the shared log
    more = [nrg.Push(5), nrg.Pop()] if ds == "stack" else [nrg.Put(1, 2), nrg.Put(3, 4)]
    b.execute_mut_batch(more, tb)
    if ds == "stack":
        model.append(5)
        model.pop()
    else:
        model[1], model[3] = 2, 4
    states = []
    for r in (a, b):
        r.verify(lambda d: states.append(d))
    assert states[0] == states[1] == model
    for r in (a, b):
        r.dev.close()


def test_late_replica_after_gc_is_refused(nrg):
    """Once GC has moved head past entry 0 a late replica cannot replay from its ltail 0 (the
    reference panics, nr/src/log.rs:486-488): registration fails with a clear error."""
    log = nrg.Log(2 * 64 * 8192)  # the smallest log: 16384 entries, GC within 8192 of full
    a = nrg.Replica(log, nrg.NrHashMap, 0, log2_slots=16, max_batch=4096, log_bytes=log.bytes)
    ta = a.register()
    for r in range(4):
        a.execute_mut_batch([nrg.Put(k, r) for k in range(3000)], ta)
    assert log.head > 0
    with pytest.raises(RuntimeError, match="garbage-collected"):
        nrg.Replica(log, nrg.NrHashMap, 0, log2_slots=16, max_batch=4096)
    a.dev.close()
