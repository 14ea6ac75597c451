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
