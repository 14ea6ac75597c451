"""nr/tests/stack.rs VerifyStack tests (:170-404) over GPU replicas: several threads on two
replicas push (seq << 16 | tid) elements through one shared log, then pop them; the elements
that came from a given thread must come off the stack in strictly decreasing seq order, and every
pushed element must be popped exactly once. The reference asserts this inside dispatch_mut; here
the pop responses returned to the callers are checked."""
import threading

import pytest

pytestmark = pytest.mark.gpu

NREP, NTHR, NOP, BATCH = 2, 4, 3000, 200


def _push_phase(nrg, reps, barrier, errors):
    def worker(rep, tid):
        try:
            tok = rep.register()
            barrier.wait()
            for s in range(0, NOP, BATCH):
                ops = [nrg.Push((i << 16) | tid) for i in range(s, min(NOP, s + BATCH))]
                rep.execute_mut_batch(ops, tok)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(reps[i], i * NTHR + j)) for i in range(NREP) for j in range(NTHR)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)


def _check_decreasing(popped):
    last = {}
    for v in popped:
        tid, seq = v & 0xFFFF, v >> 16
        assert seq < last.get(tid, 1 << 16), "Elements that came from a given thread are monotonically decreasing"
        last[tid] = seq


def test_parallel_push_sequential_pop(nrg):
    log = nrg.Log(64 << 20)
    reps = [nrg.Replica(log, nrg.Stack, 0, stack_capacity=1 << 16) for _ in range(NREP)]
    errors = []
    _push_phase(nrg, reps, threading.Barrier(NREP * NTHR), errors)
    assert not errors, errors
    total = NREP * NTHR * NOP
    rep = reps[0]
    tok = rep.register()
    popped = []
    for s in range(0, total, 1000):
        top = rep.execute(nrg.Peek(), tok)
        got = rep.execute_mut_batch([nrg.Pop()] * min(1000, total - s), tok)
        assert got[0] == top  # Peek sees the element the next Pop removes
        popped += got
    assert None not in popped
    _check_decreasing(popped)
    want = sorted((i << 16) | t for t in range(NREP * NTHR) for i in range(NOP))
    assert sorted(popped) == want
    assert rep.execute(nrg.Peek(), tok) is None
    states = []
    for r in reps:
        r.verify(lambda d: states.append(d))
    assert states[0] == states[1] == []
    for r in reps:
        r.dev.close()


def test_parallel_push_and_pop(nrg):
    log = nrg.Log(64 << 20)
    reps = [nrg.Replica(log, nrg.Stack, 0, stack_capacity=1 << 16) for _ in range(NREP)]
    errors = []
    _push_phase(nrg, reps, threading.Barrier(NREP * NTHR), errors)
    assert not errors, errors
    results = {}
    barrier = threading.Barrier(NREP * NTHR)

    def popper(rep, tid):
        try:
            tok = rep.register()
            barrier.wait()
            out = []
            for s in range(0, NOP, BATCH):
                out += rep.execute_mut_batch([nrg.Pop()] * min(BATCH, NOP - s), tok)
            results[tid] = out
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=popper, args=(reps[i], i * NTHR + j)) for i in range(NREP) for j in range(NTHR)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not errors, errors
    allp = []
    for tid, out in results.items():
        assert None not in out
        _check_decreasing(out)  # each thread's pops are a subsequence of the log order
        allp += out
    want = sorted((i << 16) | t for t in range(NREP * NTHR) for i in range(NOP))
    assert sorted(allp) == want
    for r in reps:
        r.dev.close()
