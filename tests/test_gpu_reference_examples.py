"""The reference's own example programs, run on GPU replicas through the Replica API mirror.

nr/examples/hashmap.rs and nr/examples/stack.rs are the reference's data-plane programs with a
fixed, deterministic op sequence per thread: one 2-MiB log, two replicas, three threads (two on
the first replica, one on the second) issuing `execute_mut` / `execute` in a loop of 2048. The
hashmap example carries the reference's own known answer, `assert_eq!(response, Some(i))` for the
`Get(i - 1)` that follows each thread's `Put(i - 1, i)` (nr/examples/hashmap.rs:67-78). The stack
example asserts nothing; what its sequence guarantees is checked instead: a thread pushes before it
pops (i % 3 == 0 Push(i), 1 Pop, 2 Peek, nr/examples/stack.rs), so the depth never falls below the
1000 elements of Stack::default (:24-37), every Peek finds an element, and the final stack is
exactly 0..999. Both examples end with the two replicas equal (Replica::verify).
"""
import threading

import pytest

pytestmark = pytest.mark.gpu


def _run_threads(fns):
    errors = []

    def wrap(f):
        try:
            f()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    assert not errors, errors


def test_nr_example_hashmap(nrg):
    """nr/examples/hashmap.rs main(): Put(i, i + 1) for even i, Get(i - 1) == Some(i) for odd i."""
    log = nrg.Log(2 * 1024 * 1024)
    replica1 = nrg.Replica(log, nrg.NrHashMap, 0, log2_slots=14)
    replica2 = nrg.Replica(log, nrg.NrHashMap, 0, log2_slots=14)
    seen = {}

    def thread_loop(replica, name):
        ridx = replica.register()
        assert ridx is not None, "Unable to register with log"
        got = []
        for i in range(2048):
            if i % 2 == 0:
                replica.execute_mut(nrg.Put(i, i + 1), ridx)
            else:
                response = replica.execute(nrg.Get(i - 1), ridx)
                assert response == i, (name, i, response)  # assert_eq!(response, Some(i))
                got.append(response)
        seen[name] = got

    _run_threads([lambda: thread_loop(replica1, "t1"), lambda: thread_loop(replica1, "t2"),
                  lambda: thread_loop(replica2, "t3")])
    assert sorted(seen) == ["t1", "t2", "t3"]
    states = []
    for r in (replica1, replica2):
        r.verify(lambda d: states.append(dict(d)))
    assert states[0] == states[1] == {k: k + 1 for k in range(0, 2048, 2)}
    for r in (replica1, replica2):
        r.dev.close()


def test_nr_example_stack(nrg):
    """nr/examples/stack.rs main(): Push(i) / Pop / Peek by i % 3 over Stack::default (0..999)."""
    log = nrg.Log(2 * 1024 * 1024)
    replicas = [nrg.Replica(log, nrg.Stack, 0) for _ in range(2)]
    for r in replicas:
        r.dev.st_init(list(range(1000)))  # Stack::default: DEFAULT_STACK_SIZE = 1000
    peeks = []

    def thread_loop(replica):
        ridx = replica.register()
        assert ridx is not None, "Unable to register with log"
        for i in range(2048):
            if i % 3 == 0:
                assert replica.execute_mut(nrg.Push(i), ridx) is None  # Push -> None
            elif i % 3 == 1:
                assert replica.execute_mut(nrg.Pop(), ridx) is not None  # never below 1000
            else:
                peeks.append(replica.execute(nrg.Peek(), ridx))

    _run_threads([lambda: thread_loop(replicas[0]), lambda: thread_loop(replicas[0]),
                  lambda: thread_loop(replicas[1])])
    assert len(peeks) == 3 * len(range(2, 2048, 3)) and all(p is not None for p in peeks)
    states = []
    for r in replicas:
        r.verify(lambda d: states.append(list(d)))
    assert states[0] == states[1] == list(range(1000))
    for r in replicas:
        r.dev.close()
