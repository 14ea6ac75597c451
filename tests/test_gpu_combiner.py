"""Native flat combining (nrg_combiner_*): many client threads, one GPU round per combine.

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


def test_combiner_threads(nrg, orc):
    T, ITERS, SPAN = 8, 40, 5000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=18, max_batch=1 << 12, max_reads=1 << 12,
                            log_bytes=64 * (1 << 16))
    dev.hm_prefill_range(1000, 1)  # keys 0..999 -> k + 1: thread 0's range starts with them
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


def test_combiner_limits(nrg):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=12, max_batch=64, max_reads=64)
    with pytest.raises(nrg.NrgError):  # 4 threads x 32 ops exceed max_batch
        nrg.Combiner(dev, 4)
    comb = nrg.Combiner(dev, 2)
    a, b = comb.register(), comb.register()
    assert (a, b) == (0, 1)
    with pytest.raises(nrg.NrgError):  # past max_threads
        comb.register()
    with pytest.raises(nrg.NrgError):  # more than MAX_PENDING_OPS per call
        comb.put(a, np.arange(33), np.arange(33))
    prev, some = comb.put(a, [7, 7], [1, 2])
    assert list(some) == [0, 1] and int(prev[1]) == 1
    vals, found = comb.get(b, [7, 8])
    assert list(found) == [1, 0] and int(vals[0]) == 2
    comb.close()
    dev.close()
