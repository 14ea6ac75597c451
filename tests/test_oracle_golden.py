"""Pin the C oracle (oracle/nr_oracle.c) against the golden fixtures in tests/golden/.

The fixtures come from tests/golden/make_golden.py (pure-Python dict / list / wrapping-int
models of the reference's Dispatch impls), so this test checks the oracle against an
independent restatement and against the published splitmix64 test vector. The GPU test
tests/test_gpu_golden.py replays the same fixtures through libnrgpu.so.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_splitmix_known_answer(orc):
    d = _load("splitmix.npz")
    # published splitmix64 outputs for state 0 (Vigna's reference implementation)
    assert int(d["seed0"][0]) == 0xE220A8397B1DCDAF
    assert int(d["seed0"][1]) == 0x6E789E6AA1B965F4
    assert int(d["seed0"][2]) == 0x06C45D188009454F
    np.testing.assert_array_equal(orc.gen_raw(16, 0), d["seed0"])
    np.testing.assert_array_equal(orc.gen_raw(16, 0x4E52475055310001), d["seed_x"])
    np.testing.assert_array_equal(orc.gen_uniform(64, 1234, 10_000_000), d["uniform"])


@pytest.mark.parametrize("name", ["hashmap_small.npz", "hashmap_sparse.npz"])
def test_hashmap_fixture(orc, name):
    d = _load(name)
    W, R, rounds = int(d["W"]), int(d["R"]), int(d["rounds"])
    m = orc.HashMap()
    m.prefill_range(int(d["prefill"]), 1)
    for r in range(rounds):
        pv, pf = m.replay(d["puts_k"][r * W:(r + 1) * W], d["puts_v"][r * W:(r + 1) * W])
        np.testing.assert_array_equal(pf, d["prev_f"][r * W:(r + 1) * W])
        np.testing.assert_array_equal(pv, d["prev_v"][r * W:(r + 1) * W])
        gv, gf = m.get_batch(d["gets_k"][r * R:(r + 1) * R])
        np.testing.assert_array_equal(gf, d["get_f"][r * R:(r + 1) * R])
        np.testing.assert_array_equal(gv, d["get_v"][r * R:(r + 1) * R])
    k, v = m.dump_sorted()
    np.testing.assert_array_equal(k, d["final_k"])
    np.testing.assert_array_equal(v, d["final_v"])


@pytest.mark.parametrize("name", ["stack_sequential.npz", "stack_push_some.npz"])
def test_stack_fixture(orc, name):
    d = _load(name)
    s = orc.Stack(np.arange(int(d["init_n"]), dtype=np.uint32))
    resp, some = s.replay(d["vals"], d["ops"], push_resp=bool(d["push_resp"]))
    np.testing.assert_array_equal(some, d["some"])
    np.testing.assert_array_equal(resp, d["resp"])
    np.testing.assert_array_equal(s.dump(), d["final"])


def test_synthetic_fixture(orc):
    d = _load("synthetic_small.npz")
    s = orc.Synthetic(n=int(d["words"]))
    np.testing.assert_array_equal(s.replay(d["ops"]), d["resp"])
    np.testing.assert_array_equal(s.dump(), d["final"])
    np.testing.assert_array_equal(s.read(d["reads"]), d["read_sums"])


def test_hashmap_oracle_vs_dict_random(orc):
    """Mixed put/get stream (benches/hashmap.rs:77-122 Dispatch) vs a Python dict."""
    is_put, keys, vals = orc.gen_hashmap_ops(20000, 3, 2000, 30)
    m = orc.HashMap()
    resp, some = m.run_mixed(is_put, keys, vals)
    d = {}
    for i in range(len(keys)):
        k, v = int(keys[i]), int(vals[i])
        old = d.get(k)
        if is_put[i]:
            d[k] = v
        assert bool(some[i]) == (old is not None)
        assert int(resp[i]) == (old if old is not None else 0)
    assert len(m) == len(d)
    assert m.digest()[0] == len(d)


def test_generators_shape(orc):
    is_put, keys, vals = orc.gen_hashmap_ops(10000, 11, 5000, 10)
    assert int(is_put.sum()) == 1000  # exactly write_ratio% of the stream (shuffled)
    assert keys.max() < 5000
    z = orc.gen_zipf(200_000, 5, 1000, 0.99)
    assert z.max() < 1000
    counts = np.bincount(z.astype(np.int64), minlength=1000)
    # Zipf(0.99): rank 0 is the most frequent and carries ~1/H(1000, 0.99) of the mass
    assert counts[0] == counts.max()
    zeta = sum(1.0 / (i ** 0.99) for i in range(1, 1001))
    assert abs(counts[0] / 200_000 - 1 / zeta) < 0.01
    vals, ops = orc.gen_stack_ops(1000, 1)
    assert set(np.unique(ops)) <= {0, 1}
