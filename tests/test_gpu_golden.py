"""Replay the committed golden fixtures (tests/golden/*.npz) through libnrgpu.so.

The fixtures come from tests/golden/make_golden.py: pure-Python dict / list / wrapping-int
models of the reference's Dispatch impls (nr/examples/hashmap.rs:46-50, benches/hashmap.rs:77-122,
benches/stack.rs:36-84, nr/tests/stack.rs:42-96, benches/synthetic.rs:112-195), independent of
both the C oracle and the HIP path. Here the HIP path is compared with the fixture contents
directly: every response, every read and the final replica state. The stack fixtures restate
nr/tests/stack.rs:102-168's sequential_test (random push/pop against a Vec model, then verify).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.mark.parametrize("name", ["hashmap_small.npz", "hashmap_sparse.npz"])
@pytest.mark.parametrize("path", ["stamp", "part", "wide"])
def test_hashmap_fixture_on_gpu(nrg, name, path):
    """Rounds of Log::append + Log::exec with HashMap::insert's previous values, then the
    round's Gets; sorted final contents equal the fixture's dict. The previous-value rounds take
    partition rounds; the same stream without responses also runs through the stamp rounds
    ("stamp") and through partition rounds ("part")."""
    d = _load(name)
    W, R, rounds = int(d["W"]), int(d["R"]), int(d["rounds"])
    knobs = {"part": {"PART": 2}, "wide": {"PART": 2, "PA_TPB": 1024}}.get(path, {})
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=knobs, log2_slots=16, max_batch=4096)
    dev.hm_prefill_range(int(d["prefill"]), 1)
    for r in range(rounds):
        recs = np.zeros(W, nrg.PUT_DTYPE)
        recs["key"] = d["puts_k"][r * W:(r + 1) * W]
        recs["val"] = d["puts_v"][r * W:(r + 1) * W]
        first = dev.log_append(recs, 1)
        if r % 2 == 0:
            prev, pf = dev.log_exec(first, first + W)
            np.testing.assert_array_equal(pf, d["prev_f"][r * W:(r + 1) * W], err_msg=f"round {r} prev found")
            np.testing.assert_array_equal(prev, d["prev_v"][r * W:(r + 1) * W], err_msg=f"round {r} prev")
        else:
            dev.log_exec()  # Ok(None) responses (benches/hashmap.rs:114-119)
        gv, gf = dev.hm_get(d["gets_k"][r * R:(r + 1) * R])
        np.testing.assert_array_equal(gf, d["get_f"][r * R:(r + 1) * R], err_msg=f"round {r} get found")
        np.testing.assert_array_equal(gv, d["get_v"][r * R:(r + 1) * R], err_msg=f"round {r} get vals")
    k, v = dev.hm_dump()
    np.testing.assert_array_equal(k, d["final_k"])
    np.testing.assert_array_equal(v, d["final_v"])
    dev.close()


@pytest.mark.parametrize("name", ["stack_sequential.npz", "stack_push_some.npz"])
def test_stack_fixture_on_gpu(nrg, name):
    d = _load(name)
    n = int(d["n"])
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1024, stack_capacity=1 << 16,
                            stack_push_resp=int(d["push_resp"]))
    dev.st_init(np.arange(int(d["init_n"]), dtype=np.uint32))
    recs = np.zeros(n, nrg.STACK_OP_DTYPE)
    recs["val"], recs["op"] = d["vals"], d["ops"]
    first = dev.log_append(recs, 1)
    resp, some = dev.log_exec(first, first + n)  # 4 chunks of max_batch: cross-chunk pops too
    np.testing.assert_array_equal(some, d["some"])
    np.testing.assert_array_equal(resp, d["resp"])
    np.testing.assert_array_equal(dev.st_dump(), d["final"])
    top = d["final"][-1] if len(d["final"]) else None
    assert dev.st_peek() == (int(top) if top is not None else None)
    dev.close()


def test_synthetic_fixture_on_gpu(nrg):
    d = _load("synthetic_small.npz")
    ops = np.ascontiguousarray(d["ops"])
    n = ops.shape[0]
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, synth_n=int(d["words"]), max_batch=1024)
    recs = np.zeros(n, nrg.SYNTH_OP_DTYPE)
    recs["tid"], recs["r1"], recs["r2"], recs["op"] = ops[:, 0], ops[:, 1], ops[:, 2], ops[:, 3]
    first = dev.log_append(recs, 1)
    resp, some = dev.log_exec(first, first + n)
    np.testing.assert_array_equal(resp, d["resp"])
    np.testing.assert_array_equal(dev.sy_dump(), d["final"])
    rd = np.zeros(len(d["reads"]), nrg.SYNTH_RD_DTYPE)
    rd["tid"], rd["r1"], rd["r2"] = d["reads"][:, 0], d["reads"][:, 1], d["reads"][:, 2]
    np.testing.assert_array_equal(dev.sy_read(rd), d["read_sums"])
    dev.close()
