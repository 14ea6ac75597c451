"""Stack parity: HIP depth-scan replay vs the sequential Vec<u32> oracle.

Mirrors nr/tests/stack.rs `sequential_test` (:102-168: random push/pop/peek vs a Vec
model, then verify storage and popped values) and benches/stack.rs (50/50 push/pop over
an initial 50,000-element stack, :50-63, :87-102), with seeded streams.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ops(vals, ops):
    import nrgpu

    r = np.zeros(len(ops), nrgpu.STACK_OP_DTYPE)
    r["val"] = vals
    r["op"] = ops
    return r


@pytest.mark.parametrize("init_n,n,rounds,push_resp", [(0, 50, 3, 1), (1000, 5000, 4, 0), (50000, 200000, 3, 0),
                                                       (3, 20000, 2, 1)])
def test_stack_rounds(nrg, orc, init_n, n, rounds, push_resp):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1 << 18, stack_capacity=1 << 20,
                            stack_push_resp=push_resp)
    init = np.arange(init_n, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    for r in range(rounds):
        vals, ops = orc.gen_stack_ops(n, 77 + r)
        if init_n == 3:
            ops[: n // 2] = 0  # long runs of pops on an empty stack (saturating depth)
        first = dev.log_append(_ops(vals, ops), 1)
        resp, some = dev.log_exec(first, first + n)
        oresp, osome = os_.replay(vals, ops, push_resp=bool(push_resp))
        np.testing.assert_array_equal(some, osome)
        np.testing.assert_array_equal(resp, oresp)
        assert dev.st_len() == len(os_)
        assert dev.st_peek() == os_.peek()
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())


@pytest.mark.parametrize("init_n,n,rounds,push_resp", [(1000, 5000, 4, 0), (50000, 200000, 3, 0), (3, 20000, 3, 1)])
def test_stack_round_fused(nrg, orc, init_n, n, rounds, push_resp):
    """nrg_stack_round_async (append fused into the replay pass) == append + exec == the oracle;
    the log copy it writes is what a later exec of another replica replays."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1 << 18, stack_capacity=1 << 20,
                            stack_push_resp=push_resp)
    init = np.arange(init_n, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    resp = torch.zeros(n, dtype=torch.int32, device="cuda")
    some = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for r in range(rounds):
        vals, ops = orc.gen_stack_ops(n, 91 + r)
        if init_n == 3:
            ops[: n // 2] = 0  # long runs of pops on an empty stack (saturating depth)
        d_ops = torch.from_numpy(_ops(vals, ops).view(np.int64).copy()).cuda()
        dev.st_round_device(d_ops, n, 1, resp, some)
        torch.cuda.synchronize()
        oresp, osome = os_.replay(vals, ops, push_resp=bool(push_resp))
        np.testing.assert_array_equal(some.cpu().numpy(), osome)
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint32), oresp)
        assert dev.st_len() == len(os_)
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())


def test_stack_chunked_exec(nrg, orc):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=3000, stack_capacity=1 << 16)
    init = np.arange(100, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    vals, ops = orc.gen_stack_ops(10000, 5)
    first = dev.log_append(_ops(vals, ops), 1)
    resp, some = dev.log_exec(first, first + 10000)
    oresp, osome = os_.replay(vals, ops)
    np.testing.assert_array_equal(some, osome)
    np.testing.assert_array_equal(resp, oresp)
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())


def test_stack_capacity_error(nrg, orc):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1024, stack_capacity=100)
    dev.st_init(np.arange(90, dtype=np.uint32))
    dev.log_append(_ops(np.arange(20, dtype=np.uint32), np.ones(20, np.uint32)), 1)
    with pytest.raises(nrg.NrgError) as e:
        dev.log_exec()
    assert e.value.code == nrg._lib.NRG_E_CAPACITY


def test_stack_bench_size_rounds(nrg, orc):
    """BASELINE configs[4] at full size: initial 50,000 elements, rounds of 1M ops (50/50), pop
    responses and final storage bit-exact against the sequential Vec oracle."""
    import torch

    n = 1_000_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=n, stack_capacity=1 << 22,
                            log_bytes=64 * 4 * n)
    init = np.arange(50_000, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    resp = torch.zeros(n, dtype=torch.int32, device="cuda")
    some = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for r in range(3):
        vals, ops = orc.gen_stack_ops(n, 0x5AC + r)
        d_ops = torch.from_numpy(_ops(vals, ops).view(np.int64).copy()).cuda()
        dev.st_round_device(d_ops, n, 1, resp, some)
        torch.cuda.synchronize()
        oresp, osome = os_.replay(vals, ops)
        np.testing.assert_array_equal(some.cpu().numpy(), osome)
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint32), oresp)
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())


@pytest.mark.parametrize("init_n", [50_000, 0])
def test_stack_eight_segment_round(nrg, orc, init_n):
    """configs[4] on 8 GPUs: every replica replays the all-gathered round of 8 x 1M ops (8M ops in
    one chunk, nr/src/log.rs:473-524) and answers only its own segment (nr/src/replica.rs:576-578).
    Two rounds through nrg_log_append_segments_async + nrg_log_exec_async; with init_n = 0 the
    stack starts empty, so the first tiles pop an empty stack (Pop -> None, depth stays 0)."""
    import torch

    G, W = 8, 1_000_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=G * W, stack_capacity=1 << 24,
                            log_bytes=64 * 2 * G * W)
    init = np.arange(init_n, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    for r, own in enumerate([2, 7]):
        segs = [orc.gen_stack_ops(W, 0x8E5 + 10 * r + g) for g in range(G)]
        base = np.concatenate([_ops(v, o) for v, o in segs])
        d_base = torch.from_numpy(base.view(np.int64).copy()).cuda()
        firsts = dev.log_append_segments(d_base, W, [W] * G, [g + 1 for g in range(G)])
        assert firsts == [r * G * W + g * W for g in range(G)]
        resp = torch.full((W,), -1, dtype=torch.int32, device="cuda")
        some = torch.full((W,), 7, dtype=torch.uint8, device="cuda")
        dev.log_exec_device(firsts[own], firsts[own] + W, resp, some)
        torch.cuda.synchronize()
        for g, (v, o) in enumerate(segs):
            oresp, osome = os_.replay(v, o)
            if g == own:
                np.testing.assert_array_equal(some.cpu().numpy(), osome, err_msg=f"round {r} some")
                np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint32), oresp, err_msg=f"round {r} resp")
        assert dev.st_len() == len(os_.dump())
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())
    dev.close()


@pytest.mark.parametrize("init_n,n,rounds,stall", [(50000, 200000, 4, 0), (50000, 200000, 4, 1), (3, 20000, 3, 0),
                                                  (3, 20000, 3, 1), (0, 8192 * 3 + 77, 3, 0)])
def test_stack_pipelined_rounds(nrg, orc, init_n, n, rounds, stall):
    """pipeline=1: a chunk's finish (cross-tile Pops, commit) rides in the next chunk's launch
    (Replica::combine rounds back to back, nr/src/replica.rs:544-595); every round answers into
    its own buffers, complete after nrg_join. Then chunked exec (several chunks per call, each
    fused with the previous chunk's finish) and a final dump, all against the Vec oracle.
    stall = 1 (NRG_KNOB_STALL): odd waves sleep before reading the query structures and their
    lane stacks."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, knobs={"STALL": stall}, max_batch=1 << 18,
                            stack_capacity=1 << 22, pipeline=1, log_bytes=64 * 4 * (1 << 20))
    init = np.arange(init_n, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    outs = []
    for r in range(rounds):
        vals, ops = orc.gen_stack_ops(n, 301 + r)
        if init_n == 3:
            ops[: n // 2] = 0  # pops on an empty stack first
        d_ops = torch.from_numpy(_ops(vals, ops).view(np.int64).copy()).cuda()
        resp = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        some = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        dev.st_round_device(d_ops, n, 1, resp, some)
        outs.append((d_ops, resp, some, os_.replay(vals, ops)))
    dev.join()
    torch.cuda.synchronize()
    for r, (_, resp, some, (oresp, osome)) in enumerate(outs):
        np.testing.assert_array_equal(some.cpu().numpy(), osome, err_msg=f"round {r} some")
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint32), oresp, err_msg=f"round {r} resp")
    assert dev.st_len() == len(os_)
    # exec over several max_batch chunks (append + exec, 3 chunks of 2^18)
    vals, ops = orc.gen_stack_ops(3 * (1 << 18) - 5, 999)
    first = dev.log_append(_ops(vals, ops), 1)
    resp, some = dev.log_exec(first, first + len(ops))
    oresp, osome = os_.replay(vals, ops)
    np.testing.assert_array_equal(some, osome)
    np.testing.assert_array_equal(resp, oresp)
    assert dev.st_peek() == os_.peek()
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())
    dev.close()


def test_stack_op_words_and_load_paths(nrg, orc):
    """Any nonzero op word is a Push (the oracle's `if ops[i]`); rounds through both load paths of
    the tile pass: whole 16-B-aligned waves (coalesced 16-B loads) and partial or misaligned
    waves (8-B loads) -- odd round sizes shift the ring position off 16-B alignment and wrap it."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1 << 16, stack_capacity=1 << 20,
                            log_bytes=64 * 32768)
    init = np.arange(20, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    rng = np.random.default_rng(5)
    for r, n in enumerate([4096, 3001, 8192 + 5, 2048 * 5 + 1, 6000]):
        vals = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        ops = rng.choice(np.array([0, 0, 1, 2, 0xFFFFFFFF], np.uint32), n)
        if r % 2:
            first = dev.log_append(_ops(vals, ops), 1)
            resp, some = dev.log_exec(first, first + n)
        else:
            d_ops = torch.from_numpy(_ops(vals, ops).view(np.int64).copy()).cuda()
            rt = torch.zeros(n, dtype=torch.int32, device="cuda")
            st = torch.zeros(n, dtype=torch.uint8, device="cuda")
            dev.st_round_device(d_ops, n, 1, rt, st)
            torch.cuda.synchronize()
            resp, some = rt.cpu().numpy().view(np.uint32), st.cpu().numpy()
        oresp, osome = os_.replay(vals, ops)
        np.testing.assert_array_equal(some, osome, err_msg=f"round {r}")
        np.testing.assert_array_equal(resp, oresp, err_msg=f"round {r}")
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())
    dev.close()
