"""Stream-ordering contract of nrgpu.DeviceReplica's `*_device` helpers (GPUTEST_r04's red case).

A replica opens on its own non-blocking HIP stream, which is not ordered with torch's null
stream. Torch fills and copies on its current stream; the helpers must order the replica's work
after them, and torch's later reads after the replica's outputs. These tests make the race
deterministic: torch's stream sleeps (`torch.cuda._sleep`) before it writes a sentinel into the
response buffers, so an unordered replica round would finish first and the sentinel would land
on top of its responses. The round's results are checked bit-exactly against the oracle
(nr/tests/stack.rs:102-168 sequential semantics, benches/synthetic.rs:154-174,
benches/hashmap.rs:107-119).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SLEEP_CYCLES = 50_000_000  # tens of ms of spin on torch's stream: far longer than one round


def _stack_ops(vals, ops):
    import nrgpu

    r = np.zeros(len(ops), nrgpu.STACK_OP_DTYPE)
    r["val"], r["op"] = vals, ops
    return r


@pytest.mark.parametrize("pipeline", [0, 1])
def test_stack_round_ordered_after_torch_fill(nrg, orc, pipeline):
    import torch

    n = 200_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1 << 18, stack_capacity=1 << 22,
                            pipeline=pipeline, log_bytes=64 * 4 * (1 << 20))
    assert dev._lib.nrg_get_stream(dev.handle) != torch.cuda.current_stream().cuda_stream
    init = np.arange(50_000, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    outs = []
    for r in range(3):
        vals, ops = orc.gen_stack_ops(n, 0x517 + r)
        d_ops = torch.from_numpy(_stack_ops(vals, ops).view(np.int64).copy()).cuda()
        resp = torch.empty(n, dtype=torch.int32, device="cuda")
        some = torch.empty(n, dtype=torch.uint8, device="cuda")
        torch.cuda._sleep(SLEEP_CYCLES)
        resp.fill_(-1)
        some.fill_(7)  # no kernel path writes 7: a surviving 7 is an unordered round
        dev.st_round_device(d_ops, n, 1, resp, some)
        outs.append((resp, some, os_.replay(vals, ops)))
    dev.join()
    # read back on torch's stream only: no device-wide synchronize before the copies
    for r, (resp, some, (oresp, osome)) in enumerate(outs):
        s = some.cpu().numpy()
        assert np.count_nonzero(s == 7) == 0, f"round {r}: sentinel survived"
        np.testing.assert_array_equal(s, osome, err_msg=f"round {r} some")
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint32), oresp, err_msg=f"round {r} resp")
    dev.sync()
    np.testing.assert_array_equal(dev.st_dump(), os_.dump())
    dev.close()


def test_synth_round_ordered_after_torch_fill(nrg, orc):
    import torch

    n = 100_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, max_batch=1 << 17, log_bytes=64 * 4 * (1 << 19),
                            pipeline=1)
    os_ = orc.Synthetic()
    outs = []
    for r in range(3):
        ops = np.zeros(n, nrg.SYNTH_OP_DTYPE)
        raw = orc.gen_raw(4 * n, 0xA11 + r)
        ops["tid"], ops["r1"], ops["r2"], ops["op"] = raw[0::4] % 64, raw[1::4], raw[2::4], 1
        d_ops = torch.from_numpy(ops.view(np.int64).reshape(n, -1).copy()).cuda()
        resp = torch.empty(n, dtype=torch.int64, device="cuda")
        some = torch.empty(n, dtype=torch.uint8, device="cuda")
        torch.cuda._sleep(SLEEP_CYCLES)
        resp.fill_(-1)
        some.fill_(7)
        dev.sy_round_device(d_ops, n, 1, resp, some)
        outs.append((resp, some, os_.replay(np.stack([ops["tid"], ops["r1"], ops["r2"], ops["op"]], axis=1))))
    dev.join()
    for r, (resp, some, oresp) in enumerate(outs):
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint64), oresp, err_msg=f"round {r}")
        assert np.all(some.cpu().numpy() == 1)
    dev.close()


def test_hashmap_round_ordered_after_torch_fill(nrg, orc):
    import torch

    W, R = 3000, 20000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=18, max_batch=1 << 14, max_reads=1 << 15)
    om = orc.HashMap()
    dev.hm_prefill_range(5000, 1)
    om.prefill_range(5000, 1)
    for r in range(3):
        keys = orc.gen_uniform(W, 0xB00 + r, 10000)
        vals = orc.gen_raw(W, 0xC00 + r)
        gk = orc.gen_uniform(R, 0xD00 + r, 12000)
        puts = np.zeros(W, nrg.PUT_DTYPE)
        puts["key"], puts["val"] = keys, vals
        d_puts = torch.from_numpy(puts.view(np.int64).reshape(W, 2).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64).copy()).cuda()
        prev = torch.empty(W, dtype=torch.int64, device="cuda")
        pf = torch.empty(W, dtype=torch.uint8, device="cuda")
        gv = torch.empty(R, dtype=torch.int64, device="cuda")
        gf = torch.empty(R, dtype=torch.uint8, device="cuda")
        torch.cuda._sleep(SLEEP_CYCLES)
        for t in (prev, gv):
            t.fill_(-1)
        for t in (pf, gf):
            t.fill_(7)
        dev.hm_round_device(d_puts, W, 1, d_gk, R, gv, gf, prev, pf)
        oprev, opf = om.replay(keys, vals)
        ov, of = om.get_batch(gk)
        np.testing.assert_array_equal(pf.cpu().numpy(), opf, err_msg=f"round {r} prev found")
        np.testing.assert_array_equal(prev.cpu().numpy().view(np.uint64), oprev, err_msg=f"round {r} prev")
        np.testing.assert_array_equal(gf.cpu().numpy(), of, err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), ov, err_msg=f"round {r} vals")
    dev.close()


def test_unordered_call_does_race(nrg, orc):
    """NON-GATING DIAGNOSTIC (not coverage): the same sleep + sentinel fill around a RAW C-ABI
    call (no ordering) leaves the sentinel on top of the round's responses when the replica's
    stream and torch's run on different hardware queues -- the race the helpers close. The
    process has GPU_MAX_HW_QUEUES = 4 hardware queues, so once it has created more streams than
    that (earlier tests in the same run), HIP may map the replica's stream onto the queue of
    torch's, where the two are serialised in enqueue order and no race can happen; the control
    then skips. The gating tests above do not depend on the race showing: they check bit-exact
    responses with the sentinel fill enqueued before the round either way."""
    import ctypes as C

    import torch

    n = 200_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_STACK, 0, max_batch=1 << 18, stack_capacity=1 << 22)
    dev.st_init(np.arange(50_000, dtype=np.uint32))
    vals, ops = orc.gen_stack_ops(n, 0x517)
    d_ops = torch.from_numpy(_stack_ops(vals, ops).view(np.int64).copy()).cuda()
    resp = torch.empty(n, dtype=torch.int32, device="cuda")
    some = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    torch.cuda._sleep(SLEEP_CYCLES)
    some.fill_(7)
    rc = dev._lib.nrg_stack_round_async(dev.handle, C.c_void_p(d_ops.data_ptr()), n, 1,
                                        C.c_void_p(resp.data_ptr()), C.c_void_p(some.data_ptr()))
    assert rc == 0
    dev.sync()
    torch.cuda.synchronize()
    left = int(np.count_nonzero(some.cpu().numpy() == 7))
    dev.close()
    if left == 0:
        pytest.skip("non-gating diagnostic: the unordered call ran after the fill (streams sharing a hardware queue)")
