"""The multi-GPU replica group of the C ABI (nrg_group_*, RCCL over xGMI) on the box's GPU.

A 1-GPU box can only form groups of one rank (RCCL refuses two ranks on one device), so these
tests run the whole group path -- RCCL communicator, library-owned all-gather stream, rotating
gathered buffers, replay of the gathered log, reads and origin-only responses -- with nranks = 1,
through both constructors (nrg_group_open: one process drives its GPUs; nrg_group_join: one
process per GPU), against the sequential oracle. The rank-order concatenation of several
segments is covered by tests/test_gpu_group_multi.py (G = 2, 3 and 8 members on this GPU over
the loopback collectives of nrgpu_testing.h), tests/test_parallel.py (gloo, world 2 and 3) and
nrg_hashmap_round_segments_async's tests. RCCL itself with N > 1 runs only on a multi-GPU node
(the driver's scaling runs); no such run has been recorded yet.
Reference: nr/src/log.rs:494-511 (every replica replays every entry of the shared log).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _puts(keys, vals):
    import nrgpu

    r = np.zeros(len(keys), nrgpu.PUT_DTYPE)
    r["key"] = keys
    r["val"] = vals
    return r


def _cuda(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).cuda()


def _rounds_hashmap(lib, L, g, dev_ctx_sync, orc, seg_lens_fn):
    import torch

    om = orc.HashMap()
    outs = []
    for r in range(5):
        W, R = 3000 + 500 * r, 4000
        if r == 2:
            W = 0  # a round without writes: reads only
        keys = orc.gen_uniform(W, 70 + r, 6000)
        vals = orc.gen_raw(W, 80 + r)
        if W:
            keys[::91] = 0xFFFFFFFFFFFFFFFF  # the side-slot key
        gk = orc.gen_uniform(R, 90 + r, 6500)
        d = dict(puts=_cuda(_puts(keys, vals)) if W else None, gk=_cuda(gk),
                 gv=torch.full((R,), -1, dtype=torch.int64, device="cuda"),
                 gf=torch.full((R,), 7, dtype=torch.uint8, device="cuda"),
                 pv=torch.full((max(W, 1),), -1, dtype=torch.int64, device="cuda"),
                 pf=torch.full((max(W, 1),), 7, dtype=torch.uint8, device="cuda"))
        rd = L.Round()
        rd.recs = d["puts"].data_ptr() if W else 0
        rd.n = W
        rd.resp, rd.some = d["pv"].data_ptr(), d["pf"].data_ptr()
        rd.get_keys, rd.n_gets = d["gk"].data_ptr(), R
        rd.get_vals, rd.get_found = d["gv"].data_ptr(), d["gf"].data_ptr()
        lens = seg_lens_fn(W)
        L.check(lib.nrg_group_round_async(g, C.byref(rd), lens), "group round")
        pv, pf = om.replay(keys, vals)
        outs.append((d, W, pv, pf, om.get_batch(gk)))
    L.check(lib.nrg_group_sync(g))
    for r, (d, W, pv, pf, (gv, gf)) in enumerate(outs):
        if W:
            np.testing.assert_array_equal(d["pf"][:W].cpu().numpy(), pf, err_msg=f"round {r} prev found")
            np.testing.assert_array_equal(d["pv"][:W].cpu().numpy().view(np.uint64), pv, err_msg=f"round {r} prev")
        np.testing.assert_array_equal(d["gf"].cpu().numpy(), gf, err_msg=f"round {r} found")
        np.testing.assert_array_equal(d["gv"].cpu().numpy().view(np.uint64), gv, err_msg=f"round {r} vals")
    return om


def test_group_open_one_gpu_hashmap(nrg, orc):
    """nrg_group_open(devices=[0]): the group owns the replica; pipelined rounds through RCCL."""
    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_HASHMAP)
    cfg.log2_slots, cfg.max_batch, cfg.pipeline = 16, 8192, 1
    g = C.c_void_p()
    L.check(lib.nrg_group_open((C.c_int * 1)(0), 1, C.byref(cfg), C.byref(g)), "nrg_group_open")
    nr, nl, r0 = C.c_int(), C.c_int(), C.c_int()
    L.check(lib.nrg_group_info(g, C.byref(nr), C.byref(nl), C.byref(r0)))
    assert (nr.value, nl.value, r0.value) == (1, 1, 0)
    ctx = lib.nrg_group_replica(g, 0)
    assert ctx
    om = _rounds_hashmap(lib, L, g, None, orc, lambda W: None)
    out = np.zeros(3, np.uint64)
    L.check(lib.nrg_hashmap_digest(ctx, out.ctypes.data_as(C.c_void_p)))
    assert tuple(int(x) for x in out) == om.digest()
    info = L.LogInfo()
    L.check(lib.nrg_log_state(ctx, C.byref(info)))
    assert info.tail == info.ltail == info.ctail == sum(3000 + 500 * r for r in range(5) if r != 2)
    assert info.replica_id == 1
    L.check(lib.nrg_group_close(g))


def test_group_join_one_rank_hashmap(nrg, orc):
    """nrg_group_unique_id + nrg_group_join (one process per GPU), explicit seg_lens, an input
    stream separate from the replica stream (all-gathers run ahead of replays)."""
    import torch

    L = nrg._lib
    lib = L.load()
    dev = nrg.DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=8192, pipeline=1)
    dev.use_torch_stream()
    uid = (C.c_uint8 * L.NRG_GROUP_ID_BYTES)()
    L.check(lib.nrg_group_unique_id(uid))
    g = C.c_void_p()
    L.check(lib.nrg_group_join(dev.handle, uid, 1, 0, C.byref(g)), "nrg_group_join")
    side = torch.cuda.Stream()
    L.check(lib.nrg_group_set_input_stream(g, 0, C.c_void_p(side.cuda_stream)))
    torch.cuda.synchronize()
    om = _rounds_hashmap(lib, L, g, None, orc, lambda W: (C.c_uint64 * 1)(W))
    assert dev.hm_digest() == om.digest()
    L.check(lib.nrg_group_close(g))
    dev.close()


@pytest.mark.parametrize("pipeline", [0, 1])
def test_group_stack_rounds(nrg, orc, pipeline):
    """A stack replica group: pop responses for the member's own segment, final stack equal;
    with pipeline = 1 each round's finish rides in the next round's launch (nrg_group_sync
    completes the last one)."""
    import torch

    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_STACK)
    cfg.max_batch, cfg.stack_capacity, cfg.pipeline = 1 << 16, 1 << 20, pipeline
    g = C.c_void_p()
    L.check(lib.nrg_group_open((C.c_int * 1)(0), 1, C.byref(cfg), C.byref(g)), "nrg_group_open")
    ctx = lib.nrg_group_replica(g, 0)
    init = np.arange(1000, dtype=np.uint32)
    L.check(lib.nrg_stack_init(ctx, init.ctypes.data_as(C.c_void_p), len(init)))
    st = orc.Stack(init)
    outs = []
    for r in range(4):
        n = 20000 + 3000 * r
        vals, ops = orc.gen_stack_ops(n, 500 + r)
        recs = np.zeros(n, nrg.STACK_OP_DTYPE)
        recs["val"], recs["op"] = vals, ops
        d_ops = torch.from_numpy(recs.view(np.int64).copy()).cuda()
        resp = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        some = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        rd = L.Round()
        rd.recs, rd.n, rd.resp, rd.some = d_ops.data_ptr(), n, resp.data_ptr(), some.data_ptr()
        L.check(lib.nrg_group_round_async(g, C.byref(rd), None))
        outs.append((d_ops, resp, some, st.replay(vals, ops)))
    L.check(lib.nrg_group_sync(g))
    for r, (_, resp, some, (oresp, osome)) in enumerate(outs):
        np.testing.assert_array_equal(some.cpu().numpy(), osome, err_msg=f"round {r} some")
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint32), oresp, err_msg=f"round {r} resp")
    n = C.c_uint64()
    L.check(lib.nrg_stack_len(ctx, C.byref(n)))
    out = np.zeros(n.value, np.uint32)
    m = C.c_uint64()
    L.check(lib.nrg_stack_dump(ctx, out.ctypes.data_as(C.c_void_p), n.value, C.byref(m)))
    np.testing.assert_array_equal(out[:m.value], st.dump())
    L.check(lib.nrg_group_close(g))


@pytest.mark.parametrize("pipeline", [0, 1])
def test_group_synth_rounds(nrg, orc, pipeline):
    """A synthetic replica group (benches/synthetic.rs:112-195): per-op sums for the member's
    own segment and the final storage equal to the oracle; with pipeline = 1 each round's sums
    ride in the next round's partition launch."""
    import torch

    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_SYNTHETIC)
    cfg.max_batch, cfg.pipeline = 1 << 16, pipeline
    g = C.c_void_p()
    L.check(lib.nrg_group_open((C.c_int * 1)(0), 1, C.byref(cfg), C.byref(g)), "nrg_group_open")
    ctx = lib.nrg_group_replica(g, 0)
    os_ = orc.Synthetic()
    outs = []
    for r in range(4):
        n = 20000 + 3000 * r
        raw = orc.gen_raw(4 * n, 700 + r)
        recs = np.zeros(n, nrg.SYNTH_OP_DTYPE)
        recs["tid"], recs["r1"], recs["r2"] = raw[0::4] % 64, raw[1::4], raw[2::4]
        recs["op"] = (raw[3::4] % 100 >= 5).astype(np.uint64)
        d_ops = torch.from_numpy(recs.view(np.int64).reshape(n, -1).copy()).cuda()
        resp = torch.full((n,), -1, dtype=torch.int64, device="cuda")
        some = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        rd = L.Round()
        rd.recs, rd.n, rd.resp, rd.some = d_ops.data_ptr(), n, resp.data_ptr(), some.data_ptr()
        L.check(lib.nrg_group_round_async(g, C.byref(rd), None))
        outs.append((d_ops, resp, some, os_.replay(np.stack([recs["tid"], recs["r1"], recs["r2"], recs["op"]], axis=1))))
    L.check(lib.nrg_group_sync(g))
    for r, (_, resp, some, oresp) in enumerate(outs):
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint64), oresp, err_msg=f"round {r}")
        assert np.all(some.cpu().numpy() == 1)
    words = np.zeros(cfg.synth_n, np.uint64)
    m = C.c_uint64()
    L.check(lib.nrg_synth_dump(ctx, words.ctypes.data_as(C.c_void_p), cfg.synth_n, C.byref(m)))
    np.testing.assert_array_equal(words[:m.value], os_.dump())
    L.check(lib.nrg_group_close(g))
