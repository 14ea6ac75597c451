"""group.cpp's multi-rank path on the box's one GPU, against the oracle.

A 1-GPU box cannot form an RCCL group of more than one rank, so these tests switch the replica
groups to the in-process loopback collectives of include/nrgpu_testing.h
(nrg_test_loopback_collectives) and open G = 2, 3 and 8 members on device 0
(nrg_group_open(devices = {0, ..., 0})). Everything above the collective calls is the product
code that runs over RCCL on an 8-GPU node: segment lengths and the common stride, the padding of
short segments, rank-order origins, the rotating gathered buffers (rounds > NBUF), the replay of
the gathered log on every member, origin-only responses; and for cnr-style partitioned rounds
the count exchange, the send/recv plan, the owners' replay (chunked when one owner receives more
than max_batch Puts) and the answers travelling back.

Oracle: the sequential replay of W_0 || W_1 || ... || W_{G-1} per round, then every member's
reads against the post-round state (SURVEY.md §8a round semantics). Reference:
nr/src/log.rs:494-511 (every replica replays every entry), nr/src/replica.rs:576-578 (responses
to the origin only), cnr/src/replica.rs:430-445 (operations routed to their key's log).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EMPTY = 0xFFFFFFFFFFFFFFFF


def _cuda(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).cuda()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _open(L, lib, G, cfg):
    """a G-member group on device 0 over the loopback collectives"""
    L.check(lib.nrg_test_loopback_collectives(1))
    g = C.c_void_p()
    try:
        L.check(lib.nrg_group_open((C.c_int * G)(*([0] * G)), G, C.byref(cfg), C.byref(g)), "nrg_group_open")
    finally:
        L.check(lib.nrg_test_loopback_collectives(0))
    nr, nl, r0 = C.c_int(), C.c_int(), C.c_int()
    L.check(lib.nrg_group_info(g, C.byref(nr), C.byref(nl), C.byref(r0)))
    assert (nr.value, nl.value, r0.value) == (G, G, 0)
    return g, [lib.nrg_group_replica(g, i) for i in range(G)]


def _sizes(G, r, full):
    """segment lengths of round r: equal (in-place replay), ragged with empty members, all empty,
    one writer, all but the last full (in-place with a short tail)"""
    kind = r % 5
    if kind == 0:
        return [full] * G
    if kind == 1:
        return [0 if i % 3 == 1 else (i * 977 + 311 + 131 * r) % full for i in range(G)]
    if kind == 2:
        return [0] * G
    if kind == 3:
        return [0] * (G - 1) + [full - 7]
    return [full] * (G - 1) + [full // 3]


def _digest(lib, L, ctx):
    out = np.zeros(3, np.uint64)
    L.check(lib.nrg_hashmap_digest(ctx, out.ctypes.data_as(C.c_void_p)))
    return tuple(int(x) for x in out)


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("pipeline,max_batch", [(1, 1 << 16), (0, 1 << 16), (1, 3000)])
def test_group_hashmap_members(nrg, orc, G, pipeline, max_batch):
    """Hashmap group rounds: every member's Gets and (for the members that ask) its own Puts'
    previous values, and every member's final contents, equal to the NR replay. max_batch 3000
    replays the gathered log in chunks; the small ring wraps and is garbage-collected."""
    import torch

    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_HASHMAP)
    cfg.log2_slots, cfg.max_batch, cfg.pipeline = 17, max_batch, pipeline
    cfg.log_bytes = 64 * (1 << 16)
    g, ctxs = _open(L, lib, G, cfg)
    for c in ctxs:
        L.check(lib.nrg_hashmap_prefill_range(c, 4000, 1))
    om = orc.HashMap()
    om.prefill_range(4000, 1)
    span, full, rounds = 20_000, 2500, 7
    outs = []
    for r in range(rounds):
        lens = _sizes(G, r, full)
        rd = (L.Round * G)()
        keep, want = [], []
        for i in range(G):
            W, R = lens[i], 1500 + 100 * i
            k = orc.gen_uniform(W, 1000 * r + i, span)
            if W:
                k[::50] = 7  # one key written by every member: cross-segment order
                k[3::97] = EMPTY  # the side-slot key
            v = orc.gen_raw(W, 1000 * r + i + 500)
            gk = orc.gen_uniform(R, 1000 * r + i + 700, span + 2000)
            puts = np.stack([k, v], 1).astype(np.uint64)
            d = dict(p=_cuda(puts) if W else None, gk=_cuda(gk),
                     gv=torch.full((R,), -1, dtype=torch.int64, device="cuda"),
                     gf=torch.full((R,), 7, dtype=torch.uint8, device="cuda"),
                     pv=torch.full((max(W, 1),), -1, dtype=torch.int64, device="cuda"),
                     pf=torch.full((max(W, 1),), 7, dtype=torch.uint8, device="cuda"))
            w_prev = (i + r) % 2 == 0
            rd[i].recs, rd[i].n = (d["p"].data_ptr() if W else 0), W
            rd[i].resp = d["pv"].data_ptr() if w_prev else 0
            rd[i].some = d["pf"].data_ptr() if w_prev else 0
            rd[i].get_keys, rd[i].n_gets = d["gk"].data_ptr(), R
            rd[i].get_vals, rd[i].get_found = d["gv"].data_ptr(), d["gf"].data_ptr()
            keep.append((d, k, v, gk))
            want.append(w_prev)
        torch.cuda.synchronize()  # inputs exist before the round is issued
        L.check(lib.nrg_group_round_async(g, rd, None), f"group round {r}")
        exp = []
        for i in range(G):
            _, k, v, _ = keep[i]
            exp.append(om.replay(k, v))
        for i in range(G):
            exp[i] = exp[i] + om.get_batch(keep[i][3])
        outs.append((keep, want, exp))
    L.check(lib.nrg_group_sync(g))
    for r, (keep, want, exp) in enumerate(outs):
        for i in range(G):
            d, k, _, _ = keep[i]
            pv, pf, gv, gf = exp[i]
            W = len(k)
            msg = f"G={G} round {r} member {i}"
            np.testing.assert_array_equal(d["gf"].cpu().numpy(), gf, err_msg=msg + " found")
            np.testing.assert_array_equal(_u64(d["gv"]), gv, err_msg=msg + " vals")
            if want[i] and W:
                np.testing.assert_array_equal(d["pf"][:W].cpu().numpy(), pf, err_msg=msg + " prev found")
                np.testing.assert_array_equal(_u64(d["pv"][:W]), pv, err_msg=msg + " prev")
            elif W:  # not asked: untouched
                assert np.all(d["pf"][:W].cpu().numpy() == 7), msg
    total = sum(sum(_sizes(G, r, full)) for r in range(rounds))
    for i, c in enumerate(ctxs):
        assert _digest(lib, L, c) == om.digest(), f"member {i} contents"
        info = L.LogInfo()
        L.check(lib.nrg_log_state(c, C.byref(info)))
        assert info.tail == info.ltail == total and info.replica_id == i + 1
    L.check(lib.nrg_group_close(g))


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("pipeline", [0, 1])
def test_group_stack_members(nrg, orc, G, pipeline):
    """Stack group rounds: each member's Pop responses for its own segment of the gathered log,
    and every member's final stack, equal to the Vec replay of W_0 || ... || W_{G-1}."""
    import torch

    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_STACK)
    cfg.max_batch, cfg.stack_capacity, cfg.pipeline = 1 << 16, 1 << 20, pipeline
    cfg.log_bytes = 64 * (1 << 16)
    g, ctxs = _open(L, lib, G, cfg)
    init = np.arange(700, dtype=np.uint32)
    for c in ctxs:
        L.check(lib.nrg_stack_init(c, init.ctypes.data_as(C.c_void_p), len(init)))
    st = orc.Stack(init)
    outs = []
    for r in range(6):
        lens = _sizes(G, r, 3000)
        rd = (L.Round * G)()
        keep = []
        for i in range(G):
            n = lens[i]
            vals, ops = orc.gen_stack_ops(n, 40 * r + i)
            if n and r % 2:
                ops[: n // 2] = 0  # a Pop run deep into the earlier members' pushes
            recs = np.zeros(n, nrg.STACK_OP_DTYPE)
            recs["val"], recs["op"] = vals, ops
            d_ops = _cuda(recs) if n else None
            resp = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
            some = torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda")
            rd[i].recs, rd[i].n = (d_ops.data_ptr() if n else 0), n
            rd[i].resp, rd[i].some = resp.data_ptr(), some.data_ptr()
            keep.append((d_ops, resp, some, n, st.replay(vals, ops)))
        torch.cuda.synchronize()
        L.check(lib.nrg_group_round_async(g, rd, None), f"stack group round {r}")
        outs.append(keep)
    L.check(lib.nrg_group_sync(g))
    for r, keep in enumerate(outs):
        for i, (_, resp, some, n, (oresp, osome)) in enumerate(keep):
            if n:
                np.testing.assert_array_equal(some[:n].cpu().numpy(), osome, err_msg=f"round {r} member {i} some")
                np.testing.assert_array_equal(resp[:n].cpu().numpy().view(np.uint32), oresp,
                                              err_msg=f"round {r} member {i} pop values")
    want = st.dump()
    for i, c in enumerate(ctxs):
        n = C.c_uint64()
        L.check(lib.nrg_stack_len(c, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.uint32)
        m = C.c_uint64()
        L.check(lib.nrg_stack_dump(c, out.ctypes.data_as(C.c_void_p), n.value, C.byref(m)))
        np.testing.assert_array_equal(out[:m.value], want, err_msg=f"member {i} stack")
    L.check(lib.nrg_group_close(g))


@pytest.mark.parametrize("G", [2, 3, 8])
def test_group_synth_members(nrg, orc, G):
    """Synthetic group rounds (benches/synthetic.rs:112-195), pipelined: each member's sums for
    its own segment and every member's storage equal to the oracle's replay."""
    import torch

    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_SYNTHETIC)
    cfg.max_batch, cfg.pipeline = 1 << 16, 1
    cfg.log_bytes = 64 * (1 << 16)
    g, ctxs = _open(L, lib, G, cfg)
    os_ = orc.Synthetic()
    outs = []
    for r in range(6):
        lens = _sizes(G, r, 2500)
        rd = (L.Round * G)()
        keep = []
        for i in range(G):
            n = lens[i]
            raw = orc.gen_raw(4 * n, 60 * r + i)
            recs = np.zeros(n, nrg.SYNTH_OP_DTYPE)
            recs["tid"], recs["r1"], recs["r2"] = raw[0::4] % 64, raw[1::4], raw[2::4]
            recs["op"] = (raw[3::4] % 100 >= 10).astype(np.uint64)
            d_ops = _cuda(recs) if n else None
            resp = torch.full((max(n, 1),), -1, dtype=torch.int64, device="cuda")
            some = torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda")
            rd[i].recs, rd[i].n = (d_ops.data_ptr() if n else 0), n
            rd[i].resp, rd[i].some = resp.data_ptr(), some.data_ptr()
            ops = np.stack([recs["tid"], recs["r1"], recs["r2"], recs["op"]], axis=1) if n else np.zeros((0, 4),
                                                                                                      np.uint64)
            keep.append((d_ops, resp, some, n, os_.replay(ops)))
        torch.cuda.synchronize()
        L.check(lib.nrg_group_round_async(g, rd, None), f"synthetic group round {r}")
        outs.append(keep)
    L.check(lib.nrg_group_sync(g))
    for r, keep in enumerate(outs):
        for i, (_, resp, some, n, oresp) in enumerate(keep):
            if n:
                np.testing.assert_array_equal(_u64(resp[:n]), oresp, err_msg=f"round {r} member {i}")
                assert np.all(some[:n].cpu().numpy() == 1)
    want = os_.dump()
    for i, c in enumerate(ctxs):
        words = np.zeros(cfg.synth_n, np.uint64)
        m = C.c_uint64()
        L.check(lib.nrg_synth_dump(c, words.ctypes.data_as(C.c_void_p), cfg.synth_n, C.byref(m)))
        np.testing.assert_array_equal(words[:m.value], want, err_msg=f"member {i} storage")
    L.check(lib.nrg_group_close(g))


def _digest_sum(digs):
    tot = [sum(d[0] for d in digs), sum(d[1] for d in digs) % (1 << 64), 0]
    for d in digs:
        tot[2] ^= d[2]
    return tot


@pytest.mark.parametrize("G,skew,pipelined", [(3, False, False), (8, False, False), (3, True, False), (1, False, True),
                                              (1, False, "instream"), (3, False, True), (8, False, True),
                                              (3, True, True)])
def test_group_partitioned_members(nrg, orc, G, skew, pipelined):
    """cnr-style partitioned rounds (nrg_group_partitioned_round) over G partitions: every
    member's Gets and previous values equal the NR replay of the global log, and the partitions'
    digests add up to the NR replica's. skew: every Put of every member belongs to partition 0,
    which then receives G times its max_batch in one round and replays it in chunks. pipelined:
    the rounds go through nrg_group_partitioned_round_async back to back (each call completes the
    round before it) and one flush; checked afterwards, round by round. "instream": the inputs'
    stream set (nrg_group_set_input_stream) and 7 rounds, so round 4 -- empty for the only rank --
    comes between round 3's replay and round 3's answers going back: round 3's reads, which ride
    in the next replay launch, must launch anyway."""
    import torch

    from nrgpu.parallel import key_owner

    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_HASHMAP)
    cfg.log2_slots, cfg.max_batch = 17, 4096
    cfg.pipeline = 1 if pipelined else 0  # pipelined: each round's reads ride in the next round's launch
    g, ctxs = _open(L, lib, G, cfg)
    if pipelined == "instream":
        in_stream = torch.cuda.Stream()
        L.check(lib.nrg_group_set_input_stream(g, 0, C.c_void_p(in_stream.cuda_stream)))
    prefill, span = 6000, 30_000
    for p, c in enumerate(ctxs):
        L.check(lib.nrg_hashmap_prefill_partition(c, prefill, 1, p, G))
    om = orc.HashMap()
    om.prefill_range(prefill, 1)
    pool = orc.gen_uniform(200_000, 99, span)
    owned0 = pool[key_owner(pool, G) == 0]
    posted = []
    for r in range(7 if pipelined == "instream" else 5 if pipelined else 4):
        rd = (L.Round * G)()
        keep = []
        for i in range(G):
            W = 4000 if skew else [0, 1, 2500, 4000][(i + r) % 4]
            R = [3000, 0, 1700][(i + r) % 3]
            if skew:
                k = owned0[(np.arange(W) * 7 + 131 * i + 17 * r) % len(owned0)].copy()
            else:
                k = orc.gen_uniform(W, 300 * r + i, span)
            if W > 10:
                k[::40] = owned0[3]  # one key written by every member
            v = orc.gen_raw(W, 300 * r + i + 100)
            gk = orc.gen_uniform(R, 300 * r + i + 200, span)
            w_prev = (i + r) % 2 == 1 or skew
            d = dict(p=_cuda(np.stack([k, v], 1).astype(np.uint64)) if W else None, gk=_cuda(gk) if R else None,
                     gv=torch.full((max(R, 1),), -1, dtype=torch.int64, device="cuda"),
                     gf=torch.full((max(R, 1),), 7, dtype=torch.uint8, device="cuda"),
                     pv=torch.full((max(W, 1),), -1, dtype=torch.int64, device="cuda"),
                     pf=torch.full((max(W, 1),), 7, dtype=torch.uint8, device="cuda"))
            rd[i].recs, rd[i].n = (d["p"].data_ptr() if W else 0), W
            rd[i].resp = d["pv"].data_ptr() if w_prev else 0
            rd[i].some = d["pf"].data_ptr() if w_prev else 0
            rd[i].get_keys, rd[i].n_gets = (d["gk"].data_ptr() if R else 0), R
            rd[i].get_vals, rd[i].get_found = d["gv"].data_ptr(), d["gf"].data_ptr()
            keep.append((d, k, v, gk, w_prev))
        torch.cuda.synchronize()
        if pipelined:
            L.check(lib.nrg_group_partitioned_round_async(g, rd), f"partitioned round {r} (completes round {r - 1})")
            posted.append((rd, keep))
            continue
        L.check(lib.nrg_group_partitioned_round(g, rd), f"partitioned round {r}")
        L.check(lib.nrg_group_sync(g))
        posted.append((rd, keep))
    if pipelined:
        L.check(lib.nrg_group_partitioned_flush(g), "flush")
        L.check(lib.nrg_group_sync(g))
    for r, (rd, keep) in enumerate(posted):
        exp = [om.replay(k, v) for (_, k, v, _, _) in keep]
        for i, (d, k, v, gk, w_prev) in enumerate(keep):
            msg = f"G={G} round {r} member {i}"
            W, R = len(k), len(gk)
            if w_prev and W:
                np.testing.assert_array_equal(_u64(d["pv"][:W]), exp[i][0], err_msg=msg + " prev")
                np.testing.assert_array_equal(d["pf"][:W].cpu().numpy(), exp[i][1].astype(np.uint8), err_msg=msg)
            if R:
                ev, ef = om.get_batch(gk)
                np.testing.assert_array_equal(_u64(d["gv"][:R]), ev, err_msg=msg + " gets")
                np.testing.assert_array_equal(d["gf"][:R].cpu().numpy(), ef.astype(np.uint8), err_msg=msg)
    assert _digest_sum([list(_digest(lib, L, c)) for c in ctxs]) == [int(x) for x in om.digest()]
    L.check(lib.nrg_group_close(g))


@pytest.mark.parametrize("G", [1, 3])
def test_group_partitioned_pipelined_drops_a_bad_round(nrg, orc, G):
    """Pipelined partitioned rounds (three calls deep) with one bad round in the middle: member 0
    posts Puts without records in round 2. Every member's call that moves round 2 (the call of
    round 3) returns NRG_E_INVAL, the round is dropped everywhere, and rounds 0, 1, 3, 4 answer as
    the NR replay of the log without round 2."""
    import torch

    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_HASHMAP)
    cfg.log2_slots, cfg.max_batch, cfg.pipeline = 17, 4096, 1
    g, ctxs = _open(L, lib, G, cfg)
    for p, c in enumerate(ctxs):
        L.check(lib.nrg_hashmap_prefill_partition(c, 3000, 1, p, G))
    om = orc.HashMap()
    om.prefill_range(3000, 1)
    posted = []
    for r in range(5):
        rd = (L.Round * G)()
        keep = []
        for i in range(G):
            W, R = 700 + 50 * i, 900
            k = orc.gen_uniform(W, 40 * r + i, 12_000)
            v = orc.gen_raw(W, 40 * r + i + 7)
            gk = orc.gen_uniform(R, 40 * r + i + 13, 12_000)
            d = dict(p=_cuda(np.stack([k, v], 1).astype(np.uint64)), gk=_cuda(gk),
                     gv=torch.full((R,), -1, dtype=torch.int64, device="cuda"),
                     gf=torch.full((R,), 7, dtype=torch.uint8, device="cuda"))
            rd[i].recs, rd[i].n = (0 if (r == 2 and i == 0) else d["p"].data_ptr()), W
            rd[i].resp = rd[i].some = 0
            rd[i].get_keys, rd[i].n_gets = d["gk"].data_ptr(), R
            rd[i].get_vals, rd[i].get_found = d["gv"].data_ptr(), d["gf"].data_ptr()
            keep.append((d, k, v, gk))
        torch.cuda.synchronize()
        rc = lib.nrg_group_partitioned_round_async(g, rd)
        assert rc == (L.NRG_E_INVAL if r == 3 else L.NRG_OK), (r, rc)
        posted.append(keep)
    L.check(lib.nrg_group_partitioned_flush(g), "flush")
    L.check(lib.nrg_group_sync(g))
    for r, keep in enumerate(posted):
        if r == 2:
            continue
        for (_, k, v, _) in keep:
            om.replay(k, v)
        for i, (d, k, v, gk) in enumerate(keep):
            ev, ef = om.get_batch(gk)
            np.testing.assert_array_equal(_u64(d["gv"]), ev, err_msg=f"round {r} member {i}")
            np.testing.assert_array_equal(d["gf"].cpu().numpy(), ef.astype(np.uint8))
    assert _digest_sum([list(_digest(lib, L, c)) for c in ctxs]) == [int(x) for x in om.digest()]
    L.check(lib.nrg_group_close(g))


def test_loopback_switch_does_not_leak(nrg):
    """Groups bind their collectives when they are created: with the switch off again, a new
    one-rank group is an RCCL group (it still opens and closes)."""
    L = nrg._lib
    lib = L.load()
    cfg = L.default_config(L.NRG_DS_HASHMAP)
    cfg.log2_slots, cfg.max_batch = 12, 1024
    g, _ = _open(L, lib, 2, cfg)
    g1 = C.c_void_p()
    L.check(lib.nrg_group_open((C.c_int * 1)(0), 1, C.byref(cfg), C.byref(g1)))
    L.check(lib.nrg_group_close(g1))
    L.check(lib.nrg_group_close(g))
