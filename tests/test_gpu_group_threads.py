"""group.cpp's one-member-per-process path (nrg_group_join), the one `bench.py --gpus N` runs,
at nranks = 2, 3 and 8 on the box's one GPU.

Each rank is a thread with its own replica on device 0 that joins the group through
nrgpu.parallel.ReplicaGroup / PartitionedGroup (the classes bench.py uses) over the loopback
collectives of include/nrgpu_testing.h: threads that join the same unique id form one world,
and every all-gather / send / recv is matched across the threads exactly as RCCL matches them
across processes. So each rank drives nrg_group_round_async with ONE local member, as one
process per GPU does: the length exchange when seg_lens is NULL, the per-round header that
checks explicit seg_lens on every rank, and the partitioned round's count exchange between
separate callers.

Oracle: the sequential replay of W_0 || W_1 || ... || W_{G-1} per round, then every rank's reads
against the post-round state (SURVEY.md §8a round semantics). Reference: nr/src/log.rs:343-427
(appends of any length interleave), :494-511 (every replica replays every entry),
nr/src/replica.rs:576-578 (responses to the origin only), cnr/src/replica.rs:430-445.
"""
import ctypes as C
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EMPTY = 0xFFFFFFFFFFFFFFFF


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _cuda(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).cuda()


def _sizes(G, r, full):
    """segment lengths of round r: equal, ragged with empty ranks, all empty, one writer, all but
    the last full"""
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


def _run_ranks(nrg, G, body, timeout=90):
    """Run body(rank, uid) on G threads that form one loopback world; re-raise the first failure."""
    from nrgpu.parallel import ReplicaGroup

    L = nrg._lib
    lib = L.load()
    L.check(lib.nrg_test_loopback_collectives(1))
    errors = [None] * G
    out = [None] * G
    try:
        uid = ReplicaGroup.unique_id()

        def run(rank):
            try:
                out[rank] = body(rank, uid)
            except BaseException as e:  # noqa: BLE001
                errors[rank] = e

        ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(G)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout)
        assert not any(t.is_alive() for t in ts), "a rank is still running (collective never matched)"
    finally:
        L.check(lib.nrg_test_loopback_collectives(0))
    for e in errors:
        if e is not None:
            raise e
    return out


def _hm_rounds(orc, G, rounds, full, span):
    """per round: per rank (keys, vals, get_keys, wants_prev), and the oracle's answers"""
    om = orc.HashMap()
    om.prefill_range(4000, 1)
    plan = []
    for r in range(rounds):
        lens = _sizes(G, r, full)
        parts = []
        for i in range(G):
            W, R = lens[i], 900 + 100 * i
            k = orc.gen_uniform(W, 1000 * r + i, span)
            if W:
                k[::50] = 7  # one key written by every rank: cross-segment order
                k[3::97] = EMPTY  # the side-slot key
            v = orc.gen_raw(W, 1000 * r + i + 500)
            gk = orc.gen_uniform(R, 1000 * r + i + 700, span + 2000)
            parts.append((k, v, gk, (i + r) % 2 == 0))
        exp = [om.replay(k, v) for (k, v, _, _) in parts]
        exp = [exp[i] + om.get_batch(parts[i][2]) for i in range(G)]
        plan.append((lens, parts, exp))
    return plan, om.digest()


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("explicit", [False, True])
def test_join_hashmap_rounds(nrg, orc, G, explicit):
    """Hashmap rounds with ragged and empty segments, one rank per thread. explicit=False passes
    seg_lens = NULL (the lengths are exchanged); True passes the same seg_lens on every rank (the
    header check). Every rank's Gets and (for the ranks that ask) its own Puts' previous values,
    every replica's contents and log state equal the NR replay."""
    import torch

    from nrgpu import DeviceReplica
    from nrgpu.parallel import ReplicaGroup

    L = nrg._lib
    rounds, full, span = 7, 2500, 20_000
    plan, want_digest = _hm_rounds(orc, G, rounds, full, span)
    total = sum(sum(p[0]) for p in plan)

    def body(rank, uid):
        rep = DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=17, max_batch=1 << 16, pipeline=1,
                            log_bytes=64 * (1 << 16), replica_id=rank + 1)
        rep.hm_prefill_range(4000, 1)
        grp = ReplicaGroup(rep, rank, G, uid=uid)
        keep = []
        for lens, parts, _ in plan:
            k, v, gk, w_prev = parts[rank]
            W, R = len(k), len(gk)
            d = dict(p=_cuda(np.stack([k, v], 1).astype(np.uint64)) if W else None, gk=_cuda(gk),
                     gv=torch.full((R,), -1, dtype=torch.int64, device="cuda"),
                     gf=torch.full((R,), 7, dtype=torch.uint8, device="cuda"),
                     pv=torch.full((max(W, 1),), -1, dtype=torch.int64, device="cuda"),
                     pf=torch.full((max(W, 1),), 7, dtype=torch.uint8, device="cuda"))
            torch.cuda.synchronize()  # inputs exist before the round is issued
            grp.round_async(d["p"], W, d["pv"] if w_prev else None, d["pf"] if w_prev else None, d["gk"], R,
                            d["gv"], d["gf"], seg_lens=lens if explicit else None)
            keep.append(d)
        grp.sync()
        res = [(_u64(d["gv"]), d["gf"].cpu().numpy(), _u64(d["pv"]), d["pf"].cpu().numpy()) for d in keep]
        st = rep.log_state()
        dig = rep.hm_digest()
        grp.close()
        rep.close()
        return res, st, dig

    out = _run_ranks(nrg, G, body)
    for rank in range(G):
        res, st, dig = out[rank]
        assert dig == want_digest, f"rank {rank} contents"
        assert st["tail"] == st["ltail"] == total and st["replica_id"] == rank + 1
        for r, (lens, parts, exp) in enumerate(plan):
            gv, gf, pv, pf = res[r]
            k, _, _, w_prev = parts[rank]
            epv, epf, egv, egf = exp[rank]
            msg = f"G={G} round {r} rank {rank}"
            np.testing.assert_array_equal(gf, egf, err_msg=msg + " found")
            np.testing.assert_array_equal(gv, egv, err_msg=msg + " vals")
            W = len(k)
            if w_prev and W:
                np.testing.assert_array_equal(pf[:W], epf, err_msg=msg + " prev found")
                np.testing.assert_array_equal(pv[:W], epv, err_msg=msg + " prev")
            elif W:
                assert np.all(pf[:W] == 7), msg + " untouched"


@pytest.mark.parametrize("G", [2, 3, 8])
def test_join_stack_rounds(nrg, orc, G):
    """Stack rounds (pipelined), ragged segments with seg_lens = NULL: each rank's Pop responses for
    its own segment and every rank's final stack equal the Vec replay of W_0 || ... || W_{G-1}."""
    import torch

    from nrgpu import DeviceReplica
    from nrgpu.parallel import ReplicaGroup

    L = nrg._lib
    init = np.arange(700, dtype=np.uint32)
    st = orc.Stack(init)
    plan = []
    for r in range(6):
        lens = _sizes(G, r, 3000)
        parts = []
        for i in range(G):
            vals, ops = orc.gen_stack_ops(lens[i], 40 * r + i)
            if lens[i] and r % 2:
                ops[: lens[i] // 2] = 0  # a Pop run deep into the earlier ranks' pushes
            parts.append((vals, ops))
        plan.append([(v, o, st.replay(v, o)) for v, o in parts])
    want = st.dump()

    def body(rank, uid):
        rep = DeviceReplica(L.NRG_DS_STACK, 0, max_batch=1 << 16, stack_capacity=1 << 20, pipeline=1,
                            log_bytes=64 * (1 << 16), replica_id=rank + 1)
        rep.st_init(init)
        grp = ReplicaGroup(rep, rank, G, uid=uid)
        keep = []
        for parts in plan:
            vals, ops, _ = parts[rank]
            n = len(ops)
            recs = np.zeros(n, nrg.STACK_OP_DTYPE)
            recs["val"], recs["op"] = vals, ops
            d_ops = _cuda(recs) if n else None
            resp = torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
            some = torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            grp.round_async(d_ops, n, resp, some)
            keep.append((d_ops, resp, some, n))
        grp.sync()
        res = [(resp[:n].cpu().numpy().view(np.uint32), some[:n].cpu().numpy()) for (_, resp, some, n) in keep]
        final = rep.st_dump()
        grp.close()
        rep.close()
        return res, final

    out = _run_ranks(nrg, G, body)
    for rank in range(G):
        res, final = out[rank]
        np.testing.assert_array_equal(final, want, err_msg=f"rank {rank} stack")
        for r, parts in enumerate(plan):
            _, _, (oresp, osome) = parts[rank]
            np.testing.assert_array_equal(res[r][1], osome, err_msg=f"round {r} rank {rank} some")
            np.testing.assert_array_equal(res[r][0], oresp, err_msg=f"round {r} rank {rank} pop values")


@pytest.mark.parametrize("G", [2, 3, 8])
def test_join_synth_rounds(nrg, orc, G):
    """Synthetic rounds (benches/synthetic.rs:112-195), pipelined, ragged segments with
    seg_lens = NULL: each rank's sums for its own segment and every rank's storage equal the
    oracle's replay."""
    import torch

    from nrgpu import DeviceReplica
    from nrgpu.parallel import ReplicaGroup

    L = nrg._lib
    os_ = orc.Synthetic()
    plan = []
    for r in range(6):
        lens = _sizes(G, r, 2500)
        parts = []
        for i in range(G):
            n = lens[i]
            raw = orc.gen_raw(4 * n, 60 * r + i)
            recs = np.zeros(n, nrg.SYNTH_OP_DTYPE)
            recs["tid"], recs["r1"], recs["r2"] = raw[0::4] % 64, raw[1::4], raw[2::4]
            recs["op"] = (raw[3::4] % 100 >= 10).astype(np.uint64)
            ops = np.stack([recs["tid"], recs["r1"], recs["r2"], recs["op"]], axis=1) if n else np.zeros((0, 4),
                                                                                                      np.uint64)
            parts.append((recs, os_.replay(ops)))
        plan.append(parts)
    want = os_.dump()

    def body(rank, uid):
        rep = DeviceReplica(L.NRG_DS_SYNTHETIC, 0, max_batch=1 << 16, pipeline=1, log_bytes=64 * (1 << 16),
                            replica_id=rank + 1)
        grp = ReplicaGroup(rep, rank, G, uid=uid)
        keep = []
        for parts in plan:
            recs, _ = parts[rank]
            n = len(recs)
            d_ops = _cuda(recs) if n else None
            resp = torch.full((max(n, 1),), -1, dtype=torch.int64, device="cuda")
            some = torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            grp.round_async(d_ops, n, resp, some)
            keep.append((d_ops, resp, some, n))
        grp.sync()
        res = [(_u64(resp[:n]), some[:n].cpu().numpy()) for (_, resp, some, n) in keep]
        words = rep.sy_dump()
        grp.close()
        rep.close()
        return res, words

    out = _run_ranks(nrg, G, body)
    for rank in range(G):
        res, words = out[rank]
        np.testing.assert_array_equal(words, want, err_msg=f"rank {rank} storage")
        for r, parts in enumerate(plan):
            np.testing.assert_array_equal(res[r][0], parts[rank][1], err_msg=f"round {r} rank {rank}")
            assert np.all(res[r][1] == 1)


def _digest_sum(digs):
    tot = [sum(d[0] for d in digs), sum(d[1] for d in digs) % (1 << 64), 0]
    for d in digs:
        tot[2] ^= d[2]
    return tot


@pytest.mark.parametrize("G,skew,pipelined", [(2, False, False), (3, False, False), (8, False, False),
                                              (3, True, False), (3, False, True), (8, True, True)])
def test_join_partitioned_rounds(nrg, orc, G, skew, pipelined):
    """cnr-style partitioned rounds through PartitionedGroup, one rank per thread: the count
    exchange, the send/recv plan and the answers back between separate callers. Every rank's
    Gets and previous values equal the NR replay; the partitions' digests add up to the NR
    replica's. skew: every Put belongs to partition 0 (replayed there in max_batch chunks).
    pipelined: round_async back to back, one flush, answers read afterwards."""
    import torch

    from nrgpu import DeviceReplica
    from nrgpu.parallel import PartitionedGroup, key_owner

    L = nrg._lib
    prefill, span = 6000, 30_000
    om = orc.HashMap()
    om.prefill_range(prefill, 1)
    pool = orc.gen_uniform(200_000, 99, span)
    owned0 = pool[key_owner(pool, G) == 0]
    plan = []
    for r in range(4):
        parts = []
        for i in range(G):
            W = 4000 if skew else [0, 1, 2500, 4000][(i + r) % 4]
            R = [3000, 0, 1700][(i + r) % 3]
            if skew:
                k = owned0[(np.arange(W) * 7 + 131 * i + 17 * r) % len(owned0)].copy()
            else:
                k = orc.gen_uniform(W, 300 * r + i, span)
            if W > 10:
                k[::40] = owned0[3]  # one key written by every rank
            v = orc.gen_raw(W, 300 * r + i + 100)
            gk = orc.gen_uniform(R, 300 * r + i + 200, span)
            parts.append((k, v, gk, (i + r) % 2 == 1 or skew))
        exp = [om.replay(k, v) for (k, v, _, _) in parts]
        gets = [om.get_batch(p[2]) for p in parts]
        plan.append((parts, exp, gets))
    want = [int(x) for x in om.digest()]

    def body(rank, uid):
        rep = DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=17, max_batch=4096, replica_id=rank + 1)
        rep.hm_prefill_partition(prefill, 1, rank, G)
        grp = PartitionedGroup(rep, rank, G, uid=uid)
        res, bufs = [], []
        for parts, _, _ in plan:
            k, v, gk, w_prev = parts[rank]
            W, R = len(k), len(gk)
            p = _cuda(np.stack([k, v], 1).astype(np.uint64)) if W else None
            g = _cuda(gk) if R else None
            gv = torch.full((max(R, 1),), -1, dtype=torch.int64, device="cuda")
            gf = torch.full((max(R, 1),), 7, dtype=torch.uint8, device="cuda")
            pv = torch.full((max(W, 1),), -1, dtype=torch.int64, device="cuda")
            pf = torch.full((max(W, 1),), 7, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            if pipelined:
                grp.round_async(p, W, g, R, gv, gf, pv if w_prev else None, pf if w_prev else None)
                bufs.append((p, g, gv, gf, pv, pf, R, W))
                continue
            grp.round(p, W, g, R, gv, gf, pv if w_prev else None, pf if w_prev else None)
            grp.sync()
            res.append((_u64(gv[:R]), gf[:R].cpu().numpy(), _u64(pv[:W]), pf[:W].cpu().numpy()))
        if pipelined:
            grp.flush()
            grp.sync()
            res = [(_u64(gv[:R]), gf[:R].cpu().numpy(), _u64(pv[:W]), pf[:W].cpu().numpy())
                   for (_, _, gv, gf, pv, pf, R, W) in bufs]
        dig = rep.hm_digest()
        grp.close()
        rep.close()
        return res, dig

    out = _run_ranks(nrg, G, body)
    assert _digest_sum([list(o[1]) for o in out]) == want
    for rank in range(G):
        for r, (parts, exp, gets) in enumerate(plan):
            gv, gf, pv, pf = out[rank][0][r]
            k, _, gk, w_prev = parts[rank]
            msg = f"G={G} round {r} rank {rank}"
            if w_prev and len(k):
                np.testing.assert_array_equal(pv, exp[rank][0], err_msg=msg + " prev")
                np.testing.assert_array_equal(pf, exp[rank][1].astype(np.uint8), err_msg=msg + " prev found")
            if len(gk):
                np.testing.assert_array_equal(gv, gets[rank][0], err_msg=msg + " gets")
                np.testing.assert_array_equal(gf, gets[rank][1].astype(np.uint8), err_msg=msg + " found")


@pytest.mark.parametrize("case", ["null_bad_rank", "explicit_wrong_n", "explicit_disagree"])
def test_join_mismatched_lengths_refused_everywhere(nrg, case):
    """A round the ranks disagree on fails with NRG_E_INVAL on EVERY rank, and no rank is left
    inside a collective:
      null_bad_rank      seg_lens = NULL, one rank's segment is invalid (n > 0, no records): the
                         length exchange carries its error to all ranks;
      explicit_wrong_n   one rank's n differs from the seg_lens every rank passes: that rank
                         still takes part (zeros) and returns NRG_E_INVAL; the header check makes
                         the others' sync return it;
      explicit_disagree  two ranks pass different seg_lens with the same longest segment: every
                         rank's header check catches it at sync."""
    import torch

    from nrgpu import DeviceReplica, NrgError
    from nrgpu.parallel import ReplicaGroup

    L = nrg._lib
    G = 3

    def body(rank, uid):
        rep = DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=14, max_batch=4096, replica_id=rank + 1)
        grp = ReplicaGroup(rep, rank, G, uid=uid)
        W = [100, 60, 80][rank]
        puts = torch.zeros((W, 2), dtype=torch.int64, device="cuda")
        puts[:, 0] = torch.arange(W, device="cuda") + 1000 * rank
        lens = [100, 60, 80]
        seg, n, recs = None, W, puts
        if case == "null_bad_rank" and rank == 1:
            recs = None
        elif case == "explicit_wrong_n":
            seg = lens
            if rank == 2:
                n = 70
        elif case == "explicit_disagree":
            seg = lens if rank != 0 else [100, 61, 79]
        torch.cuda.synchronize()
        codes = []
        try:
            grp.round_async(recs, n, seg_lens=seg)
            codes.append(0)
        except NrgError as e:
            codes.append(e.code)
        try:
            grp.sync()
            codes.append(0)
        except NrgError as e:
            codes.append(e.code)
        grp.close()
        rep.close()
        return codes

    out = _run_ranks(nrg, G, body)
    inval = L.NRG_E_INVAL
    for rank, (c_round, c_sync) in enumerate(out):
        assert inval in (c_round, c_sync), f"rank {rank}: round {c_round}, sync {c_sync}"
        assert c_round in (0, inval) and c_sync in (0, inval), (rank, c_round, c_sync)


def test_join_rounds_with_reads_only(nrg, orc):
    """Rounds in which no rank writes (every length 0, exchanged and explicit) still answer each
    rank's Gets; a later writing round lines up (the all-gather sequence is not disturbed)."""
    import torch

    from nrgpu import DeviceReplica
    from nrgpu.parallel import ReplicaGroup

    L = nrg._lib
    G = 3
    om = orc.HashMap()
    om.prefill_range(500, 1)
    gk = orc.gen_uniform(300, 5, 1000)
    k = orc.gen_uniform(200, 6, 1000)
    v = orc.gen_raw(200, 7)
    ev0 = om.get_batch(gk)
    for i in range(G):
        om.replay(k + i, v)
    ev1 = om.get_batch(gk)

    def body(rank, uid):
        rep = DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=14, max_batch=4096, replica_id=rank + 1)
        rep.hm_prefill_range(500, 1)
        grp = ReplicaGroup(rep, rank, G, uid=uid)
        d_gk = _cuda(gk)
        res = []
        for r, (W, seg) in enumerate([(0, None), (0, [0] * G), (200, None), (200, [200] * G)]):
            gv = torch.zeros(300, dtype=torch.int64, device="cuda")
            gf = torch.zeros(300, dtype=torch.uint8, device="cuda")
            p = _cuda(np.stack([k + rank, v], 1).astype(np.uint64)) if W else None
            torch.cuda.synchronize()
            grp.round_async(p, W, None, None, d_gk, 300, gv, gf, seg_lens=seg)
            grp.sync()
            res.append((_u64(gv), gf.cpu().numpy()))
        grp.close()
        rep.close()
        return res

    out = _run_ranks(nrg, G, body)
    for rank in range(G):
        for r in range(2):
            np.testing.assert_array_equal(out[rank][r][0], ev0[0])
            np.testing.assert_array_equal(out[rank][r][1], ev0[1].astype(np.uint8))
        np.testing.assert_array_equal(out[rank][2][0], ev1[0])
        # round 3 replays the same Puts again: contents unchanged, same answers
        np.testing.assert_array_equal(out[rank][3][0], ev1[0])


@pytest.mark.parametrize("case", ["exchanged", "explicit", "partitioned"])
def test_join_missing_rank_times_out(nrg, case):
    """A rank that never posts its part of a round must not hang its peers:
    with a 2-s group deadline (nrg_group_set_timeout) every other rank's round fails with
    NRG_E_TIMEOUT within the deadline, the message names the rank and the round, and the failure
    is sticky (a later sync reports it too; the group can still be closed). One full round runs
    first, so the missing rank is absent from round 1, not from the group's formation."""
    import time

    import torch

    from nrgpu import DeviceReplica, NrgError
    from nrgpu.parallel import PartitionedGroup, ReplicaGroup

    L = nrg._lib
    G, W, R, deadline_ms = 3, 500, 300, 2000
    missing = G - 1

    def body(rank, uid):
        rep = DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=14, max_batch=4096, replica_id=rank + 1)
        cls = PartitionedGroup if case == "partitioned" else ReplicaGroup
        grp = cls(rep, rank, G, uid=uid, timeout_ms=deadline_ms)
        puts = torch.zeros((W, 2), dtype=torch.int64, device="cuda")
        puts[:, 0] = torch.arange(W, device="cuda") + 1000 * rank
        gk = torch.arange(R, dtype=torch.int64, device="cuda")
        gv = torch.zeros(R, dtype=torch.int64, device="cuda")
        gf = torch.zeros(R, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()

        def one_round():
            if case == "partitioned":
                grp.round(puts, W, gk, R, gv, gf)
            else:
                grp.round_async(puts, W, None, None, gk, R, gv, gf,
                                seg_lens=[W] * G if case == "explicit" else None)
            grp.sync()

        one_round()  # everyone
        out = {"rank": rank}
        if rank != missing:
            t0 = time.monotonic()
            try:
                one_round()
                out["round"] = 0
            except NrgError as e:
                out["round"], out["msg"] = e.code, str(e)
            out["elapsed"] = time.monotonic() - t0
            try:
                grp.sync()
                out["again"] = 0
            except NrgError as e:
                out["again"] = e.code
            out["diag"] = grp.last_error()
        else:
            time.sleep(deadline_ms / 1000 + 3)  # keep the world alive, post nothing
        grp.close()
        rep.close()
        return out

    out = _run_ranks(nrg, G, body, timeout=60)
    for o in out:
        if o["rank"] == missing:
            continue
        r = o["rank"]
        assert o["round"] == L.NRG_E_TIMEOUT, o
        assert o["elapsed"] < deadline_ms / 1000 + 3.0, o
        assert o["again"] == L.NRG_E_TIMEOUT, o  # sticky
        assert f"rank {r} of {G}, round 1" in o["diag"], o
        assert "within 2000 ms" in o["diag"], o
