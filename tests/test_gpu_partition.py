"""cnr-style key-partitioned NrHashMap on the GPU.

cnr maps each operation to one of several logs with LogMapper::hash (cnr/src/lib.rs:134-167,
cnr/src/replica.rs:430-445) and each log replays on its own (:673-736). Across GPUs partition p's
log lives on GPU p, which holds only its keys: Puts and Gets travel to their owners, each owner
replays what it received in rank order and answers, and the answers come back. Checked here:
  * the device partition (nrg_hashmap_partition_async) is the stable partition by nrg_key_owner
    that a numpy argsort gives, and nrg_route_back_async inverts it;
  * partition prefills add up to NrHashMap::default;
  * rounds over 3 partitions held by 3 replicas on this GPU (routing done with the device
    partition kernel) answer exactly what the NR replay of the global log answers, and the
    partitions' digests add up to the NR replica's;
  * the C-ABI round (nrg_group_partitioned_round: RCCL send/recv) with one rank.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cuda(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).cuda()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _puts(keys, vals):
    return np.stack([keys, vals], 1).astype(np.uint64)


@pytest.mark.parametrize("W,R,parts", [(0, 0, 3), (1, 5, 2), (2047, 2049, 3), (100_000, 70_000, 8), (5000, 4000, 64),
                                       (3000, 3000, 1)])
def test_partition_kernel(nrg, orc, W, R, parts):
    import torch

    from nrgpu.parallel import key_owner

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=12, max_batch=1 << 10)
    dev.use_torch_stream()
    keys = orc.gen_raw(W, 11 + W)
    keys[::17] = 5  # repeated keys keep their issue order
    vals = orc.gen_raw(W, 12 + W)
    gk = orc.gen_raw(R, 13 + R)
    puts = _puts(keys, vals)
    d_puts, d_gk = _cuda(puts), _cuda(gk)
    p_out = torch.full((max(W, 1), 2), -1, dtype=torch.int64, device="cuda")
    p_pos = torch.full((max(W, 1),), -1, dtype=torch.int32, device="cuda")
    k_out = torch.full((max(R, 1),), -1, dtype=torch.int64, device="cuda")
    k_pos = torch.full((max(R, 1),), -1, dtype=torch.int32, device="cuda")
    counts = torch.full((2 * parts,), -1, dtype=torch.int64, device="cuda")
    dev.hm_partition_device(d_puts, W, d_gk, R, parts, p_out, p_pos, k_out, k_pos, counts)
    torch.cuda.synchronize()
    po = np.argsort(key_owner(keys, parts), kind="stable")
    ko = np.argsort(key_owner(gk, parts), kind="stable")
    np.testing.assert_array_equal(counts.cpu().numpy()[:parts], np.bincount(key_owner(keys, parts), minlength=parts))
    np.testing.assert_array_equal(counts.cpu().numpy()[parts:], np.bincount(key_owner(gk, parts), minlength=parts))
    if W:
        np.testing.assert_array_equal(_u64(p_out[:W]), puts[po])
        np.testing.assert_array_equal(p_pos[:W].cpu().numpy()[po], np.arange(W))
        # answers in partitioned order come back in issue order
        back = torch.empty(W, dtype=torch.int64, device="cuda")
        back8 = torch.empty(W, dtype=torch.uint8, device="cuda")
        src8 = (p_out[:W, 1] & 0xFF).to(torch.uint8).contiguous()
        dev.route_back_device(p_out[:W, 1].contiguous(), src8, p_pos, W, back, back8)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_u64(back), vals)
        np.testing.assert_array_equal(back8.cpu().numpy(), (vals & np.uint64(0xFF)).astype(np.uint8))
    if R:
        np.testing.assert_array_equal(_u64(k_out[:R]), gk[ko])
        np.testing.assert_array_equal(k_pos[:R].cpu().numpy()[ko], np.arange(R))
    dev.close()


def _digest_sum(digs):
    tot = [sum(d[0] for d in digs), sum(d[1] for d in digs) % (1 << 64), 0]
    for d in digs:
        tot[2] ^= d[2]
    return tot


def test_prefill_partition_digests_add_up(nrg, orc):
    n, parts = 50_000, 3
    reps = [nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=1 << 10) for _ in range(parts)]
    for p, r in enumerate(reps):
        r.hm_prefill_partition(n, 1, p, parts)
    om = orc.HashMap()
    om.prefill_range(n, 1)
    assert sum(r.hm_size() for r in reps) == n
    assert _digest_sum([[int(x) for x in r.hm_digest()] for r in reps]) == [int(x) for x in om.digest()]
    with pytest.raises(nrg.NrgError):
        reps[0].hm_prefill_partition(n, 1, 3, 3)
    for r in reps:
        r.close()


def test_partitioned_rounds_three_partitions_one_gpu(nrg, orc):
    """Three ranks' rounds over three partitions held by three replicas on this GPU; each rank's
    Puts and Gets are partitioned by the device kernel and routed by owner in Python (the
    exchange RCCL does across GPUs), owners replay in rank order."""
    import torch

    G, span, prefill = 3, 40_000, 10_000
    reps = [nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=1 << 16, replica_id=p + 1)
            for p in range(G)]
    for p, r in enumerate(reps):
        r.use_torch_stream()
        r.hm_prefill_partition(prefill, 1, p, G)
    om = orc.HashMap()
    om.prefill_range(prefill, 1)
    for rnd in range(4):
        segs, parts_of = [], []
        for rank in range(G):
            W, R = 6000 + 1000 * rank, 5000 + 700 * rank
            k = orc.gen_uniform(W, 100 * rnd + rank, span)
            k[::50] = 7  # a hot key written by every rank
            v = orc.gen_raw(W, 100 * rnd + rank + 10)
            gk = orc.gen_uniform(R, 100 * rnd + rank + 20, span)
            d_p, d_k = _cuda(_puts(k, v)), _cuda(gk)
            po = torch.empty((W, 2), dtype=torch.int64, device="cuda")
            pp = torch.empty(W, dtype=torch.int32, device="cuda")
            ko = torch.empty(R, dtype=torch.int64, device="cuda")
            kp = torch.empty(R, dtype=torch.int32, device="cuda")
            cnt = torch.empty(2 * G, dtype=torch.int64, device="cuda")
            reps[rank].hm_partition_device(d_p, W, d_k, R, G, po, pp, ko, kp, cnt)
            torch.cuda.synchronize()
            c = cnt.cpu().tolist()
            segs.append((k, v, gk))
            parts_of.append((po, pp, ko, kp, c))
        # owners: the Puts they received in rank order, then their Gets
        ans = {}
        for o in range(G):
            pin, kin, src = [], [], []
            for rank in range(G):
                po, _, ko, _, c = parts_of[rank]
                p0, k0 = sum(c[:o]), sum(c[G:G + o])
                pin.append(po[p0:p0 + c[o]])
                kin.append(ko[k0:k0 + c[G + o]])
                src.append((c[o], c[G + o]))
            vals, found, pv, pf = reps[o].partitioned_replay(torch.cat(pin), torch.cat(kin), True)
            ans[o] = (vals, found, pv, pf, src)
        for rank in range(G):
            po, pp, ko, kp, c = parts_of[rank]
            W, R = po.shape[0], ko.shape[0]
            # this rank's answers in partitioned order: owner o's slice for it
            gv, gf, pvv, pff = [], [], [], []
            for o in range(G):
                vals, found, pv, pf, src = ans[o]
                p0 = sum(s[0] for s in src[:rank])
                k0 = sum(s[1] for s in src[:rank])
                gv.append(vals[k0:k0 + src[rank][1]])
                gf.append(found[k0:k0 + src[rank][1]])
                pvv.append(pv[p0:p0 + src[rank][0]])
                pff.append(pf[p0:p0 + src[rank][0]])
            out_v = torch.empty(R, dtype=torch.int64, device="cuda")
            out_f = torch.empty(R, dtype=torch.uint8, device="cuda")
            reps[rank].route_back_device(torch.cat(gv), torch.cat(gf), kp, R, out_v, out_f)
            prev_v = torch.empty(W, dtype=torch.int64, device="cuda")
            prev_f = torch.empty(W, dtype=torch.uint8, device="cuda")
            reps[rank].route_back_device(torch.cat(pvv), torch.cat(pff), pp, W, prev_v, prev_f)
            torch.cuda.synchronize()
            parts_of[rank] = (out_v, out_f, prev_v, prev_f)
        # the NR replay of the global log W_0 || W_1 || W_2, then every rank's reads
        for rank in range(G):
            k, v, _ = segs[rank]
            p, f = om.replay(k, v)
            np.testing.assert_array_equal(_u64(parts_of[rank][2]), p, err_msg=f"round {rnd} rank {rank} prev")
            np.testing.assert_array_equal(parts_of[rank][3].cpu().numpy(), f.astype(np.uint8))
        for rank in range(G):
            ev, ef = om.get_batch(segs[rank][2])
            np.testing.assert_array_equal(_u64(parts_of[rank][0]), ev, err_msg=f"round {rnd} rank {rank} gets")
            np.testing.assert_array_equal(parts_of[rank][1].cpu().numpy(), ef.astype(np.uint8))
    assert _digest_sum([[int(x) for x in r.hm_digest()] for r in reps]) == [int(x) for x in om.digest()]
    for r in reps:
        r.close()


@pytest.mark.parametrize("move", [0, 1])
def test_partitioned_group_round_one_rank(nrg, orc, move):
    """nrg_group_partitioned_round through RCCL with one rank: answers and previous values against
    the NR replay. A one-rank group owns every key, so by default its partition and route-back are
    the identity (the replay reads the caller's records and answers into the caller's buffers);
    move = 1 (NRG_KNOB_EXP bit 16) moves the data as a multi-rank group does (partition copy on the
    side stream, route-back launch)."""
    import torch

    from nrgpu.parallel import PartitionedGroup

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs={"EXP": 0x10000 * move}, log2_slots=17,
                            max_batch=1 << 16, replica_id=1)
    dev.use_torch_stream()
    dev.hm_prefill_partition(20_000, 1, 0, 1)
    om = orc.HashMap()
    om.prefill_range(20_000, 1)
    g = PartitionedGroup(dev, rank=0, world=1)
    for rnd in range(3):
        W, R = 30_000 + 1000 * rnd, 50_000
        k = orc.gen_uniform(W, 700 + rnd, 60_000)
        v = orc.gen_raw(W, 710 + rnd)
        gk = orc.gen_uniform(R, 720 + rnd, 60_000)
        d_p, d_k = _cuda(_puts(k, v)), _cuda(gk)
        gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        want = rnd != 1
        pv = torch.full((W,), -1, dtype=torch.int64, device="cuda") if want else None
        pf = torch.full((W,), 7, dtype=torch.uint8, device="cuda") if want else None
        g.round(d_p, W, d_k, R, gv, gf, pv, pf)
        g.sync()
        p, f = om.replay(k, v)
        if want:
            np.testing.assert_array_equal(_u64(pv), p)
            np.testing.assert_array_equal(pf.cpu().numpy(), f.astype(np.uint8))
        ev, ef = om.get_batch(gk)
        np.testing.assert_array_equal(_u64(gv), ev)
        np.testing.assert_array_equal(gf.cpu().numpy(), ef.astype(np.uint8))
    assert [int(x) for x in dev.hm_digest()] == [int(x) for x in om.digest()]
    g.close()
    dev.close()


@pytest.mark.parametrize("move", [0, 1])
def test_partitioned_group_one_rank_pipelined(nrg, orc, move):
    """One rank, rounds pipelined three calls deep (round_async: call e partitions round e, replays
    e-1, answers e-2), the caller's buffers distinct per round, then flush: every answer and
    previous value against the NR replay, in both the identity and the data-moving form."""
    import torch

    from nrgpu.parallel import PartitionedGroup

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs={"EXP": 0x10000 * move}, log2_slots=17,
                            max_batch=1 << 16, replica_id=1)
    dev.use_torch_stream()
    dev.hm_prefill_partition(20_000, 1, 0, 1)
    om = orc.HashMap()
    om.prefill_range(20_000, 1)
    g = PartitionedGroup(dev, rank=0, world=1)
    keep, exp = [], []
    for rnd in range(6):
        W, R = 20_000 + 500 * rnd, 40_000 - 1000 * rnd
        k = orc.gen_uniform(W, 800 + rnd, 60_000)
        v = orc.gen_raw(W, 810 + rnd)
        gk = orc.gen_uniform(R, 820 + rnd, 60_000)
        d_p, d_k = _cuda(_puts(k, v)), _cuda(gk)
        gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        want = rnd % 2 == 0
        pv = torch.full((W,), -1, dtype=torch.int64, device="cuda") if want else None
        pf = torch.full((W,), 7, dtype=torch.uint8, device="cuda") if want else None
        g.round_async(d_p, W, d_k, R, gv, gf, pv, pf)
        keep.append((d_p, d_k, gv, gf, pv, pf))
        p, f = om.replay(k, v)
        exp.append((om.get_batch(gk), (p, f) if want else None))
    g.flush()
    torch.cuda.synchronize()
    for rnd, ((_, _, gv, gf, pv, pf), ((ev, ef), pp)) in enumerate(zip(keep, exp)):
        np.testing.assert_array_equal(_u64(gv), ev, err_msg=f"round {rnd}")
        np.testing.assert_array_equal(gf.cpu().numpy(), ef.astype(np.uint8), err_msg=f"round {rnd}")
        if pp is not None:
            np.testing.assert_array_equal(_u64(pv), pp[0], err_msg=f"round {rnd} prev")
            np.testing.assert_array_equal(pf.cpu().numpy(), pp[1].astype(np.uint8), err_msg=f"round {rnd} prev")
    assert [int(x) for x in dev.hm_digest()] == [int(x) for x in om.digest()]
    g.close()
    dev.close()
