"""NrHashMap parity: the HIP replay (through the C ABI) vs the sequential CPU oracle.

Semantics under test (SURVEY.md §8a "Round semantics"): the writes of a round are replayed
in global log order (Put -> HashMap::insert, response = previous value,
nr/examples/hashmap.rs:46-50), then the round's reads are answered against the post-round
state (dispatch after sync-to-tail, nr/src/replica.rs:483-497). Bit-exact comparison of every
response and of the final replica contents.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EMPTY = 0xFFFFFFFFFFFFFFFF


def _puts(keys, vals):
    import nrgpu

    r = np.zeros(len(keys), nrgpu.PUT_DTYPE)
    r["key"] = keys
    r["val"] = vals
    return r


def _check_state(dev, om):
    gk, gv = dev.hm_dump()
    ok, ov = om.dump_sorted()
    assert len(gk) == len(ok) == len(om)
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv, ov)
    assert dev.hm_size() == len(om)
    assert dev.hm_digest() == om.digest()


# knobs of the replay paths: default selection, partition rounds for every round, and the
# one-launch small rounds (the combiner's) for rounds of up to 2048 Puts
PATHS = {"default": {}, "part": {"PART": 2}, "wide": {"PART": 2, "PA_TPB": 1024}, "w512": {"PART": 2, "PA_TPB": 512},
         "small": {"SMALL_MAX": 2048}}


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("span,W,R,rounds", [(64, 300, 500, 6), (5000, 2000, 3000, 5), (1 << 40, 4000, 4000, 3)])
def test_rounds_prev_and_gets(nrg, orc, span, W, R, rounds, path):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=PATHS[path], log2_slots=16, max_batch=8192)
    om = orc.HashMap()
    dev.hm_prefill_range(min(span, 1000), 1)
    om.prefill_range(min(span, 1000), 1)
    for r in range(rounds):
        keys = orc.gen_uniform(W, 1000 + r, span)
        vals = orc.gen_raw(W, 2000 + r)
        if r % 2 == 1:
            keys[::97] = EMPTY  # the side-slot key
        gkeys = orc.gen_uniform(R, 3000 + r, span + span // 10 + 1)
        gkeys[::131] = EMPTY
        first = dev.log_append(_puts(keys, vals), 1)
        prev, pf = dev.log_exec(first, first + W)
        oprev, opf = om.replay(keys, vals)
        np.testing.assert_array_equal(pf, opf)
        np.testing.assert_array_equal(prev, oprev)
        gv, gf = dev.hm_get(gkeys)
        ov, of = om.get_batch(gkeys)
        np.testing.assert_array_equal(gf, of)
        np.testing.assert_array_equal(gv, ov)
    _check_state(dev, om)
    dev.close()


@pytest.mark.parametrize("path", list(PATHS))
def test_exec_without_responses_matches(nrg, orc, path):
    """benches/hashmap.rs:114-119 returns Ok(None): no previous-value pipeline."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=PATHS[path], log2_slots=16, max_batch=4096)
    om = orc.HashMap()
    for r in range(4):
        keys = orc.gen_uniform(3000, 7 + r, 700)
        vals = orc.gen_raw(3000, 70 + r)
        dev.log_append(_puts(keys, vals), 1)
        dev.log_exec()
        om.replay(keys, vals)
    _check_state(dev, om)


@pytest.mark.parametrize("path", list(PATHS))
def test_exec_chunks_longer_than_max_batch(nrg, orc, path):
    """An exec range longer than max_batch is replayed in order, chunk by chunk."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=PATHS[path], log2_slots=15, max_batch=1000)
    om = orc.HashMap()
    keys = orc.gen_uniform(4500, 5, 300)  # heavy duplication across chunk boundaries
    vals = orc.gen_raw(4500, 6)
    first = dev.log_append(_puts(keys, vals), 1)
    prev, pf = dev.log_exec(first, first + 4500)
    oprev, opf = om.replay(keys, vals)
    np.testing.assert_array_equal(pf, opf)
    np.testing.assert_array_equal(prev, oprev)
    _check_state(dev, om)


@pytest.mark.parametrize("path", list(PATHS))
def test_zipf_conflicts(nrg, orc, path):
    """Zipf 0.99 stream: hot keys stress last-writer-wins ordering and CAS contention."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=PATHS[path], log2_slots=20, max_batch=1 << 17)
    om = orc.HashMap()
    dev.hm_prefill_range(10000, 1)
    om.prefill_range(10000, 1)
    for r in range(3):
        W = 100_000
        keys = orc.gen_zipf(W, 11 + r, 100_000, 0.99, scramble=(r == 1))
        vals = orc.gen_raw(W, 12 + r)
        first = dev.log_append(_puts(keys, vals), 1)
        prev, pf = dev.log_exec(first, first + W)
        oprev, opf = om.replay(keys, vals)
        np.testing.assert_array_equal(pf, opf)
        np.testing.assert_array_equal(prev, oprev)
    _check_state(dev, om)


def test_fused_round_device(nrg, orc):
    """nrg_hashmap_round_async: append + replay + reads in one call on device buffers."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=18, max_batch=1 << 14)
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(20000, 1)
    om.prefill_range(20000, 1)
    W, R = 10000, 30000
    for r in range(4):
        keys = orc.gen_uniform(W, 40 + r, 25000)
        vals = orc.gen_raw(W, 50 + r)
        gk = orc.gen_uniform(R, 60 + r, 26000)
        d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.empty(R, dtype=torch.int64, device="cuda")
        d_gf = torch.empty(R, dtype=torch.uint8, device="cuda")
        d_pv = torch.empty(W, dtype=torch.int64, device="cuda")
        d_pf = torch.empty(W, dtype=torch.uint8, device="cuda")
        dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, d_pv, d_pf)
        torch.cuda.synchronize()
        oprev, opf = om.replay(keys, vals)
        ov, of = om.get_batch(gk)
        np.testing.assert_array_equal(d_pf.cpu().numpy(), opf)
        np.testing.assert_array_equal(d_pv.cpu().numpy().view(np.uint64), oprev)
        np.testing.assert_array_equal(d_gf.cpu().numpy(), of)
        np.testing.assert_array_equal(d_gv.cpu().numpy().view(np.uint64), ov)
    dev.sync()
    _check_state(dev, om)


@pytest.mark.parametrize("path", ["stamp", "part", "wide"])
def test_pipelined_rounds_back_to_back(nrg, orc, path):
    """config.pipeline = 1: rounds enqueued back to back, no host sync in between. Each round's
    reads run in the next round's launch, beside its index pass (and, for stamp rounds, beside
    the apply of their own round's writes), and must see exactly their own round's state (keys
    created by later rounds invisible, values overwritten later not yet there).
    Knob PART = 2 sends every round through partition rounds instead (their reads ride in the
    next round's partition launch); PA_TPB = 1024 applies them with 1024-thread workgroups."""
    import torch

    knobs = {"part": {"PART": 2}, "wide": {"PART": 2, "PA_TPB": 1024}}.get(path, {})
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=knobs, log2_slots=17, max_batch=1 << 14, pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(3000, 1)
    om.prefill_range(3000, 1)
    W, R, rounds = 6000, 20000, 8
    outs, want = [], []
    for r in range(rounds):
        keys = orc.gen_uniform(W, 140 + r, 9000)  # ~1/3 of each round's keys are new
        vals = orc.gen_raw(W, 150 + r)
        keys[::89] = EMPTY
        gk = orc.gen_uniform(R, 160 + r, 9500)
        gk[::101] = EMPTY
        d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        d_gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, None, None)
        outs.append((d_puts, d_gk, d_gv, d_gf))
        om.replay(keys, vals)
        want.append(om.get_batch(gk))
    dev.join()  # orders the last round's reads on the torch stream
    got = [(gv.cpu().numpy().view(np.uint64), gf.cpu().numpy()) for (_, _, gv, gf) in outs]
    for r in range(rounds):
        np.testing.assert_array_equal(got[r][1], want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(got[r][0], want[r][0], err_msg=f"round {r} vals")
    dev.sync()
    _check_state(dev, om)


def test_pipelined_empty_round_completes_the_last(nrg, orc):
    """config.pipeline = 1: an empty round (no Puts, no Gets) is "the next call" too -- it
    launches the last round's deferred apply and reads, for every data structure, so their
    outputs are complete once the stream passes it (no join)."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=17, max_batch=1 << 14, pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    W, R = 6000, 20000
    keys, vals = orc.gen_uniform(W, 170, 9000), orc.gen_raw(W, 171)
    gk = orc.gen_uniform(R, 172, 9500)
    d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
    d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
    d_gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
    d_gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
    dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, None, None)
    dev.hm_round_device(None, 0, 1, None, 0, None, None, None, None)  # the empty round
    torch.cuda.synchronize()
    om.replay(keys, vals)
    ev, ef = om.get_batch(gk)
    np.testing.assert_array_equal(d_gf.cpu().numpy(), ef.astype(np.uint8))
    np.testing.assert_array_equal(d_gv.cpu().numpy().view(np.uint64), ev)
    dev.sync()
    _check_state(dev, om)

    for kind, rnd in ((nrg._lib.NRG_DS_STACK, "st_round_device"), (nrg._lib.NRG_DS_SYNTHETIC, "sy_round_device")):
        d = nrg.DeviceReplica(kind, 0, max_batch=1 << 14, pipeline=1)
        d.use_torch_stream()
        n = 10_000
        if kind == nrg._lib.NRG_DS_STACK:
            ops = torch.from_numpy((orc.gen_raw(n, 173) & 0x1FFFFFFFF).astype(np.int64)).cuda()
            resp = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        else:
            raw = orc.gen_raw(4 * n, 174)
            o = np.stack([raw[0::4] % 64, raw[1::4], raw[2::4], np.ones(n, np.uint64)], 1).astype(np.uint64)
            ops = torch.from_numpy(o.view(np.int64)).cuda()
            resp = torch.full((n,), -1, dtype=torch.int64, device="cuda")
        some = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        getattr(d, rnd)(ops, n, 1, resp, some)
        getattr(d, rnd)(ops, 0, 1, None, None)  # the empty round
        torch.cuda.synchronize()
        assert np.all(some.cpu().numpy() != 7), f"{rnd}: the last round's deferred outputs did not complete"
        d.close()


@pytest.mark.parametrize("span", [40, 3000, 1 << 40])
def test_small_rounds_device(nrg, orc, span):
    """One-launch small rounds (hashmap.hip hm_small_round_kernel, the combiner's path):
    previous values of every Put with duplicate keys in log order (span 40: every key many
    times per round), the side-slot key, fresh claims, Gets after the round's writes, pipelined
    and plain contexts, rounds at the size limits (2048 Puts, 8192 Gets) and past them."""
    import torch

    for pipeline in (0, 1):
        dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs={"SMALL_MAX": 2048}, log2_slots=15,
                                max_batch=1 << 13, max_reads=1 << 14, pipeline=pipeline)
        dev.use_torch_stream()
        om = orc.HashMap()
        dev.hm_prefill_range(min(span, 500), 1)
        om.prefill_range(min(span, 500), 1)
        for r, (W, R) in enumerate([(1, 0), (300, 700), (2048, 8192), (2049, 100), (0, 500), (1000, 8193), (17, 5)]):
            keys = orc.gen_uniform(max(W, 1), 500 + r, span)[:W]
            vals = orc.gen_raw(max(W, 1), 600 + r)[:W]
            keys[::37] = EMPTY
            gk = orc.gen_uniform(max(R, 1), 700 + r, span + 50)[:R]
            gk[::41] = EMPTY
            d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
            d_gk = torch.from_numpy(gk.view(np.int64).copy()).cuda()
            d_gv = torch.full((max(R, 1),), -1, dtype=torch.int64, device="cuda")
            d_gf = torch.full((max(R, 1),), 7, dtype=torch.uint8, device="cuda")
            d_pv = torch.full((max(W, 1),), -1, dtype=torch.int64, device="cuda")
            d_pf = torch.full((max(W, 1),), 7, dtype=torch.uint8, device="cuda")
            dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, d_pv, d_pf)
            dev.join()
            torch.cuda.synchronize()
            oprev, opf = om.replay(keys, vals)
            ov, of = om.get_batch(gk)
            np.testing.assert_array_equal(d_pf.cpu().numpy()[:W], opf, err_msg=f"round {r}")
            np.testing.assert_array_equal(d_pv.cpu().numpy().view(np.uint64)[:W], oprev, err_msg=f"round {r}")
            np.testing.assert_array_equal(d_gf.cpu().numpy()[:R], of, err_msg=f"round {r}")
            np.testing.assert_array_equal(d_gv.cpu().numpy().view(np.uint64)[:R], ov, err_msg=f"round {r}")
        dev.sync()
        _check_state(dev, om)
        dev.close()


def test_small_round_table_full(nrg, orc):
    """A small round that cannot claim a slot latches NRG_E_TABLE_FULL (as the other paths)."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs={"SMALL_MAX": 2048}, log2_slots=8, max_batch=1024)
    keys = orc.gen_uniform(300, 9, 1 << 40)
    first = dev.log_append(_puts(keys, keys), 1)
    with pytest.raises(Exception):
        dev.log_exec(first, first + 300)
    dev.close()


def test_device_generator_matches_oracle(nrg, orc):
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=10, max_batch=1024)
    dev.use_torch_stream()
    d = torch.empty(100_000, dtype=torch.int64, device="cuda")
    dev.gen_uniform_device(d, 100_000, 1234, 10_000_000)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy().view(np.uint64), orc.gen_uniform(100_000, 1234, 10_000_000))
    dev.gen_raw_device(d, 100_000, 99)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy().view(np.uint64), orc.gen_raw(100_000, 99))


def test_not_synced_read_is_refused(nrg, orc):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=10, max_batch=1024)
    dev.log_append(_puts(np.array([1], np.uint64), np.array([2], np.uint64)), 1)
    with pytest.raises(nrg.NrgError) as e:
        dev.hm_get(np.array([1], np.uint64))
    assert e.value.code == nrg._lib.NRG_E_NOT_SYNCED
    dev.log_exec()
    v, f = dev.hm_get(np.array([1, 3], np.uint64))
    assert list(f) == [1, 0] and int(v[0]) == 2


def test_ring_wrap_and_gc(nrg, orc):
    """Many appends through a minimum-size log (16384 entries): ring wrap-around and the GC
    path of Log::append (exec before advancing head, nr/src/log.rs:364-387)."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=4096, log_bytes=1024)
    st = dev.log_state()
    assert st["size"] == 16384
    om = orc.HashMap()
    total = 0
    for r in range(12):
        n = 3000 + 17 * r
        keys = orc.gen_uniform(n, 300 + r, 5000)
        vals = orc.gen_raw(n, 400 + r)
        dev.log_append(_puts(keys, vals), 1)  # no exec: append's GC path replays when needed
        om.replay(keys, vals)
        total += n
    dev.log_exec()
    st = dev.log_state()
    assert st["tail"] == total and st["ltail"] == total and st["ctail"] == total
    _check_state(dev, om)


@pytest.mark.parametrize("pipeline", [0, 1])
def test_dense_segment_rounds(nrg, orc, pipeline):
    """nrg_hashmap_round_segments_async on equal-length segments (the all-gathered round of the
    multi-GPU bench): replayed in place in segment order, Put responses for one segment only,
    reads against the post-round state; with pipeline=1 the reads complete at the next call."""
    import torch

    G, W, R = 4, 3000, 5000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=17, max_batch=G * W, pipeline=pipeline)
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(2000, 1)
    om.prefill_range(2000, 1)
    outs, want = [], []
    for r in range(4):
        segs = [(orc.gen_uniform(W, 500 + 10 * r + g, 9000), orc.gen_raw(W, 600 + 10 * r + g)) for g in range(G)]
        segs[1][0][::37] = EMPTY
        base = np.concatenate([_puts(k, v) for k, v in segs])
        gk = orc.gen_uniform(R, 700 + r, 9500)
        d_base = torch.from_numpy(base.view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.empty(R, dtype=torch.int64, device="cuda")
        d_gf = torch.empty(R, dtype=torch.uint8, device="cuda")
        d_pv = torch.empty(W, dtype=torch.int64, device="cuda")
        d_pf = torch.empty(W, dtype=torch.uint8, device="cuda")
        own = r % G
        dev.hm_round_segments_device(d_base, W, [W] * G, [g + 1 for g in range(G)], own, d_gk, R, d_gv, d_gf,
                                     d_pv, d_pf)
        outs.append((d_base, d_gk, d_gv, d_gf, d_pv, d_pf))
        exp_prev = None
        for g, (k, v) in enumerate(segs):
            p, f = om.replay(k, v)
            if g == own:
                exp_prev = (p, f)
        want.append((om.get_batch(gk), exp_prev))
    dev.join()
    torch.cuda.synchronize()
    for (_, _, gv, gf, pv, pf), ((ov, of), (op, opf)) in zip(outs, want):
        np.testing.assert_array_equal(gf.cpu().numpy(), of)
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), ov)
        np.testing.assert_array_equal(pf.cpu().numpy(), opf)
        np.testing.assert_array_equal(pv.cpu().numpy().view(np.uint64), op)
    dev.sync()
    _check_state(dev, om)


def _mix64(x):
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


@pytest.mark.parametrize("knobs", [{}, {"PART": 2}, {"PART": 2, "STALL": 1}, {"PART": 2, "PA_TPB": 1024, "STALL": 1},
                                   {"PART": 2, "PA_TPB": 512, "STALL": 1}])
def test_one_bucket_rounds(nrg, orc, knobs):
    """Pipelined rounds whose keys all fall into ONE slot bucket (many chunks, finer parts,
    duplicates across index tiles), with side-slot keys and a Zipf round, against the oracle.
    Also as partition rounds (PART = 2: one apply workgroup takes the bucket in many chunks), and
    with odd waves stalled where a chunk's tile map is read (STALL = 1) before the next chunk
    rebuilds it."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=knobs, log2_slots=17, max_batch=8192, pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(3000, 1)
    om.prefill_range(3000, 1)
    cand = np.arange(1, 4_000_000, dtype=np.uint64)
    one_bucket = cand[(_mix64(cand) >> np.uint64(58)) == 0][:6000]  # top 6 home bits 0: bucket 0 of 64
    assert len(one_bucket) == 6000
    rounds = [orc.gen_uniform(6000, 240 + r, 9000) for r in range(3)]
    rounds.append(orc.gen_zipf(8000, 250, 20000, 0.99))
    rounds.append(np.concatenate([one_bucket, one_bucket[:1500]]))  # duplicates across tiles
    outs, want = [], []
    for r, keys in enumerate(rounds):
        keys = keys.copy()
        if r < 3:
            keys[::97] = EMPTY
        W = len(keys)
        vals = orc.gen_raw(W, 260 + r)
        R = 7000
        gk = np.concatenate([orc.gen_uniform(R - 100, 270 + r, 9500), one_bucket[:100]])
        d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        d_gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, None, None)
        outs.append((d_puts, d_gk, d_gv, d_gf))
        om.replay(keys, vals)
        want.append(om.get_batch(gk))
    dev.join()
    for r, (_, _, gv, gf) in enumerate(outs):
        np.testing.assert_array_equal(gf.cpu().numpy(), want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), want[r][0], err_msg=f"round {r} vals")
    dev.sync()
    _check_state(dev, om)


def _bucket_rounds(nrg, orc, dev, om, rounds):
    import torch

    outs, want = [], []
    for r, keys in enumerate(rounds):
        W = len(keys)
        vals = orc.gen_raw(W, 330 + r)
        R = 5000
        gk = np.concatenate([orc.gen_uniform(R - len(keys[:500]), 340 + r, 1 << 22), keys[:500]])
        R = len(gk)
        d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        d_gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, None, None)
        outs.append((d_puts, d_gk, d_gv, d_gf))
        om.replay(keys, vals)
        want.append(om.get_batch(gk))
    dev.join()
    for r, (_, _, gv, gf) in enumerate(outs):
        np.testing.assert_array_equal(gf.cpu().numpy(), want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), want[r][0], err_msg=f"round {r} vals")
    assert dev.hm_digest() == om.digest()


@pytest.mark.parametrize("knobs", [{"PART": 1}, {"PART": 2}, {"PART": 2, "PA_TPB": 256}])
def test_large_pipelined_rounds(nrg, orc, knobs):
    """Large pipelined rounds (300k-400k Puts: 2048-Put partition tiles, 256 wide buckets, or 1024
    with PA_TPB = 256): uniform and Zipf rounds with side-slot keys and a small round in between,
    against the sequential oracle; default round kinds, and every round a partition round
    (PART = 2)."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=knobs, log2_slots=22, max_batch=1 << 19,
                            pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(1 << 20, 1)
    om.prefill_range(1 << 20, 1)
    rounds = [orc.gen_uniform(300_000, 300, 3_000_000), orc.gen_zipf(400_000, 301, 2_000_000, 0.99),
              orc.gen_uniform(50_000, 302, 3_000_000), orc.gen_uniform(260_000, 303, 1 << 22)]
    rounds[0] = rounds[0].copy()
    rounds[0][::997] = EMPTY
    _bucket_rounds(nrg, orc, dev, om, rounds)


@pytest.mark.parametrize("knobs", [{"PART": 1}, {"PART": 2}, {"PART": 2, "PA_TPB": 1024}])
def test_crowded_bucket_rounds(nrg, orc, knobs):
    """2500 new keys of a round home into the first 4096 slots of the table (one partition bucket,
    taken in several chunks; their claims crowd one region, long probe chains), repeated and
    reversed in later rounds, against the sequential oracle."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs=knobs, log2_slots=20, max_batch=1 << 14,
                            pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    cand = np.arange(1, 4_000_000, dtype=np.uint64)
    low = cand[(_mix64(cand) >> np.uint64(44)) < 4096][:2500]
    assert len(low) == 2500
    rounds = [np.concatenate([low, low[:600]]), orc.gen_uniform(9000, 310, 50_000),
              np.concatenate([low[::-1], low[:300]])]
    _bucket_rounds(nrg, orc, dev, om, rounds)


def test_b1_full_size_rounds(nrg, orc):
    """BASELINE configs[1] at full size: 2^26-slot table, prefill [0, 2^23) -> k+1, uniform keys
    over 10M, rounds of 100k Puts + 900k Gets (stamp election), then an 800k-Put round (the
    per-GPU replay at 8 GPUs, bucket election) -- every Get response and the final replica
    digest bit-exact against the sequential oracle."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, log2_slots=26, max_batch=1 << 20, pipeline=1,
                            log_bytes=64 * 4 * (1 << 20))
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(1 << 23, 1)
    om.prefill_range(1 << 23, 1)
    outs, want = [], []
    for r, (W, R) in enumerate([(100_000, 900_000), (100_000, 900_000), (800_000, 900_000)]):
        keys = orc.gen_uniform(W, 0x4E52 + 3 * r, 10_000_000)
        vals = orc.gen_raw(W, 0x4E52 + 3 * r + 1)
        gk = orc.gen_uniform(R, 0x4E52 + 3 * r + 2, 10_000_000)
        d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        d_gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, None, None)
        outs.append((d_puts, d_gk, d_gv, d_gf))
        om.replay(keys, vals)
        want.append(om.get_batch(gk))
    dev.join()
    for r, (_, _, gv, gf) in enumerate(outs):
        np.testing.assert_array_equal(gf.cpu().numpy(), want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), want[r][0], err_msg=f"round {r} vals")
    assert dev.hm_digest() == om.digest()


def test_epoch_renormalisation(nrg, orc):
    """Replay epochs are 32-bit; before they wrap every stamp is renormalised to epoch 1. A limit
    of 6 (knob EPOCH_LIMIT) renormalises every few rounds: pipelined stamp and partition rounds with
    new keys, overwrites and side-slot keys across several renormalisations, against the oracle."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs={"EPOCH_LIMIT": 6, "STAMP_MAX": 5000},
                            log2_slots=16, max_batch=8192, pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(500, 1)
    om.prefill_range(500, 1)
    outs, want = [], []
    for r in range(17):
        W = 3000 if r % 3 else (7000 if r % 2 else 6000)  # > STAMP_MAX: partition rounds
        keys = orc.gen_uniform(W, 900 + r, 4000 + 150 * r)
        keys[::113] = EMPTY
        vals = orc.gen_raw(W, 950 + r)
        R = 3000
        gk = orc.gen_uniform(R, 990 + r, 7000)
        gk[::127] = EMPTY
        d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        d_gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, None, None)
        outs.append((d_puts, d_gk, d_gv, d_gf))
        om.replay(keys, vals)
        want.append(om.get_batch(gk))
    dev.join()
    for r, (_, _, gv, gf) in enumerate(outs):
        np.testing.assert_array_equal(gf.cpu().numpy(), want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), want[r][0], err_msg=f"round {r} vals")
    dev.sync()
    _check_state(dev, om)


@pytest.mark.parametrize("part", [0, 2])
def test_skew_switches_round_kind(nrg, orc, part):
    """Stamp rounds (one launch, one stamp atomic per distinct key per block) are faster for
    uniform keys, partition rounds (no atomics per Put) for skewed ones; the replica switches from
    the sampled share of Puts combined inside their block (every 2 rounds here). Uniform rounds,
    then Zipf(0.99), then uniform again, pipelined: every Get and the final state bit-exact
    across both switches, and the switches happen. part = 2: partition rounds, which drop the
    Puts overwritten inside their tile only while the stream is skewed (and in the last round of
    every sample window, which measures it)."""
    import ctypes as C

    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs={"SKEW_EVERY": 2, "PART": part}, log2_slots=19,
                            max_batch=1 << 15, pipeline=1)
    dev.use_torch_stream()
    om = orc.HashMap()
    dev.hm_prefill_range(5000, 1)
    om.prefill_range(5000, 1)
    W, R, span = 8000, 16000, 200_000
    kinds, outs, want = [], [], []
    for r in range(18):
        zipf = 6 <= r < 12
        keys = orc.gen_zipf(W, 300 + r, span, 0.99) if zipf else orc.gen_uniform(W, 300 + r, span)
        vals = orc.gen_raw(W, 330 + r)
        gk = orc.gen_zipf(R, 360 + r, span, 0.99) if zipf else orc.gen_uniform(R, 360 + r, span)
        d_puts = torch.from_numpy(_puts(keys, vals).view(np.int64).copy()).cuda()
        d_gk = torch.from_numpy(gk.view(np.int64)).cuda()
        d_gv = torch.full((R,), -1, dtype=torch.int64, device="cuda")
        d_gf = torch.full((R,), 7, dtype=torch.uint8, device="cuda")
        dev.hm_round_device(d_puts, W, 1, d_gk, R, d_gv, d_gf, None, None)
        outs.append((d_puts, d_gk, d_gv, d_gf))
        om.replay(keys, vals)
        want.append(om.get_batch(gk))
        torch.cuda.synchronize()  # the skew sample lands before the next decision
        flag = C.c_int(-1)
        nrg._lib.check(nrg.load().nrg_test_hm_skewed(dev.handle, C.byref(flag)))
        kinds.append(flag.value)
    dev.join()
    for r, (_, _, gv, gf) in enumerate(outs):
        np.testing.assert_array_equal(gf.cpu().numpy(), want[r][1], err_msg=f"round {r} found")
        np.testing.assert_array_equal(gv.cpu().numpy().view(np.uint64), want[r][0], err_msg=f"round {r} vals")
    dev.sync()
    _check_state(dev, om)
    assert kinds[:6] == [0] * 6, kinds
    assert kinds[11] == 1, kinds
    assert kinds[17] == 0, kinds
