"""AbstractDataStructure parity (benches/synthetic.rs): HIP replay vs oracle.

Both replay paths are covered: the default sort-free bucket replay (one launch per round, and
the two-launch form, knob NRG_KNOB_SY_FUSED = 0) and the sort-based one (knob NRG_KNOB_SY_SORT =
1, kept for configurations the bucket path does not take).

The bench uses ReadWrite only with tid = core id (:296-335); WriteOnly and ReadOnly are
part of the data structure's Dispatch (:177-195) and are covered too, including the
wrapping corner cases (r2 = u64::MAX empties the hot range; r1*tid overflow).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ops(orc, n, seed, tids, wo_frac):
    import nrgpu

    r = np.zeros(n, nrgpu.SYNTH_OP_DTYPE)
    raw = orc.gen_raw(4 * n, seed)
    r["tid"] = np.asarray(tids, np.uint64)[raw[0::4] % len(tids)]
    r["r1"] = raw[1::4]
    r["r2"] = raw[2::4]
    r["op"] = (raw[3::4] % 100 >= wo_frac).astype(np.uint64)  # 1 = ReadWrite
    return r


@pytest.fixture(params=["bucket", "bucket2", "sort"])
def path(request):
    """the replay path's knobs (nrg_test_set_knob): the bucket path in one launch per round
    (default: chunk e's partition, e-1's bucket pass and e-2's sums side by side), in two launches
    per round (SY_FUSED = 0), and the sort path"""
    return {"sort": {"SY_SORT": 1}, "bucket2": {"SY_FUSED": 0}, "bucket": {}}[request.param]


def _check_rounds(nrg, orc, dev, os_, rounds, n, seed, tids, wo, tweak=None):
    for r in range(rounds):
        ops = _ops(orc, n, seed + r, tids, wo)
        if tweak:
            tweak(ops)
        first = dev.log_append(ops, 1)
        resp, some = dev.log_exec(first, first + n)
        oresp = os_.replay(np.stack([ops["tid"], ops["r1"], ops["r2"], ops["op"]], axis=1))
        np.testing.assert_array_equal(resp, oresp)
        assert np.all(some == 1)
    np.testing.assert_array_equal(dev.sy_dump(), os_.dump())


@pytest.mark.parametrize("n,wo,tids", [(1000, 0, [0]), (20000, 0, [0, 1, 5, 63]), (20000, 30, [3, 7]),
                                       (5000, 100, [1, 2])])
def test_synth_rounds(nrg, orc, path, n, wo, tids):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs=path, max_batch=1 << 15)
    os_ = orc.Synthetic()
    for r in range(3):
        ops = _ops(orc, n, 900 + r, tids, wo)
        ops["r2"][::101] = 0xFFFFFFFFFFFFFFFF  # empty hot range
        ops["r2"][::113] = 0  # every cold touch on the same word
        first = dev.log_append(ops, 1)
        resp, some = dev.log_exec(first, first + n)
        oresp = os_.replay(np.stack([ops["tid"], ops["r1"], ops["r2"], ops["op"]], axis=1))
        np.testing.assert_array_equal(resp, oresp)
        rd = np.zeros(500, nrg.SYNTH_RD_DTYPE)
        raw = orc.gen_raw(1500, 50 + r)
        rd["tid"] = raw[0::3] % 8
        rd["r1"] = raw[1::3]
        rd["r2"] = raw[2::3]
        np.testing.assert_array_equal(dev.sy_read(rd),
                                      os_.read(np.stack([rd["tid"], rd["r1"], rd["r2"]], axis=1)))
    np.testing.assert_array_equal(dev.sy_dump(), os_.dump())


def test_synth_large_rounds(nrg, orc, path):
    """Many 2048-op tiles and all 391 buckets: the bench's op kind (ReadWrite, tid < 64)."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs=path, max_batch=1 << 19)
    _check_rounds(nrg, orc, dev, orc.Synthetic(), 3, 300_000, 4242, list(range(64)), 0)
    dev.close()


@pytest.mark.parametrize("wo", [0, 10])
def test_synth_one_word(nrg, orc, path, wo):
    """tid = 0 and r2 = 0: every cold touch of every op lands on word hot_reads (one bucket
    with 5n touches, several 16K-touch passes) and every hot touch on word 0."""
    def tweak(ops):
        ops["r2"][:] = 0
        ops["tid"][::7] = 0

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs=path, max_batch=1 << 16)
    _check_rounds(nrg, orc, dev, orc.Synthetic(), 2, 40_000, 77, [0], wo, tweak)
    dev.close()


@pytest.mark.parametrize("n", [1, 2, 3, 5, 4099])
def test_synth_word0_parts(nrg, orc, n):
    """Cold word 0 (every op's first cold touch for tid 0) is replayed by four workgroups in a
    chunk without a WriteOnly, each from the word's value plus the touches before its part
    (synthetic.hip SY_B0_PARTS): chunks of 1-3 touches leave parts empty, and a chunk with one
    WriteOnly goes back to one workgroup; words and responses against the oracle."""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, max_batch=1 << 13)
    os_ = orc.Synthetic()

    def one_wo(ops):
        ops["op"][len(ops) // 2] = 0  # WriteOnly
    _check_rounds(nrg, orc, dev, os_, 2, n, 600 + n, [0], 0)
    _check_rounds(nrg, orc, dev, os_, 1, n, 700 + n, [0], 0, one_wo)
    _check_rounds(nrg, orc, dev, os_, 1, n, 800 + n, [0, 0, 0, 9], 0)
    dev.close()


def test_synth_wide_values(nrg, orc, path):
    """Seen values past 2^32. The bucket pass stores 4-B seen values only while every word is
    < 2^31 and no WriteOnly of the chunk writes a tid >= 2^31 (synthetic.hip SyFlags): a chunk
    whose WriteOnlys write 2^40-scale tids, chunks that read the words they left (8-B seen
    values), then WriteOnlys with small tids over every word, which bring the 4-B path back."""
    n = 30_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs=path, max_batch=1 << 15)
    os_ = orc.Synthetic()
    big = [(1 << 40) + 3, (1 << 31), 0xFFFFFFFFFFFFFFF0]

    def wide(ops):
        ops["tid"][::5] = np.asarray(big, np.uint64)[np.arange(len(ops["tid"][::5])) % 3]
        ops["op"][::5] = 0  # WriteOnly
    _check_rounds(nrg, orc, dev, os_, 1, n, 31, [1, 2, 3], 0)      # 4-B seen values
    _check_rounds(nrg, orc, dev, os_, 1, n, 32, [1, 2, 3], 0, wide)  # big tids this chunk
    _check_rounds(nrg, orc, dev, os_, 2, n, 34, [1, 2, 3], 0)      # big words left over
    # WriteOnly with tid 1 on every cold word: op i's touches are words [5i, 5i + 5) (r1 = 5i, r2 = 1)
    w = np.zeros(40_000, nrg.SYNTH_OP_DTYPE)
    w["tid"], w["r1"], w["r2"], w["op"] = 1, np.arange(40_000, dtype=np.uint64) * 5, 1, 0
    for a in range(0, 40_000, 10_000):
        first = dev.log_append(w[a:a + 10_000], 1)
        dev.log_exec(first, first + 10_000)
        os_.replay(np.stack([w["tid"][a:a + 10_000], w["r1"][a:a + 10_000], w["r2"][a:a + 10_000],
                             w["op"][a:a + 10_000]], axis=1))
    np.testing.assert_array_equal(dev.sy_dump(), os_.dump())
    assert int(dev.sy_dump()[2:].max()) < (1 << 31)
    _check_rounds(nrg, orc, dev, os_, 2, n, 36, [1, 2, 3], 0)      # 4-B seen values again
    dev.close()


def test_synth_partial_tiles_mixed(nrg, orc, path):
    """Round sizes that end mid-tile and mid-wave, WriteOnly runs, wrapped hot ranges."""
    def tweak(ops):
        ops["op"][1000:1300] = 0
        ops["r2"][::37] = 0xFFFFFFFFFFFFFFFF

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs=path, max_batch=1 << 15)
    os_ = orc.Synthetic()
    for n, seed in ((1, 5), (63, 6), (2049, 7), (4095, 8), (12345, 9)):
        _check_rounds(nrg, orc, dev, os_, 1, n, seed, [0, 2, 9, 31, 63], 5, tweak if n > 1300 else None)
    dev.close()


@pytest.mark.parametrize("n,wo,tids", [(20000, 0, [0, 1, 5, 63]), (20000, 30, [3, 7])])
def test_synth_round_fused(nrg, orc, path, n, wo, tids):
    """nrg_synth_round_async (append fused into the first replay pass) == the oracle, over
    several rounds whose ring positions wrap (small log)."""
    import torch

    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs=path, max_batch=1 << 15, log_bytes=64 * 65536)
    os_ = orc.Synthetic()
    resp = torch.zeros(n, dtype=torch.int64, device="cuda")
    some = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for r in range(5):
        ops = _ops(orc, n, 950 + r, tids, wo)
        d_ops = torch.from_numpy(ops.view(np.int64).reshape(n, -1).copy()).cuda()
        dev.sy_round_device(d_ops, n, 1, resp, some)
        torch.cuda.synchronize()
        oresp = os_.replay(np.stack([ops["tid"], ops["r1"], ops["r2"], ops["op"]], axis=1))
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint64), oresp)
        assert np.all(some.cpu().numpy() == 1)
    np.testing.assert_array_equal(dev.sy_dump(), os_.dump())


@pytest.mark.parametrize("fused", [1, 0])
def test_synth_bench_size_rounds(nrg, orc, fused):
    """The bench's synthetic rounds at full size: 1M ReadWrite ops (tid < 64) against the
    200,000-word storage, every sum and the final storage bit-exact against the oracle."""
    import torch

    n = 1_000_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs={"SY_FUSED": fused}, max_batch=n,
                            log_bytes=64 * 4 * n)
    os_ = orc.Synthetic()
    resp = torch.zeros(n, dtype=torch.int64, device="cuda")
    some = torch.zeros(n, dtype=torch.uint8, device="cuda")
    for r in range(2):
        ops = _ops(orc, n, 970 + r, list(range(64)), 0)
        d_ops = torch.from_numpy(ops.view(np.int64).reshape(n, -1).copy()).cuda()
        dev.sy_round_device(d_ops, n, 1, resp, some)
        torch.cuda.synchronize()
        oresp = os_.replay(np.stack([ops["tid"], ops["r1"], ops["r2"], ops["op"]], axis=1))
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint64), oresp)
    np.testing.assert_array_equal(dev.sy_dump(), os_.dump())


def _heavy(ops):
    ops["tid"][::3] = 0
    ops["r2"][::20] = 0


@pytest.mark.parametrize("fused", [1, 0])
@pytest.mark.parametrize("stall", [0, 1])
@pytest.mark.parametrize("wo", [0, 40])
def test_synth_heavy_buckets(nrg, orc, wo, stall, fused):
    """Skewed rounds: tid 0 (whose cold touches start at word hot_reads) on 30 % of the ops and
    r2 = 0 (all of an op's cold touches on one word) on 5 %, so a few buckets carry several times
    the mean and take many passes; WriteOnly ops make the values depend on each word's last SET.
    stall = 1 (NRG_KNOB_STALL): odd waves of every bucket workgroup sleep before each pass's value
    stores, which read the pass's tile map while the next-but-one pass rebuilds it."""
    tweak = _heavy
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs={"STALL": stall, "SY_FUSED": fused}, max_batch=1 << 18)
    _check_rounds(nrg, orc, dev, orc.Synthetic(), 4, 200_000, 0x4EA + wo, list(range(64)), wo, tweak)
    dev.close()


@pytest.mark.parametrize("fused", [1, 0])
def test_stall_exposes_a_missing_barrier(nrg, orc, fused):
    """The stall knob makes the race that 2a46f39's barrier closes deterministic: with the barrier
    after each pass's value stores dropped (STALL = 3, diagnostic only) the slow waves store
    through a tile map the fast waves have already rebuilt for a later pass, and the heavy rounds
    come out wrong every time; test_synth_heavy_buckets[stall=1] is the same stall with the
    barrier in place. (Stores the broken map would send outside V are dropped.)"""
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs={"STALL": 3, "SY_FUSED": fused}, max_batch=1 << 18)
    os_ = orc.Synthetic()
    ops = _ops(orc, 200_000, 0x4EA, list(range(64)), 0)
    _heavy(ops)
    first = dev.log_append(ops, 1)
    resp, _ = dev.log_exec(first, first + len(ops))
    oresp = os_.replay(np.stack([ops["tid"], ops["r1"], ops["r2"], ops["op"]], axis=1))
    assert np.count_nonzero(resp != oresp) > 0, "the stall did not expose the missing barrier"
    dev.close()


@pytest.mark.parametrize("fused", [1, 0])
def test_synth_pipelined_rounds(nrg, orc, fused):
    """pipeline=1: with one launch per round a chunk's bucket pass rides in the next chunk's launch
    and its sums in the one after (two launches per round: its sums in the next chunk's
    partition launch); every round answers into its own buffers, complete after nrg_join. Then reads
    (ReadOnly, which see the folded hot words), a multi-chunk exec and the final storage, all
    against the oracle (benches/synthetic.rs:112-195)."""
    import torch

    n = 100_000
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, knobs={"SY_FUSED": fused}, max_batch=1 << 17,
                            log_bytes=64 * 4 * (1 << 19), pipeline=1)
    os_ = orc.Synthetic()
    outs = []
    for r in range(4):
        ops = _ops(orc, n, 1200 + r, list(range(64)), 10 if r == 2 else 0)
        d_ops = torch.from_numpy(ops.view(np.int64).reshape(n, -1).copy()).cuda()
        resp = torch.zeros(n, dtype=torch.int64, device="cuda")
        some = torch.zeros(n, dtype=torch.uint8, device="cuda")
        dev.sy_round_device(d_ops, n, 1, resp, some)
        outs.append((d_ops, resp, some, os_.replay(np.stack([ops["tid"], ops["r1"], ops["r2"], ops["op"]], axis=1))))
    dev.join()
    torch.cuda.synchronize()
    for r, (_, resp, some, oresp) in enumerate(outs):
        np.testing.assert_array_equal(resp.cpu().numpy().view(np.uint64), oresp, err_msg=f"round {r}")
        assert np.all(some.cpu().numpy() == 1)
    rd = np.zeros(500, nrg.SYNTH_RD_DTYPE)
    raw = orc.gen_raw(1500, 77)
    rd["tid"], rd["r1"], rd["r2"] = raw[0::3] % 8, raw[1::3], raw[2::3]
    np.testing.assert_array_equal(dev.sy_read(rd), os_.read(np.stack([rd["tid"], rd["r1"], rd["r2"]], axis=1)))
    _check_rounds(nrg, orc, dev, os_, 1, 3 * (1 << 17) - 11, 1300, [0, 3, 63], 5)
    dev.close()
