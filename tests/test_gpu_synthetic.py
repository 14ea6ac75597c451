"""AbstractDataStructure parity (benches/synthetic.rs): HIP sort-based replay vs oracle.

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


@pytest.mark.parametrize("n,wo,tids", [(1000, 0, [0]), (20000, 0, [0, 1, 5, 63]), (20000, 30, [3, 7]),
                                       (5000, 100, [1, 2])])
def test_synth_rounds(nrg, orc, n, wo, tids):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_SYNTHETIC, 0, max_batch=1 << 15)
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
