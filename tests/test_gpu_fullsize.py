"""Full-size NrHashMap rounds of every BASELINE config that fits one GPU, against the oracle.

BASELINE.json configs and the per-GPU replay each one implies:
  configs[1] (B1)  2^26 slots, prefill [0, 2^23) -> k+1, 10M keys, rounds of 100k Put + 900k Get
  configs[2] (B8)  8 GPUs at 50 % writes: every replica replays 8 x 500k Puts per round (all
                   ranks' all-gathered segments, nr/src/log.rs:473-524) and answers its own 500k
                   Gets; Put responses only for its own segment (nr/src/replica.rs:576-578)
  configs[3] (Z)   Zipf theta = 0.99 at 50 % writes, hot keys adjacent and scrambled
Every round here asks for HashMap::insert's previous values (nr/examples/hashmap.rs:46-50) as
well as the Gets, so the whole response stream and the final replica are checked bit-exactly.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = 10_000_000
PREFILL = 1 << 23


def _puts(keys, vals):
    import nrgpu

    r = np.zeros(len(keys), nrgpu.PUT_DTYPE)
    r["key"] = keys
    r["val"] = vals
    return r


def _dev(nrg, max_batch, part=0):
    dev = nrg.DeviceReplica(nrg._lib.NRG_DS_HASHMAP, 0, knobs={"PART": part}, log2_slots=26, max_batch=max_batch,
                            pipeline=1, log_bytes=64 * 4 * max_batch)
    dev.use_torch_stream()
    dev.hm_prefill_range(PREFILL, 1)
    return dev


def _prefilled_oracle(orc):
    om = orc.HashMap(PREFILL + (1 << 21))
    om.prefill_range(PREFILL, 1)
    return om


def _cuda(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).cuda()


def _out(n, dtype, fill):
    import torch

    return torch.full((n,), fill, dtype=dtype, device="cuda")


def _check(got, want, what):
    import torch

    g = got.cpu().numpy()
    if got.dtype == torch.int64:
        g = g.view(np.uint64)
    np.testing.assert_array_equal(g, want, err_msg=what)


@pytest.mark.parametrize("part", [0, 2])
def test_b1_rounds_with_previous_values(nrg, orc, part):
    """configs[1] with HashMap::insert's previous values: 3 pipelined 100k + 900k rounds (partition
    rounds with the log-order walk; part = 2 changes nothing here but is kept as the forced path)."""
    import torch

    dev = _dev(nrg, 1 << 20, part)
    om = _prefilled_oracle(orc)
    outs = []
    for r in range(3):
        W, R = 100_000, 900_000
        keys = orc.gen_uniform(W, 0xB1 + 3 * r, KEYS)
        vals = orc.gen_raw(W, 0xB1 + 3 * r + 1)
        gk = orc.gen_uniform(R, 0xB1 + 3 * r + 2, KEYS)
        d = dict(puts=_cuda(_puts(keys, vals)), gk=_cuda(gk), gv=_out(R, torch.int64, -1), gf=_out(R, torch.uint8, 7),
                 pv=_out(W, torch.int64, -1), pf=_out(W, torch.uint8, 7))
        dev.hm_round_device(d["puts"], W, 1, d["gk"], R, d["gv"], d["gf"], d["pv"], d["pf"])
        pv, pf = om.replay(keys, vals)
        gv, gf = om.get_batch(gk)
        outs.append((d, pv, pf, gv, gf))
    dev.join()
    for r, (d, pv, pf, gv, gf) in enumerate(outs):
        _check(d["pf"], pf, f"round {r} prev found")
        _check(d["pv"], pv, f"round {r} prev vals")
        _check(d["gf"], gf, f"round {r} get found")
        _check(d["gv"], gv, f"round {r} get vals")
    assert dev.hm_digest() == om.digest()
    dev.close()


@pytest.mark.parametrize("part", [0, 2])
@pytest.mark.parametrize("prev", [True, False])
def test_configs2_per_gpu_round(nrg, orc, prev, part):
    """configs[2]'s per-GPU work: 8 segments x 500k Puts (the all-gathered round of 8 ranks at 50 %
    writes, 4M Puts replayed in place) + this rank's 500k Gets, two pipelined rounds through
    nrg_hashmap_round_segments_async; with previous values for the rank's own segment or without
    (Ok(None)). Rounds this large take partition rounds by default (part = 0 sends only those with
    previous values there, the others through 4M-Put stamp rounds); part = 2: partition rounds
    either way."""
    import torch

    G, W, R = 8, 500_000, 500_000
    dev = _dev(nrg, G * W, part)
    om = _prefilled_oracle(orc)
    outs = []
    for r, own in enumerate([3, 6]):
        segs = [(orc.gen_uniform(W, 0xC2 + 100 * r + g, KEYS), orc.gen_raw(W, 0xC2 + 100 * r + 50 + g))
                for g in range(G)]
        base = np.concatenate([_puts(k, v) for k, v in segs])
        gk = orc.gen_uniform(R, 0xC2 + 100 * r + 99, KEYS)
        d = dict(base=_cuda(base), gk=_cuda(gk), gv=_out(R, torch.int64, -1), gf=_out(R, torch.uint8, 7),
                 pv=_out(W, torch.int64, -1), pf=_out(W, torch.uint8, 7))
        dev.hm_round_segments_device(d["base"], W, [W] * G, [g + 1 for g in range(G)], own, d["gk"], R, d["gv"],
                                     d["gf"], d["pv"] if prev else None, d["pf"] if prev else None)
        exp = None
        for g, (k, v) in enumerate(segs):
            p = om.replay(k, v)
            if g == own:
                exp = p
        outs.append((d, exp, om.get_batch(gk)))
    dev.join()
    for r, (d, (pv, pf), (gv, gf)) in enumerate(outs):
        if prev:
            _check(d["pf"], pf, f"round {r} prev found")
            _check(d["pv"], pv, f"round {r} prev vals")
        _check(d["gf"], gf, f"round {r} get found")
        _check(d["gv"], gv, f"round {r} get vals")
    assert dev.hm_digest() == om.digest()
    st = dev.log_state()
    assert st["tail"] == st["ltail"] == st["ctail"] == 2 * G * W
    dev.close()


def test_largest_round(nrg, orc):
    """The largest round one call replays (HM_MAX_BATCH = 2^23 Puts) + 1M Gets, pipelined twice:
    4096 partition tiles, the apply's 1024-thread workgroups with their tile prefix at its largest
    LDS size, 256 buckets of ~32k Puts (8 chunks each), against the oracle."""
    import torch

    W, R = 1 << 23, 1_000_000
    dev = _dev(nrg, W, 1)
    om = _prefilled_oracle(orc)
    outs = []
    for r in range(2):
        k = orc.gen_uniform(W, 0x1A7 + r, KEYS)
        v = orc.gen_raw(W, 0x2A7 + r)
        gk = orc.gen_uniform(R, 0x3A7 + r, KEYS)
        d = dict(p=_cuda(_puts(k, v)), gk=_cuda(gk), gv=_out(R, torch.int64, -1), gf=_out(R, torch.uint8, 7))
        dev.hm_round_device(d["p"], W, 1, d["gk"], R, d["gv"], d["gf"], None, None)
        om.replay(k, v)
        outs.append((d, om.get_batch(gk)))
    dev.join()
    for r, (d, (gv, gf)) in enumerate(outs):
        _check(d["gf"], gf, f"round {r} get found")
        _check(d["gv"], gv, f"round {r} get vals")
    assert dev.hm_digest() == om.digest()
    dev.close()


@pytest.mark.parametrize("part", [0, 2])
@pytest.mark.parametrize("scramble", [False, True])
def test_zipf_50pct_full_size(nrg, orc, scramble, part):
    """configs[3]: Zipf(0.99) over the 10M key space at 50 % writes (500k Puts + 500k Gets per
    round), hot keys adjacent or scrambled; last-writer-wins and every previous value under
    heavy same-key conflicts, pipelined rounds with and without responses."""
    import torch

    W, R = 500_000, 500_000
    dev = _dev(nrg, 1 << 20, part)
    om = _prefilled_oracle(orc)
    outs = []
    for r in range(3):
        keys = orc.gen_zipf(W, 0x21F + 3 * r, KEYS, 0.99, scramble=scramble)
        vals = orc.gen_raw(W, 0x21F + 3 * r + 1)
        gk = orc.gen_zipf(R, 0x21F + 3 * r + 2, KEYS, 0.99, scramble=scramble)
        want_prev = r != 1
        d = dict(puts=_cuda(_puts(keys, vals)), gk=_cuda(gk), gv=_out(R, torch.int64, -1), gf=_out(R, torch.uint8, 7),
                 pv=_out(W, torch.int64, -1), pf=_out(W, torch.uint8, 7))
        dev.hm_round_device(d["puts"], W, 1, d["gk"], R, d["gv"], d["gf"], d["pv"] if want_prev else None,
                            d["pf"] if want_prev else None)
        pv, pf = om.replay(keys, vals)
        outs.append((d, want_prev, pv, pf, om.get_batch(gk)))
    dev.join()
    for r, (d, want_prev, pv, pf, (gv, gf)) in enumerate(outs):
        if want_prev:
            _check(d["pf"], pf, f"round {r} prev found")
            _check(d["pv"], pv, f"round {r} prev vals")
        _check(d["gf"], gf, f"round {r} get found")
        _check(d["gv"], gv, f"round {r} get vals")
    assert dev.hm_digest() == om.digest()
    dev.close()
