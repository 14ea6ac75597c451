"""Generate the golden fixtures in tests/golden/ from pure-Python models.

The reference (Rust `nr`) cannot run here and ships no golden vectors,
so the fixtures are produced by the plainest possible restatement of each data structure's
Dispatch semantics, independent of the C oracle and of the HIP path:
  - NrHashMap  : a Python dict      (HashMap::insert -> previous value, get -> Option)
                 nr/examples/hashmap.rs:46-50, benches/hashmap.rs:77-122
  - Stack      : a Python list      (Vec::push / Vec::pop)  benches/stack.rs:36-84,
                 nr/tests/stack.rs:42-96
  - Synthetic  : Python ints mod 2^64 (release-build wrapping)  benches/synthetic.rs:60-195
Inputs come from the seeded splitmix64 stream shared by oracle/ and the GPU generator
(first value for seed 0 is the published splitmix64 test vector 0xe220a8397b1dcdaf).

Run:  python tests/golden/make_golden.py   (writes *.npz next to this file)
"""
import os

import numpy as np

M64 = (1 << 64) - 1
HERE = os.path.dirname(os.path.abspath(__file__))


def mix64(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def sm64_at(seed, i):
    return mix64((seed + (i + 1) * 0x9E3779B97F4A7C15) & M64)


def uniform(seed, i, span):
    return (sm64_at(seed, i) * span) >> 64


def hashmap_fixture(seed, rounds, W, R, span, prefill):
    d = {k: k + 1 for k in range(prefill)}
    puts_k, puts_v, gets_k = [], [], []
    prev_v, prev_f, get_v, get_f = [], [], [], []
    c = 0
    for r in range(rounds):
        for i in range(W):
            k = uniform(seed, c, span)
            c += 1
            if (c % 53) == 0:
                k = M64  # the one key equal to the GPU table's empty marker
            v = sm64_at(seed + 1, c)
            puts_k.append(k)
            puts_v.append(v)
            old = d.get(k)
            prev_v.append(old if old is not None else 0)
            prev_f.append(1 if old is not None else 0)
            d[k] = v
        for i in range(R):
            k = uniform(seed + 2, c, span + span // 4)
            c += 1
            if (c % 71) == 0:
                k = M64
            gets_k.append(k)
            got = d.get(k)
            get_v.append(got if got is not None else 0)
            get_f.append(1 if got is not None else 0)
    fk = np.array(sorted(d), dtype=np.uint64)
    fv = np.array([d[k] for k in sorted(d)], dtype=np.uint64)
    return dict(seed=seed, rounds=rounds, W=W, R=R, span=span, prefill=prefill,
                puts_k=np.array(puts_k, np.uint64), puts_v=np.array(puts_v, np.uint64),
                gets_k=np.array(gets_k, np.uint64), prev_v=np.array(prev_v, np.uint64),
                prev_f=np.array(prev_f, np.uint8), get_v=np.array(get_v, np.uint64),
                get_f=np.array(get_f, np.uint8), final_k=fk, final_v=fv)


def stack_fixture(seed, n, init_n, push_resp):
    s = list(range(init_n))
    vals, ops, resp, some = [], [], [], []
    for i in range(n):
        r = sm64_at(seed, i)
        op, v = r & 1, r >> 32
        if i % 500 < 60:
            op = 0  # runs of pops that drain the stack (saturating depth at 0)
        vals.append(v)
        ops.append(op)
        if op:
            s.append(v)
            resp.append(v if push_resp else 0)
            some.append(1 if push_resp else 0)
        elif s:
            resp.append(s.pop())
            some.append(1)
        else:
            resp.append(0)
            some.append(0)
    return dict(seed=seed, n=n, init_n=init_n, push_resp=push_resp, vals=np.array(vals, np.uint32),
                ops=np.array(ops, np.uint32), resp=np.array(resp, np.uint32), some=np.array(some, np.uint8),
                final=np.array(s, np.uint32))


def synth_fixture(seed, n, words, tids):
    HR, HW, CW, CR = 2, 1, 5, 20
    st = list(range(words))
    ops = np.zeros((n, 4), np.uint64)
    resp = []
    for i in range(n):
        tid = tids[sm64_at(seed, 4 * i) % len(tids)]
        r1, r2 = sm64_at(seed, 4 * i + 1), sm64_at(seed, 4 * i + 2)
        if i % 97 == 0:
            r2 = M64
        if i % 89 == 0:
            r2 = 0
        rw = 1 if sm64_at(seed, 4 * i + 3) % 10 else 0
        ops[i] = (tid, r1, r2, rw)
        end = (r2 + HW) & M64
        hot = range(HW) if end >= r2 else range(0)
        if rw:
            for j in hot:
                x = ((r2 + j) & M64) % HR
                st[x] = (st[x] + 1) & M64
            s, b = 0, (r1 * tid) & M64
            for _ in range(CW):
                x = b % (words - HR) + HR
                b = (b + r2) & M64
                s = (s + st[x]) & M64
                st[x] = (st[x] + 1) & M64
            resp.append(s)
        else:
            for j in hot:
                st[((r2 + j) & M64) % HR] = tid
            b = (r1 * tid) & M64
            for _ in range(CW):
                st[b % (words - HR) + HR] = tid
                b = (b + r2) & M64
            resp.append(0)
    reads = np.zeros((200, 3), np.uint64)
    rsum = []
    for i in range(200):
        tid, r1, r2 = i % 5, sm64_at(seed + 9, 2 * i), sm64_at(seed + 9, 2 * i + 1)
        reads[i] = (tid, r1, r2)
        end = (r2 + HW) & M64
        s = 0
        for j in (range(HW) if end >= r2 else range(0)):
            s = (s + st[((r2 + j) & M64) % HR]) & M64
        b = (r1 * tid) & M64
        for _ in range(CR):
            s = (s + st[b % (words - HR) + HR]) & M64
            b = (b + r2) & M64
        rsum.append(s)
    return dict(seed=seed, n=n, words=words, ops=ops, resp=np.array(resp, np.uint64), final=np.array(st, np.uint64),
                reads=reads, read_sums=np.array(rsum, np.uint64))


def main():
    np.savez_compressed(os.path.join(HERE, "hashmap_small.npz"), **hashmap_fixture(7, 4, 600, 900, 1500, 1000))
    np.savez_compressed(os.path.join(HERE, "hashmap_sparse.npz"), **hashmap_fixture(8, 2, 2000, 2000, 1 << 48, 100))
    np.savez_compressed(os.path.join(HERE, "stack_sequential.npz"), **stack_fixture(5, 4096, 1000, 0))
    np.savez_compressed(os.path.join(HERE, "stack_push_some.npz"), **stack_fixture(6, 2048, 0, 1))
    np.savez_compressed(os.path.join(HERE, "synthetic_small.npz"), **synth_fixture(4, 3000, 2000, [0, 1, 7, 63]))
    np.savez_compressed(os.path.join(HERE, "splitmix.npz"),
                        seed0=np.array([sm64_at(0, i) for i in range(16)], np.uint64),
                        seed_x=np.array([sm64_at(0x4E52475055310001, i) for i in range(16)], np.uint64),
                        uniform=np.array([uniform(1234, i, 10_000_000) for i in range(64)], np.uint64))
    print("wrote golden fixtures to", HERE)


if __name__ == "__main__":
    main()
