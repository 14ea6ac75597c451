"""Throughput of the native flat combiner (nrg_combiner_*) with many client threads.

B1's table and stream on one MI355X (2^26 slots, prefill [0, 2^23) -> k+1, keys uniform over
10M): each client thread loops on synchronous calls of B ops -- one call in ten a Put batch
(execute_mut), the others Get batches (execute) -- for a fixed time. Prints ops/s, GPU rounds
and ops per round for each (threads, B). Usage: python microbench/combiner.py [seconds]
"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "node-replication_amd"))
import nrgpu  # noqa: E402
from nrgpu import _lib as L  # noqa: E402

SECS = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
KEYS = 10_000_000


def run(threads, batch):
    dev = nrgpu.DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=26, max_batch=1 << 16, max_reads=1 << 16)
    dev.hm_prefill_range(1 << 23, 1)
    comb = nrgpu.Combiner(dev, threads)
    counts = [0] * threads
    stop = threading.Event()

    def client(i):
        tok = comb.register()
        rng = np.random.default_rng(1000 + i)
        c = 0
        n = 0
        while not stop.is_set():
            keys = rng.integers(0, KEYS, batch, dtype=np.uint64)
            if c % 10 == 0:
                comb.put(tok, keys, keys + 7)
            else:
                comb.get(tok, keys)
            c += 1
            n += batch
        counts[i] = n

    th = [threading.Thread(target=client, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    time.sleep(SECS)
    stop.set()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    rounds, ops = comb.stats()
    comb.close()
    dev.close()
    tot = sum(counts)
    print(f"threads {threads:4d} ops/call {batch:3d}: {tot / dt / 1e6:8.3f} Mops/s  rounds {rounds:7d}  "
          f"ops/round {ops / max(rounds, 1):7.1f}  round rate {rounds / dt / 1e3:6.1f} k/s", flush=True)


for t, b in [(8, 1), (8, 32), (64, 1), (64, 32), (256, 32)]:
    run(t, b)
