"""Diagnostic: one client thread through the combiner's round server, with a watchdog that
prints the server's words (Combiner.probe) if a call does not return. Usage: python microbench/serve_debug.py"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "node-replication_amd"))
import nrgpu  # noqa: E402

dev = nrgpu.DeviceReplica(nrgpu._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=4096, max_reads=4096)
dev.hm_prefill_range(100, 1)
comb = nrgpu.Combiner(dev, 2)
done = []


def client():
    tok = comb.register()
    for it in range(20):
        prev, some = comb.put(tok, [5, 500 + it], [7, 8])
        got, found = comb.get(tok, [5, 1, 99999])
        done.append((it, list(some), list(got), list(found)))


t = threading.Thread(target=client, daemon=True)
t.start()
for _ in range(30):
    time.sleep(0.1)
    print("probe", comb.probe(), "calls done", len(done), flush=True)
    if not t.is_alive():
        break
print("last", done[-1] if done else None, flush=True)
if t.is_alive():
    print("HUNG", comb.probe(), flush=True)
    os._exit(1)
comb.close()
print("closed ok", flush=True)
