"""bench.py's CPU-side record (no GPU): the cpu_baseline object and the host topology it carries.

cpu_baseline runs the C++ restatement of nr (oracle/nr_cpu.cpp) on the host: the B1 stream on the
thread budget, BASELINE configs[0] (5M keys, prefill 2^22), and a 1-thread point. Here each leg
runs for a fraction of a second; the fields must be present and well-formed.
"""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench(orc):  # orc: the oracle library is built
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_cpu_baseline_record(bench):
    out = bench.cpu_baseline(0.3, 10, 1_000_000, 1 << 16)
    json.dumps(out)  # one JSON line
    assert out["kind"] == "port" and out["unit"] == "Mops/s"
    assert out["value"] > 0 and out["cores"] >= 1
    assert out["configs0"]["value"] > 0 and "configs[0]" in out["configs0"]["sample"]
    assert out["one_thread"]["cores"] == 1 and out["one_thread"]["value"] > 0
    host = out["host"]
    assert host["nproc"] >= 1 and "numa_nodes" in host


def test_watchdog_ends_a_stalled_process():
    """bench.py's whole-process deadline: a process stuck past --deadline exits with status 3 and
    names its rank and phase (what a rank blocked in a collective whose peer never came does)."""
    import subprocess
    import sys

    code = ("import importlib.util, time, sys; sys.path.insert(0, %r)\n"
            "spec = importlib.util.spec_from_file_location('b', %r); b = importlib.util.module_from_spec(spec)\n"
            "spec.loader.exec_module(b); b.WATCH.phase = 'timed region'; b.WATCH.arm(0.5); time.sleep(30)\n"
            % (ROOT, os.path.join(ROOT, "bench.py")))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env={**os.environ, "RANK": "5", "WORLD_SIZE": "8"})
    assert p.returncode == 3, p.stderr
    assert "rank 5 of 8 still in phase 'timed region'" in p.stderr
