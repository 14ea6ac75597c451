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


def _run_bench(args, env_extra=None, timeout=120):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_world_size_mismatch_refused():
    """A launcher's WORLD_SIZE that disagrees with --gpus exits non-zero before any GPU call
    (the run used to log and bench WORLD_SIZE ranks under a --gpus N command)."""
    p = _run_bench(["--gpus", "8", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE=1 but --gpus=8" in p.stderr
    assert not p.stdout.strip()


def test_launcher_spawns_ranks_and_relays_rank0(bench, tmp_path):
    """`bench.py --gpus N` with no launcher starts N ranks with torch.distributed.run's env and
    relays rank 0's JSON line (a stand-in rank script, so no GPU is needed)."""
    script = tmp_path / "rank.py"
    script.write_text(
        "import json, os, sys\n"
        "if os.environ['RANK'] == '0':\n"
        "    print('noise'); print(json.dumps({k: os.environ[k] for k in\n"
        "        ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')} | {'argv': sys.argv[1:]}))\n")
    import argparse
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.launch_ranks(argparse.Namespace(gpus=3, deadline=60.0), ["--gpus", "3", "--x"], script=str(script))
    assert rc == 0
    line = json.loads(buf.getvalue().strip())
    assert line["RANK"] == "0" and line["WORLD_SIZE"] == "3" and line["MASTER_ADDR"] == "127.0.0.1"
    assert line["argv"] == ["--gpus", "3", "--x"]


def test_launcher_fails_when_a_rank_fails(bench, tmp_path):
    """One failing rank ends the run non-zero and stops the others (which would otherwise wait in
    a collective for it)."""
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1': sys.exit(7)\n"
                      "time.sleep(60)\n")
    import argparse
    import time

    t = time.monotonic()
    rc = bench.launch_ranks(argparse.Namespace(gpus=2, deadline=120.0), [], script=str(script))
    assert rc == 7
    assert time.monotonic() - t < 40


def test_launcher_without_gpu_exits_nonzero():
    """The real bench through its own launcher on a host without a GPU: every rank fails, so
    the run must fail rather than print a line."""
    p = _run_bench(["--gpus", "2", "--backend", "gloo", "--share-gpu", "--steps", "2", "--warmup", "1",
                    "--no-cpu-baseline", "--deadline", "100"], timeout=200)
    assert p.returncode != 0
    assert "exited with status" in p.stderr
    assert not p.stdout.strip()


def test_amdahl_model(bench):
    assert bench.amdahl_speedup(1, 10) == pytest.approx(1.0)
    assert bench.amdahl_speedup(8, 10) == pytest.approx(8 * 1.1 / 2.5)
    assert bench.amdahl_speedup(8, 100) == pytest.approx(1.0)


def test_stack_and_synth_cpu_baselines_go_through_nr(bench):
    """the stack and synthetic lines' cpu_baseline is the nr restatement (log + flat
    combining, one replica per NUMA node), with the sequential oracle only as a labelled point."""
    for out in (bench.stack_cpu_baseline(0.3, 20_000, 50_000), bench.synth_cpu_baseline(0.3, 20_000)):
        json.dumps(out)
        assert out["kind"] == "port" and out["value"] > 0 and "restatement of nr" in out["sample"]
        assert out["one_thread_nr"]["cores"] == 1 and out["one_thread_sequential"]["value"] > 0


def test_roofline_prefers_the_window(bench):
    """The line's kernel time is the steady-state window ((stop - start) / rounds between two stream
    events) when it was measured; the dispatch-bracketed average is reported beside it."""
    import argparse

    args = argparse.Namespace(timing_every=4, steps=400, workload="stack", ops_per_gpu=1_000_000, stack_init=50_000,
                              write_ratio=10, key_space=10_000_000, prefill=1 << 23, log2_slots=26, dist="uniform",
                              theta=0.99, scramble=False, gpus=1)
    r = bench.roofline("st_replay", 12_000_000, 100, 100 * 0.0175, args, None, win=(399, 399 * 0.0147))
    assert r["avg_launch_us"] == pytest.approx(14.7)
    assert r["bracketed_avg_launch_us"] == pytest.approx(17.5)
    assert r["achieved"] == pytest.approx(12e6 / 14.7e-6 / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["launches"] == 399 and r["bracketed_launches"] == 100
    # without a window (--no-kernel-timing has neither), the bracketed average stands in
    r2 = bench.roofline("st_replay", 12_000_000, 100, 100 * 0.0175, args, None)
    assert r2["avg_launch_us"] == pytest.approx(17.5)
