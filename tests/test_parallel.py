"""Multi-replica NR rounds across processes: write segments all-gathered,
every replica replays the identical global log, reads stay local, Put responses only at the
origin. Runs tests/dist_worker.py once per rank over gloo on 127.0.0.1."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(world, backend, timeout=180, extra=()):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), "--backend", backend,
                                       *extra], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            outs.append((p.returncode, o, e))
    except subprocess.TimeoutExpired:
        # name where each rank stalled (dist_worker prints its phases to stderr)
        for p in procs:
            p.kill()
        tails = [p.communicate()[1][-1500:] for p in procs]
        pytest.fail(f"ranks still running after {timeout} s; stderr tails:\n" +
                    "\n".join(f"--- rank {r}:\n{t}" for r, t in enumerate(tails)))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res = []
    for rc, o, e in outs:
        assert rc == 0, f"rank failed rc={rc}\nstdout:\n{o}\nstderr:\n{e[-3000:]}"
        res.append(json.loads(o.strip().splitlines()[-1]))
    assert all(r["ok"] for r in res)
    assert len({tuple(r["digest"]) for r in res}) == 1
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_replicated_rounds_gloo_cpu(world):
    run_ranks(world, "cpu")


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_rounds_gloo_cpu(world):
    """cnr-style key partitions: answers equal the NR replay, partitions add up."""
    run_ranks(world, "cpu", extra=("--mode", "partitioned", "--rounds", "4"))


@pytest.mark.gpu
def test_partitioned_rounds_gloo_gpu():
    run_ranks(2, "gpu", timeout=110, extra=("--mode", "partitioned"))


@pytest.mark.gpu
def test_replicated_rounds_gloo_gpu():
    # two replicas (two processes) on the box's one GPU; exchange over gloo
    run_ranks(2, "gpu", timeout=110)
