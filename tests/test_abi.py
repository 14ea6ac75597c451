"""C-ABI boundary checks that need no GPU: libnrgpu.so loads, exports every function that
include/*.h declares, and answers the non-compute queries (version, error strings, config
defaults, device count) without touching a device."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("nrgpu.h", "nrgpu_testing.h")]
DECL = re.compile(r"^\s*(?:const\s+)?(?:int|void|char|nrg_ctx)\s*\**\s*(nrg_\w+)\s*\(", re.M)


def declared():
    names = []
    for h in HEADERS:
        with open(h) as f:
            names += DECL.findall(f.read())
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    import nrgpu

    return nrgpu.load()


def test_header_parse_finds_the_abi():
    names = declared()
    for must in ("nrg_open", "nrg_close", "nrg_log_append", "nrg_log_exec", "nrg_hashmap_get",
                 "nrg_hashmap_round_segments_async", "nrg_stack_peek", "nrg_synth_read", "nrg_test_sort_pairs"):
        assert must in names
    for must in ("nrg_group_open", "nrg_group_join", "nrg_group_round_async", "nrg_group_replica"):
        assert must in names
    assert len(names) >= 50


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, f"declared in include/ but not exported by libnrgpu.so: {missing}"


def test_exports_are_c_linkage():
    # nm -D lists the dynamic symbols; every nrg_ export must be unmangled (extern "C")
    import subprocess

    so = os.path.join(ROOT, "node-replication_amd", "lib", "libnrgpu.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for n in declared():
        assert n in syms, n


def test_non_compute_queries(lib):
    from nrgpu import _lib as L

    assert lib.nrg_version().decode().endswith("gfx950")
    for code in range(0, -10, -1):
        assert lib.nrg_strerror(code)
    assert lib.nrg_device_count() >= 0
    cfg = L.Config()
    lib.nrg_config_default(C.byref(cfg), L.NRG_DS_HASHMAP)
    assert cfg.ds_kind == L.NRG_DS_HASHMAP and cfg.log2_slots == 26
    lib.nrg_config_default(C.byref(cfg), L.NRG_DS_SYNTHETIC)
    assert (cfg.synth_n, cfg.synth_cold_reads, cfg.synth_cold_writes, cfg.synth_hot_reads,
            cfg.synth_hot_writes) == (200000, 20, 5, 2, 1)


def test_null_and_bad_arguments_are_errors_not_crashes(lib):
    from nrgpu import _lib as L

    assert lib.nrg_close(None) == L.NRG_E_INVAL
    out = C.c_void_p()
    cfg = L.Config()
    lib.nrg_config_default(C.byref(cfg), 99)
    rc = lib.nrg_open(0, C.byref(cfg), C.byref(out))
    assert rc in (L.NRG_E_INVAL, L.NRG_E_NODEV)
    assert lib.nrg_sync(None) == L.NRG_E_INVAL


def test_scaleout_csv_format(tmp_path):
    """bench.py --csv writes the reference harness's scaleout_benchmarks.csv columns
    (benches/mkbench.rs:518-545), header once, one row per replica."""
    import csv
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    p = tmp_path / "scaleout_benchmarks.csv"
    bench.write_scaleout_csv(str(p), "nrhashmap-gpu", 2, 1_000_000, 10, 0.005)
    bench.write_scaleout_csv(str(p), "nrhashmap-gpu", 2, 1_000_000, 10, 0.005)
    rows = list(csv.reader(open(p)))
    assert rows[0] == ["name", "rs", "tm", "batch_size", "threads", "duration", "thread_id", "core_id",
                       "exp_time_in_sec", "iterations"]
    assert len(rows) == 5 and rows[1][6] == "0" and rows[2][6] == "1"
    assert int(rows[1][9]) == 2_000_000_000


def test_group_api_argument_checks(lib):
    """The RCCL group entry points reject bad arguments before touching RCCL or a device."""
    from nrgpu import _lib as L

    out = C.c_void_p()
    assert lib.nrg_group_close(None) == L.NRG_E_INVAL
    assert lib.nrg_group_sync(None) == L.NRG_E_INVAL
    assert lib.nrg_group_round_async(None, None, None) == L.NRG_E_INVAL
    assert lib.nrg_group_replica(None, 0) is None
    assert lib.nrg_group_join(None, None, 2, 0, C.byref(out)) == L.NRG_E_INVAL
    cfg = L.default_config(L.NRG_DS_HASHMAP)
    assert lib.nrg_group_open(None, 1, C.byref(cfg), C.byref(out)) == L.NRG_E_INVAL
    devs = (C.c_int * 1)(0)
    assert lib.nrg_group_open(devs, 0, C.byref(cfg), C.byref(out)) == L.NRG_E_INVAL
    assert lib.nrg_strerror(L.NRG_E_COMM).decode().startswith("RCCL")


def test_key_owner_matches_the_python_mirror(lib):
    """nrg_key_owner (the C ABI's partition function) == nrgpu.parallel.key_owner (numpy), and it
    spreads keys evenly over the partitions (SURVEY.md §8 f4 routing)."""
    import numpy as np

    from nrgpu.parallel import key_owner

    rng = np.random.default_rng(7)
    keys = np.concatenate([np.arange(2000, dtype=np.uint64), rng.integers(0, 2**64 - 1, 3000, dtype=np.uint64),
                           np.array([2**64 - 1, 2**63], dtype=np.uint64)])
    for parts in (1, 2, 3, 7, 8, 64):
        mine = key_owner(keys, parts)
        theirs = [lib.nrg_key_owner(C.c_uint64(int(k)), parts) for k in keys]
        assert mine.tolist() == theirs
        assert mine.min() >= 0 and mine.max() < parts
    counts = np.bincount(key_owner(np.arange(80000, dtype=np.uint64), 8), minlength=8)
    assert counts.min() > 0.9 * 10000 and counts.max() < 1.1 * 10000
    from nrgpu import _lib as L

    assert lib.nrg_group_partitioned_round(None, None) == L.NRG_E_INVAL
    assert lib.nrg_group_partitioned_round_async(None, None) == L.NRG_E_INVAL
    assert lib.nrg_group_partitioned_flush(None) == L.NRG_E_INVAL
    assert lib.nrg_hashmap_partition_async(None, None, 0, None, 0, 2, None, None, None, None, None) == L.NRG_E_INVAL
