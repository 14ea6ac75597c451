"""The gfx950 code objects inside libnrgpu.so: every kernel fits its registers (no scratch).

A register spill turns a kernel's hot loop into scratch traffic; the compiler reports it only as
a remark. This reads the kernel descriptors' metadata from the built library (llvm-objdump
--offloading extracts the code objects, llvm-readelf --notes prints their metadata) and fails on
any kernel with a private segment.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "node-replication_amd", "lib", "libnrgpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(tmp_path):
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(LIB) and os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("library or LLVM tools absent")
    lib = tmp_path / "libnrgpu.so"
    shutil.copy(LIB, lib)  # extraction writes next to its input
    subprocess.run([objdump, "--offloading", str(lib)], cwd=tmp_path, capture_output=True, check=True)
    out = {}
    for f in sorted(os.listdir(tmp_path)):
        if not f.endswith("gfx950"):
            continue
        notes = subprocess.run([readelf, "--notes", str(tmp_path / f)], capture_output=True, text=True,
                               check=True).stdout
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
            if m and name:
                out[name] = int(m.group(1))
    return out


def test_no_kernel_spills(tmp_path):
    k = _kernels(tmp_path)
    assert any("hm_round_kernel" in n for n in k) and any("sy_bucket_kernel" in n for n in k)
    spilled = {n: b for n, b in k.items() if b}
    assert not spilled, "kernels with scratch (register spills): %s" % spilled
