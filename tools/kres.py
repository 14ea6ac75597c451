#!/usr/bin/env python3
"""Per-kernel resources of a built libnrgpu.so (VGPRs, SGPRs, LDS, scratch) from its gfx950 code
object metadata. Usage: tools/kres.py [path/to/libnrgpu.so] [name-substring ...]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    lib = args.pop(0) if args and args[0].endswith(".so") else os.path.join(ROOT, "node-replication_amd/lib/libnrgpu.so")
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(lib, os.path.join(d, "l.so"))
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", "l.so"], cwd=d, capture_output=True, check=True)
        for f in sorted(os.listdir(d)):
            if not f.endswith("gfx950"):
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(d, f)],
                                   capture_output=True, text=True, check=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, blk) or [None, "?"])[1]
                name = g("name")
                if args and not any(a in name for a in args):
                    continue
                print(f"{name[:60]:60s} vgpr {g('vgpr_count'):>4s} agpr {blk.split()[1] if blk.split() else '?':>3s} "
                      f"sgpr {g('sgpr_count'):>4s} lds {g('group_segment_fixed_size'):>6s} "
                      f"scratch {g('private_segment_fixed_size'):>4s} wg {g('max_flat_workgroup_size')}")


if __name__ == "__main__":
    main()
