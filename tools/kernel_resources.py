#!/usr/bin/env python3
"""Per-kernel register / spill / LDS / scratch figures of a built library, read from the gfx950 code
objects' metadata notes (no recompilation): python tools/kernel_resources.py [lib] [name-filter]."""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def main():
    lib = Path(sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else Path(__file__).resolve().parents[1]
               / "ccmmshadowratevar-code_amd/csrc/libccmm.so").resolve()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td) / lib.name
        tmp.write_bytes(lib.read_bytes())
        subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(tmp)], cwd=td, capture_output=True)
        rows = []
        for co in sorted(Path(td).glob("*amdgcn*gfx950")):
            notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], capture_output=True,
                                   text=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, blk) or [None, "?"])[1]
                name = g("name")
                if filt and filt not in name:
                    continue
                dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
                rows.append((dem.split("(")[0], g("vgpr_count"), g("vgpr_spill_count"), g("sgpr_spill_count"),
                             g("private_segment_fixed_size"), g("group_segment_fixed_size")))
    for r in rows:
        print("%-60s vgpr=%-4s vspill=%-4s sspill=%-4s scratch=%-6s lds=%s" % r)


if __name__ == "__main__":
    main()
