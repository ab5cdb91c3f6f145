#!/usr/bin/env python3
"""Print VGPR / AGPR / scratch / LDS / occupancy per kernel of libccmm (compiler view)."""
import re
import subprocess
from pathlib import Path

here = Path(__file__).resolve().parent
out = "".join(subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                              "-c", tu, "-o", "/tmp/_ccmm_ru.o", "-Rpass-analysis=kernel-resource-usage"],
                             cwd=here, capture_output=True, text=True).stderr
              for tu in ("ccmm_abi.hip", "ccmm_lag.hip", "ccmm_svpart.hip", "ccmm_big.hip",
                         "ccmm_bign.hip"))
rows, cur = [], None
pats = {"vgpr": r"VGPRs: (\d+)", "agpr": r"AGPRs: (\d+)", "scratch": r"ScratchSize \[bytes/lane\]: (\d+)",
        "lds": r"LDS Size \[bytes/block\]: (\d+)", "occ": r"Occupancy \[waves/SIMD\]: (\d+)"}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = {"name": name.split("(")[0]}
        rows.append(cur)
        continue
    for k, p in pats.items():
        m = re.search(p, line)
        if m and cur is not None:
            cur[k] = m.group(1)
for r in rows:
    print("%-40s vgpr=%-4s agpr=%-4s scratch=%-5s lds=%-6s occ=%s" % (
        r["name"], r.get("vgpr"), r.get("agpr"), r.get("scratch"), r.get("lds"), r.get("occ")))
