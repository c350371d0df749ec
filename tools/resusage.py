#!/usr/bin/env python3
"""Register / spill / occupancy table of every kernel in one source (analysis aid):
    python3 tools/resusage.py phoneme_contrast_amd/csrc/conv_wino.hip [extra hipcc flags]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Iinclude", "-munsafe-fp-atomics",
       "-fno-slp-vectorize", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:] + ["-c", sys.argv[1], "-o",
                                                                                        "/tmp/resusage.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
        continue
    k, _, v = t.partition(":")
    if cur is not None:
        cur[k.strip()] = v.strip()
for r in rows:
    g = r.get
    print(f"{g('VGPRs', '?'):>4}v {g('AGPRs', '?'):>3}a spill v{g('VGPRs Spill', '?')} s{g('SGPRs Spill', '?')} "
          f"occ {g('Occupancy [waves/SIMD]', '?')} lds {g('LDS Size [bytes/block]', '?')}  {r['name'][:140]}")
