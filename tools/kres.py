"""Kernel resource usage (VGPRs, spills, occupancy, LDS) of one HIP source for gfx950, from the
compiler's -Rpass-analysis=kernel-resource-usage remarks (no GPU needed).
usage: python tools/kres.py csrc/fwi.hip [name-regex]   (run from red-diffeq_amd/)"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
flags = ["-ffp-contract=off", "-fno-slp-vectorize"] if "fwi" in src else []
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I../include", *flags,
       "--cuda-device-only", "-c", "-o", "/tmp/kres.o", src, "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
for name, v in rows.items():
    if pat.search(name):
        print(f"{name[:70]:70s} vgpr {v.get('VGPRs')} vspill {v.get('VGPRs Spill')} sspill {v.get('SGPRs Spill')} "
              f"occ {v.get('Occupancy')} lds {v.get('LDS Size')}")
for line in out.splitlines():
    if "error" in line:
        print(line)
