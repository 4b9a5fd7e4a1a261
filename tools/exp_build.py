"""Timing-only experiment builds of the HIP library (never shipped): apply textual edits to a copy of
csrc/fwi.hip and link it with the current unet.o / loop.o into red-diffeq_amd/lib_exp/lib<name>.so;
select one at run time with RDQ_HIP_LIB.  The product source stays unchanged.
python tools/exp_build.py <name> '<old>' '<new>' ['<old>' '<new>' ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "red-diffeq_amd")
name, edits = sys.argv[1], sys.argv[2:]
src = open(os.path.join(PKG, "csrc", "fwi.hip")).read()
for old, new in zip(edits[::2], edits[1::2]):
    n = src.count(old)
    if n == 0:
        sys.exit(f"edit not found: {old!r}")
    src = src.replace(old, new)
os.makedirs("/tmp/exp", exist_ok=True)
hip = f"/tmp/exp/fwi_{name}.hip"
open(hip, "w").write(src)
obj = f"/tmp/exp/fwi_{name}.o"
flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"),
         "-I" + os.path.join(PKG, "csrc"), "-ffp-contract=off", "-fno-slp-vectorize"]
subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", "-o", obj, hip])
out = os.path.join(PKG, "lib_exp", f"lib{name}.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", out, obj,
                       os.path.join(PKG, "build", "unet.o"), os.path.join(PKG, "build", "loop.o")])
print(out)
