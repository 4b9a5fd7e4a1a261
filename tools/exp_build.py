"""Timing-only experiment builds of the HIP library (never shipped): apply textual edits to a copy of
csrc/fwi.hip (or, with --src unet, csrc/unet.hip) and link it with the other current objects into
red-diffeq_amd/lib_exp/lib<name>.so; select one at run time with RDQ_HIP_LIB.  The product source stays
unchanged.
python tools/exp_build.py [--src fwi|unet] <name> '<old>' '<new>' ['<old>' '<new>' ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "red-diffeq_amd")
args = sys.argv[1:]
which = "fwi"
if args[0] == "--src":
    which, args = args[1], args[2:]
name, edits = args[0], args[1:]
src = open(os.path.join(PKG, "csrc", which + ".hip")).read()
for old, new in zip(edits[::2], edits[1::2]):
    n = src.count(old)
    if n == 0:
        sys.exit(f"edit not found: {old!r}")
    src = src.replace(old, new)
os.makedirs("/tmp/exp", exist_ok=True)
hip = f"/tmp/exp/{which}_{name}.hip"
open(hip, "w").write(src)
obj = f"/tmp/exp/{which}_{name}.o"
flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"),
         "-I" + os.path.join(PKG, "csrc")] + (["-ffp-contract=off", "-fno-slp-vectorize"] if which == "fwi" else [])
subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", "-o", obj, hip])
os.makedirs(os.path.join(PKG, "lib_exp"), exist_ok=True)
out = os.path.join(PKG, "lib_exp", f"lib{name}.so")
others = [os.path.join(PKG, "build", f"{o}.o") for o in ("fwi", "unet", "loop") if o != which]
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", out, obj, *others])
print(out)
