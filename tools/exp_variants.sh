#!/bin/bash
# Build timing-experiment variants of the FWI library (compile-time knobs; the RDQ_EXP_* knockouts
# give WRONG results; never used by tests or the product): lib/exp/<name>.so.  Run on the GPU with
# RDQ_EXP_LIB=<name>.so (tools/exp_run.sh).
cd "$(dirname "$0")/../red-diffeq_amd"
mkdir -p lib/exp build/exp
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -ffp-contract=off -fno-slp-vectorize"
build() {  # name, defines
  /opt/rocm/bin/hipcc $FL $2 -c -o build/exp/$1.o csrc/fwi.hip &&
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/exp/$1.so build/exp/$1.o build/unet.o build/loop.o
}


build noload "-DRDQ_EXP_NOPLOAD=1" &
build noinepoch "-DRDQ_EXP_NOINEPOCH=1" &
wait
ls -la lib/exp
