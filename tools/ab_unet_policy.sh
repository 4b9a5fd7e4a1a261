#!/bin/bash
# A/B of the conv's load cache policy (RDQ_CC_WPOL / RDQ_CC_APOL builds) on the notebook loop and the
# U-Net co-run: default lib vs lib/libred_diffeq_hip_{ntw,nta}.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3/pol; mkdir -p $O
L=red-diffeq_amd/lib
for rep in 1 2; do
  for v in "" ntw nta; do
    lib=$L/libred_diffeq_hip${v:+_$v}.so
    echo "{\"variant\": \"${v:-default}\"}" >> $O/corun.jsonl
    RDQ_HIP_LIB=$lib timeout -k 10 200 python -u tools/unet_corun.py 5 >> $O/corun.jsonl 2>/dev/null || exit $?
    echo "{\"variant\": \"${v:-default}\"}" >> $O/loop.jsonl
    RDQ_HIP_LIB=$lib timeout -k 10 200 python -u tools/notebook_floor.py 30 diffusion >> $O/loop.jsonl 2>/dev/null || exit $?
  done
done
cat $O/loop.jsonl
