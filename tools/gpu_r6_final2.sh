#!/bin/bash
# Round 6 final evidence (tools/gpu_r6_final.sh) plus the bf16 halo conv's per-workgroup phase stamps
# (timing-only lib_exp/libc3prof.so from tools/exp_c3prof.py; tools/c3_phase.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/final2}
mkdir -p $O
bash tools/gpu_r6_final.sh $O || exit $?
RDQ_HIP_LIB=red-diffeq_amd/lib_exp/libc3prof.so timeout -k 10 200 python -u tools/c3_phase.py l72_3x3_64_64 l36_3x3_64_64 l9_3x3_512_512 \
    > $O/c3_phase.jsonl 2> $O/c3_phase.err || { echo "c3_phase rc=$?"; tail -5 $O/c3_phase.err; exit 1; }
cat $O/c3_phase.jsonl
