#!/bin/bash
# RED loop A/B: default, no side-stream overlap, no XCD-local padding (tools/red_loop_ab.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/red_ab.jsonl
: > $O
timeout -k 10 200 python -u tools/red_loop_ab.py 20 >> $O 2> gpurun_out/red_ab.err || exit $?
RDQ_NO_OVERLAP=1 timeout -k 10 200 python -u tools/red_loop_ab.py 20 >> $O 2>> gpurun_out/red_ab.err || exit $?
RDQ_NO_XCD_LOCAL=1 timeout -k 10 200 python -u tools/red_loop_ab.py 20 >> $O 2>> gpurun_out/red_ab.err || exit $?
cat $O
