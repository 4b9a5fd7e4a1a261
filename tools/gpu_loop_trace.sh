#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/loop_trace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 -c "
import sys, torch, argparse; sys.path.insert(0, 'red-diffeq_amd'); sys.path.insert(0, '.')
import bench
a = argparse.Namespace(nt=1000, steps=4, warmup=2)
print(bench.red_loop_wallclock(torch.device('cuda'), a, ns=5, family='curvefault'))
" > $O/run.log 2>&1 || exit $?
python3 tools/loop_timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/timeline.txt || exit $?
cat $O/timeline.txt
