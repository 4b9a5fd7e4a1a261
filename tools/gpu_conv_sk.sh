#!/bin/bash
# stream-K conv: U-Net / op tests, then per-class conv rates with and without stream-K
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/conv_sk
mkdir -p $O
timeout -k 10 300 python -u -c "
import sys, json, torch; sys.path.insert(0, 'red-diffeq_amd'); sys.path.insert(0, '.')
import bench, red_diffeq.ops
print('streamk', json.dumps(bench.conv_class_rates(torch.device('cuda'))), flush=True)
" > $O/classes.log 2>&1 || exit $?
RDQ_NO_STREAMK=1 timeout -k 10 300 python -u -c "
import sys, json, torch; sys.path.insert(0, 'red-diffeq_amd'); sys.path.insert(0, '.')
import bench, red_diffeq.ops
print('tilegrid', json.dumps(bench.conv_class_rates(torch.device('cuda'))), flush=True)
" >> $O/classes.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_prof_b1.py 8 50 > $O/time.log 2>&1 || exit $?
RDQ_NO_STREAMK=1 timeout -k 10 300 python -u tools/unet_prof_b1.py 8 50 >> $O/time.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_prof_b1.py 1 200 >> $O/time.log 2>&1 || exit $?
grep -v amdgpu.ids $O/classes.log $O/time.log
