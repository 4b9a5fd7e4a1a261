#!/bin/bash
# A/B of the RED loop's side stream: unrestricted vs CU-masked to XCDs ${1:-5,6,7} (the XCDs a
# 5-shot persistent launch leaves to its padding blocks).  CU-bit -> XCD map, U-Net co-run, loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3; mkdir -p $O
X=${1:-5,6,7}
timeout -k 10 120 ./tools/probe/cumask_probe > $O/cumask.txt 2>&1 || exit $?
awk '{print $4}' $O/cumask.txt | sort | uniq -c | tr '\n' ' '; echo
for xs in "" "$X"; do
  RDQ_SIDE_XCDS=$xs timeout -k 10 300 python -u tools/unet_corun.py 5 >> $O/unet_corun_xcd.jsonl || exit $?
done
for xs in "" "$X" "" "$X"; do
  RDQ_SIDE_XCDS=$xs timeout -k 10 300 python -u tools/notebook_floor.py 30 >> $O/notebook_xcd.jsonl || exit $?
done
cat $O/unet_corun_xcd.jsonl $O/notebook_xcd.jsonl
