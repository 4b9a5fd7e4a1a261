set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r5/u1
mkdir -p $O
timeout -k 10 300 python -u tools/unet_prof_b1.py 1 200 > $O/time.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/conv_micro.py --B 1 > $O/micro.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/unet_prof_b1.py 1 5 > $O/prof.log 2>&1 || exit $?
python3 tools/unet_timeline.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/timeline.txt || exit $?
cat $O/time.log $O/micro.log
