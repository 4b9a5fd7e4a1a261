export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/laf \
 "tests|300|python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread" \
 "b25|300|rocprofv3 --kernel-trace -d gpurun_out/r4/laf/prof -o run -- python3 tools/unet_prof.py --B 25 --precision fp32 --reps 5" \
 "b1|300|python3 tools/unet_bench.py"
