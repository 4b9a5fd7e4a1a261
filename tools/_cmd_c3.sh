export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/st \
 "tests|300|python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread" \
 "new|300|rocprofv3 --kernel-trace -d gpurun_out/r4/st/new -o run -- python3 tools/bench_configs4.py --unet-only --precision bf16"
