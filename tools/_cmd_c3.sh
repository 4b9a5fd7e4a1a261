export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/wd \
 "tests|300|python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread -k 'time_mlp or bf16 or stem'" \
 "new|300|rocprofv3 --kernel-trace -d gpurun_out/r4/wd/new -o run -- python3 tools/bench_configs4.py --unet-only --precision bf16"
