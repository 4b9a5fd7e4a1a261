export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/sg \
 "tests|400|python -u -m pytest tests/test_gpu_fwi.py -x -q --timeout 200 --timeout-method thread -k 'slice_groups or shot_groups or xcd_local or rows_per_wave or forward_bitexact'" \
 "unet344|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r4/sg/prof344 -o run -- python3 tools/bench_configs4.py --unet-only --precision bf16" \
 "bench|420|python -u bench.py"
