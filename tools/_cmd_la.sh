export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/la \
 "tests|300|python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread -k 'linear_attention_bf16 or bf16_close'" \
 "unet344|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r4/la/prof344 -o run -- python3 tools/bench_configs4.py --unet-only --precision bf16"
