export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/tl \
 "tl|400|rocprofv3 --kernel-trace -d gpurun_out/r4/tl/prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-loop --no-red --no-configs4 --no-cpu-baseline"
