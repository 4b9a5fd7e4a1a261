export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/p25 \
 "prof|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r4/p25/prof -o run -- python3 tools/unet_prof.py --B 25 --precision fp32 --reps 10"
