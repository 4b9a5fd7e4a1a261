export TMPDIR=/tmp
tools/gpu_steps.sh gpurun_out/r4/p344f \
 "prof|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r4/p344f/prof -o run -- python3 tools/unet_prof.py --B 344 --precision fp32 --reps 3"
