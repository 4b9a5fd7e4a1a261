export TMPDIR=/tmp RDQ_EVIDENCE_DIR=gpurun_out/r4/final6
tools/gpu_steps.sh gpurun_out/r4/final6 \
 "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "profbench|900|rocprofv3 --kernel-trace --stats -d gpurun_out/r4/final6/prof -o bench -- python3 bench.py" \
 "bench|600|python -u bench.py"
