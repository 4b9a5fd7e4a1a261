export TMPDIR=/tmp RDQ_EVIDENCE_DIR=gpurun_out/r4/full
tools/gpu_steps.sh gpurun_out/r4/full \
 "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench|600|python -u bench.py"
