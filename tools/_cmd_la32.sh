export TMPDIR=/tmp RDQ_EVIDENCE_DIR=gpurun_out/r4/la32
tools/gpu_steps.sh gpurun_out/r4/la32 \
 "off|300|python -u tools/conv3_threshold_ab.py --precision fp32 --B 344 100 25 --fused-la-f32 off" \
 "auto|300|python -u tools/conv3_threshold_ab.py --precision fp32 --B 344 100 25 --fused-la-f32 auto"
