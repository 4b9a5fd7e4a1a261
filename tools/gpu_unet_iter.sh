bash tools/gpu_unet_b1.sh && mkdir -p gpurun_out/conv_micro && timeout -k 10 300 python -u tools/conv_micro.py --B 1 8 > gpurun_out/conv_micro/time.jsonl 2>&1
