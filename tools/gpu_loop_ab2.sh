set -o pipefail
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_loop_parity.py tests/test_gpu_loop.py tests/test_gpu_sharding.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
for i in 1 2; do timeout -k 10 300 python -u -c "
import sys, os, torch, argparse; sys.path.insert(0, 'red-diffeq_amd'); sys.path.insert(0, '.')
import bench
a = argparse.Namespace(nt=1000, steps=30, warmup=3)
dev = torch.device('cuda')
print('notebook (5 shots) ms/iter', bench.red_loop_wallclock(dev, a, ns=5, family='curvefault'), flush=True)
print('configs2 (32 shots) ms/iter', bench.red_loop_wallclock(dev, a, ns=32), flush=True)
" 2>&1 | grep -v amdgpu || exit 1; done
