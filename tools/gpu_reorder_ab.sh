set -o pipefail
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 120 python -u tools/replay_host_time.py 2>&1 | grep -v amdgpu || exit 1
for i in 1 2; do
for v in "" 1; do RDQ_REG_FIRST=$v timeout -k 10 300 python -u -c "
import sys, os, torch, argparse; sys.path.insert(0, 'red-diffeq_amd'); sys.path.insert(0, '.')
import bench
a = argparse.Namespace(nt=1000, steps=30, warmup=3)
dev = torch.device('cuda')
tag = 'reg_first' if os.environ.get('RDQ_REG_FIRST') else 'fwd_first'
print(tag, 'notebook (5 shots) ms/iter', bench.red_loop_wallclock(dev, a, ns=5, family='curvefault'), flush=True)
print(tag, 'configs2 (32 shots) ms/iter', bench.red_loop_wallclock(dev, a, ns=32), flush=True)
" 2>&1 | grep -v amdgpu || exit 1; done; done
