set -o pipefail
cd "${GRAFT_REPO_ROOT}"
cp red-diffeq_amd/lib/libred_diffeq_hip.so red-diffeq_amd/lib/lib_new.so
for i in 1 2; do
  cp red-diffeq_amd/lib/lib_new.so red-diffeq_amd/lib/libred_diffeq_hip.so
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-loop --no-red --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('new', d['value'], d['phases_ms'])" || exit 1
  cp red-diffeq_amd/lib/lib_prev.so red-diffeq_amd/lib/libred_diffeq_hip.so
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-loop --no-red --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('prev', d['value'], d['phases_ms'])" || exit 1
done
