cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in base noload noinepoch; do
  if [ $v = base ]; then unset RDQ_EXP_LIB; else export RDQ_EXP_LIB=$v.so; fi
  timeout -k 10 120 python tools/sweep_tb.py --only 4 --profile --reps 3 > gpurun_out/exp_$v.log 2>&1 || exit 1
  echo "== $v"; python -c "
import json,sys
d=json.loads(open('gpurun_out/exp_$v.log').read().strip().splitlines()[-1])
p=d['profile_us_per_wave']
print(d['fwd_ms'], d['adj_ms'], {k:(round(p[k]['wait_us']),round(p[k]['steps_us']),round(p[k]['publish_us']),round(p[k]['first_pass_us']),round(p[k]['passes'])) for k in p})"
done
