# bench A/B: one bench run (as the driver runs it, without the CPU baseline and the
# other configs' legs) per ';'-separated argument set in ARGSETS (env assignments allowed
# before the bench arguments, e.g. "BT2X_STREAMS=2 --slots 262144")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r04x}
i=0
IFS=';' read -ra SETS <<< "${ARGSETS:-}"
for set in "${SETS[@]}"; do
  i=$((i+1))
  envs=(); args=()
  for t in $set; do case "$t" in *=*) envs+=("$t");; *) args+=("$t");; esac; done
  env "${envs[@]}" timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-legs --no-replay-whole "${args[@]}" \
    > gpurun_out/${TAG}_ab$i.json 2> gpurun_out/${TAG}_ab$i.err
  rc=$?; echo "[$i] $set rc=$rc"
  python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_ab$i.json').read().strip().splitlines()[-1])
e=d['end_to_end']; g=e.get('gpu',{}); s=e.get('stats',{})
print('  value',d['value'],'t_align',e['t_align_s'],'host_cpu_us',e.get('host_cpu_us_per_read'),'t_step',s.get('t_step'),'t_wait',s.get('t_wait'),'t_host',s.get('t_host'),'t_gather',s.get('t_gather'),'round_call',g.get('t_round_call'),'dp_call',g.get('t_dp_call'))
k=d.get('kernels',{}); r=d.get('roofline',{}); print('  dp_ms',k.get('dp_ms'),'seed_ms',k.get('seed_ms'),'resolve_ms',k.get('resolve_ms'),'frac',r.get('frac'),'dp_launches',k.get('launches',{}).get('dp'))
" || true
  [ $rc -eq 0 ] || exit $rc
done
