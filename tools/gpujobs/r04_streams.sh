# two contexts per aligner (one per cohort) vs one: the round/e2e GPU tests, then the bench
# as the driver runs it, with BT2X_STREAMS=2 (default) and =1, and the host prefetch off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r04x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_round.py tests/test_e2e.py tests/test_integration.py \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-"BT2X_STREAMS=2" "BT2X_STREAMS=1" "BT2X_HOST_PREFETCH=0"}; do
  env $cfg timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-legs --no-replay-whole ${BENCH_ARGS} > gpurun_out/${TAG}_bench_$cfg.json 2> gpurun_out/${TAG}_bench_$cfg.err
  rc=$?; echo "bench $cfg rc=$rc"; python3 -c "
import json,sys
d=json.loads(open('gpurun_out/${TAG}_bench_$cfg.json').read().strip().splitlines()[-1])
e=d['end_to_end']; g=e.get('gpu',{}); s=e.get('stats',{})
print('value',d['value'],'t_align',e['t_align_s'],'host_cpu_us',e.get('host_cpu_us_per_read'),'t_step',s.get('t_step'),'t_wait',s.get('t_wait'),'round_call',g.get('t_round_call'),'dp_call',g.get('t_dp_call'))
k=d.get('kernels',{}); print('dp_ms',k.get('dp_ms'),'seed_ms',k.get('seed_ms'),'resolve_ms',k.get('resolve_ms'),'round',k.get('round_sampling'))
" || true
  [ $rc -eq 0 ] || exit $rc
done
