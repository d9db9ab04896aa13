# DP replay at cohort shapes under rocprofv3: instruction-cache and issue counters of the
# fill alone (BT2X_DP_ABLATE=1) and of the default fused kernel (fill + walks)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dp_replay.py --slots 65536 --steps 1 "" > gpurun_out/dpic_prep.log 2>&1
rc=$?; echo "prep rc=$rc"; grep -E "config|launches" gpurun_out/dpic_prep.log
[ $rc -eq 0 ] || exit $rc
PMC="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY"
for cfg in BT2X_DP_ABLATE=1 BT2X_DP_NONE=0; do
  env $cfg true
  export $cfg
  timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/dpic_$cfg -o run -- python3 tools/dp_replay.py --slots 65536 --steps 1 "" > gpurun_out/dpic_$cfg.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; grep -E "config" gpurun_out/dpic_$cfg.log
  unset ${cfg%%=*}
  [ $rc -eq 0 ] || exit $rc
done
