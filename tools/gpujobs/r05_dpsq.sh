#!/bin/bash
# SQ / SQC counters of the DP fill alone (BT2X_DP_ABLATE=1) at cohort shapes, one-lane fill
# (BT2X_DP_DUO=0) and duo fill, each counter set its own rocprofv3 pass
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05e}
timeout -k 10 400 python -u tools/dp_replay.py --slots 65536 --steps 1 "" > gpurun_out/${TAG}_prep.log 2>&1
rc=$?; echo "prep rc=$rc"; grep -E "^config|launches" gpurun_out/${TAG}_prep.log; [ $rc -eq 0 ] || exit $rc
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"
P3="SQC_ICACHE_HITS SQC_ICACHE_MISSES"
for duo in 0 1; do
  for k in 1 2 3; do
    eval PM=\$P$k
    timeout -s KILL 240 rocprofv3 --pmc $PM --kernel-trace --output-format csv -d gpurun_out/${TAG}_d${duo}_p$k -o run -- python3 tools/dp_replay.py --slots 65536 --steps 1 BT2X_DP_ABLATE=1,BT2X_DP_DUO=$duo > gpurun_out/${TAG}_d${duo}_p$k.log 2>&1
    rc=$?; echo "duo=$duo pass $k rc=$rc"; grep -E "^config" gpurun_out/${TAG}_d${duo}_p$k.log
    [ $rc -eq 0 ] || exit $rc
  done
done
