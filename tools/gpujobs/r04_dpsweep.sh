# DP replay sweep at the timed run's cohort shapes (and optionally whole-file shapes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r04x}
for s in ${SLOTS:-65536}; do
timeout -k 10 500 python -u tools/dp_replay.py --slots $s "" ${DP_CFGS} > gpurun_out/${TAG}_dpreplay_$s.log 2>&1
rc=$?; echo "slots $s rc=$rc"; grep -E "config|launches|Error|error" gpurun_out/${TAG}_dpreplay_$s.log | tail -12
[ $rc -eq 0 ] || exit $rc
done
