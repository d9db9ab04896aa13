#!/bin/bash
# round 6: what bounds the DP fill at cohort shapes -- fill-only replays (BT2X_DP_ABLATE=1)
# of the one-lane and split fills with development builds that drop the traceback stores
# (nost), the reference-window loads (nowin) or both
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06e}
out=gpurun_out/${T}_fillab.log
: > $out
for v in main nost nowin both; do
	lib=omp-bowtie2-prime_amd/bt2x/variants/libbt2x_$v.so
	[ $v = main ] && lib=omp-bowtie2-prime_amd/bt2x/libbt2x.so
	echo "== variant $v" >> $out
	BT2X_LIB=$PWD/$lib timeout -k 10 400 python -u tools/dp_replay.py --slots 65536 --steps 3 \
		BT2X_DP_SPLIT=0,BT2X_DP_DUO=0,BT2X_DP_ABLATE=1 BT2X_DP_ABLATE=1 >> $out 2>&1
	rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -E "^== |^config" $out
