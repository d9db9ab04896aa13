#!/bin/bash
# round 5: DP walk variants (development builds under bt2x/variants, BT2X_LIB) replayed at
# the timed run's cohort shapes; the one-lane fill throughout (BT2X_DP_DUO=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05k}
out=gpurun_out/${TAG}_walkab.log
: > $out
for v in ${VARIANTS:-A B b8 b16 main}; do
	lib=omp-bowtie2-prime_amd/bt2x/variants/libbt2x_$v.so
	[ $v = main ] && lib=omp-bowtie2-prime_amd/bt2x/libbt2x.so
	echo "== variant $v" >> $out
	BT2X_LIB=$PWD/$lib timeout -k 10 600 python -u tools/dp_replay.py --slots 65536 --steps 3 BT2X_DP_DUO=0 ${DP_CFGS} >> $out 2>&1
	rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -E "^== |^config" $out
