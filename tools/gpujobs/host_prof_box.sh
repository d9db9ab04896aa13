# host-driver profile on the GPU box's CPUs (no GPU work): the replay harness
# (tests/cpp/test_e2e_oracle --host-timing: kernel results recorded by the CPU oracle, then
# replayed) under tools/sprof.c, 16 threads, cohorts of the timed run's size
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
gcc -O2 -shared -fPIC -o /tmp/sprof.so tools/sprof.c -ldl || exit 1
timeout -k 10 600 python3 -u tools/host_profile.py --mb 200 --reads 200000 -p 16 --slots 131072 > gpurun_out/hp_plain.log 2>&1
rc=$?; tail -4 gpurun_out/hp_plain.log; [ $rc -eq 0 ] || exit $rc
cd /tmp/bt2x_hostprof && SPROF_SKIP=1 SPROF_WAIT=1 SPROF_RAW=$GRAFT_REPO_ROOT/gpurun_out/hp_raw.txt SPROF_OUT=$GRAFT_REPO_ROOT/gpurun_out/hp_flat.txt LD_PRELOAD=/tmp/sprof.so $GRAFT_REPO_ROOT/tests/cpp/test_e2e_oracle g200000000 g200000000_r200000_L150.fq --host-timing --reps 4 -p 16 --slots 131072 --dpad 12 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/hp_timing.err
rc=$?; cd $GRAFT_REPO_ROOT; grep HOST_TIMING gpurun_out/hp_timing.err | tail -3
timeout -k 10 300 python3 tools/sprof_report.py gpurun_out/hp_raw.txt --top 40 > gpurun_out/hp_report.txt 2>&1
timeout -k 10 300 python3 tools/sprof_report.py gpurun_out/hp_raw.txt --top 30 --callers > gpurun_out/hp_callers.txt 2>&1
head -30 gpurun_out/hp_report.txt; exit $rc
