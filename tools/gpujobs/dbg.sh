timeout -k 10 300 python -u tools/gpujobs/dbg_i16.py > gpurun_out/r03_dbg.log 2>&1; echo rc=$?; tail -60 gpurun_out/r03_dbg.log
