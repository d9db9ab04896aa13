timeout -k 10 900 python -u tools/gpujobs/genome_probe.py 3100 > gpurun_out/r03_probe.log 2>&1; echo rc=$?; tail -20 gpurun_out/r03_probe.log
