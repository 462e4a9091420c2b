timeout -k 10 60 tools/calib/launch_rate > gpurun_out/r05al/launch_rate.txt
