mkdir -p gpurun_out/r05t && timeout -k 10 120 ./tools/calib/launch_rate > gpurun_out/r05t/launch_rate.txt 2>&1; cat gpurun_out/r05t/launch_rate.txt
