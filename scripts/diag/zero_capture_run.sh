mkdir -p gpurun_out && timeout -k 10 500 python scripts/diag/zero_capture_bisect.py > gpurun_out/zero_capture2.log 2>&1; grep "^{" gpurun_out/zero_capture2.log | cut -c1-300
