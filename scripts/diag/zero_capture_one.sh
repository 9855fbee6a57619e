# one ZeRO capture variant with the Python fault handler and HIP runtime error logging
mkdir -p gpurun_out
MASTER_ADDR=127.0.0.1 MASTER_PORT=29811 DTD_ZERO_ALLOW_CAPTURE=1 AMD_LOG_LEVEL=2 timeout -k 10 120 python -X faulthandler scripts/diag/zero_capture_bisect.py --child s1_fwd_bwd_only > gpurun_out/zc_one.log 2>&1
echo "rc=$?"
grep -v "^\s*$" gpurun_out/zc_one.log | grep -iE "error|fail|capture|hipStream|Fatal|File \"/" | head -40
