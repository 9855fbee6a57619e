#!/usr/bin/env bash
# Round 5 session 10: full GPU suite on the round-5 tree; the RCCL-init experiment (verdict r4 item 6:
# code objects loaded eagerly instead of the pre-group warm-up); the capture crash under
# AMD_LOG_LEVEL=4 (verdict r4 item 5) LAST -- it segfaults, nothing runs on the GPU after it.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step ab_rccl_init 900 python -u scripts/ab.py fc fc_noprewarm fc_noprewarm_eagerload --rounds 3
echo "=== [capture_amdlog] $(date +%T)" | tee -a gpurun_out/session.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29655 AMD_LOG_LEVEL=4 timeout -k 10 120 python scripts/diag/capture_collectives.py --child side_stream_rs > gpurun_out/cap_amdlog.txt 2>&1
rc=$?
echo "capture rc=$rc" | tee -a gpurun_out/session.log
tail -n 3000 gpurun_out/cap_amdlog.txt > gpurun_out/cap_amdlog_tail.txt
grep -n "hipStreamEndCapture\|hipGraph\|ncclGroup\|ncclReduceScatter\|Segmentation\|signal" gpurun_out/cap_amdlog.txt | tail -n 200 > gpurun_out/cap_amdlog_grep.txt
rm -f gpurun_out/cap_amdlog.txt
echo done
