#!/usr/bin/env bash
# Mask generator with NCH interleaved word chains per wave: checksums (bit-identical masks across
# 1/2/4 chains and the ballot generator), timing, counters, GPU attention tests, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
rm -f gpurun_out/session.log
for r in 1 2; do
  for c in 1 2 4; do step mask_ch${c}_$r 120 env DTD_ATTN_MASK_CH=$c python -u scripts/bench_mask.py; done
done
step mask_ballot 120 env DTD_ATTN_MASK=0 python -u scripts/bench_mask.py
step mask_pmc_ch4 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/mask_pmc_ch4 -o run --output-format csv -- python scripts/bench_mask.py
step attn_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py
step ab 900 python -u scripts/ab.py base mask_ch1 --rounds 3
echo done
