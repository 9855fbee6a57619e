#!/usr/bin/env bash
# Swizzled backward attention tiles (0 LDS bank conflicts): numerics, kernel timings new vs base,
# PMC counters, whole-step A/B; LayerNorm kernel timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step attn_tests 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_attn_new 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_attn_base 300 env B=256 DTD_KERNELS_SO=distributed_training_and_deepspeed_amd/ops/_dtd_kernels_base.so python scripts/bench_attn.py 3,2,3
step bench_attn_new2 300 env B=256 python scripts/bench_attn.py 3,2,3
step bench_attn_base2 300 env B=256 DTD_KERNELS_SO=distributed_training_and_deepspeed_amd/ops/_dtd_kernels_base.so python scripts/bench_attn.py 3,2,3
step attn_pmc 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU -d gpurun_out/attn_pmc -o run --output-format csv -- python scripts/bench_attn.py 3,2,3
step bench_ln 300 python scripts/bench_ln.py
step ab_attn 900 python scripts/ab.py base base_so --rounds 3
echo done
