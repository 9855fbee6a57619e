#!/usr/bin/env bash
# Memory-efficient / prefetching LayerNorm backward (tests, kernel timings, whole-step bench),
# world-1 replicated ZeRO layout (GPU tests, bloom-560m stages with graphs), GEMM PMC counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step ln_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm" -x -q --timeout 120 --timeout-method thread
step bench_ln 300 python scripts/bench_ln.py
step bench_default 300 python bench.py
step bench_ln_z 300 env DTD_LN_MEMEFF=0 python bench.py
step bench_ln_pf 300 env DTD_LN_BWD_PREFETCH=1 python bench.py
step pytest_zero 600 python -u -m pytest tests/test_parallel_gpu.py tests/test_graph_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step zero_bloom_s2_graph 400 python zero_dp_training.py --stage 2 --training-steps 60 --no-memstats --quiet
step zero_bloom_s2_eager 400 python zero_dp_training.py --stage 2 --training-steps 60 --no-memstats --quiet --graph off
step zero_bloom_s3_graph 400 python zero_dp_training.py --stage 3 --training-steps 60 --no-memstats --quiet
step zero_bloom_s1_graph 400 python zero_dp_training.py --stage 1 --training-steps 60 --no-memstats --quiet
step pmc_a 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/gp_a -o run --output-format csv -- python scripts/gemm_pmc_probe.py
step pmc_b 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES -d gpurun_out/gp_b -o run --output-format csv -- python scripts/gemm_pmc_probe.py
step pmc_c 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT FETCH_SIZE -d gpurun_out/gp_c -o run --output-format csv -- python scripts/gemm_pmc_probe.py
step summarize 60 python scripts/gemm_pmc_probe.py summarize gpurun_out/gp_a/run_counter_collection.csv gpurun_out/gp_b/run_counter_collection.csv gpurun_out/gp_c/run_counter_collection.csv
echo done
