#!/usr/bin/env bash
# Round 4 session 2c: hipGraph b4 with/without real RCCL collectives, fp32 reference-precision
# benches, RCCL kernels in the profile, and the graphed-collectives capture test (riskiest, last).
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step prof_force 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_force -o run --output-format csv -- python bench.py --force-collectives --steps 3 --warmup 2
step bench_f32_gemm 200 python scripts/bench_f32_gemm.py
step tests_zero_w2 400 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_parallel_gpu.py -k two_ranks
step bench_b4_graph_force 300 python bench.py --batch-size 4 --graph on --force-collectives --steps 50 --warmup 10
step bench_b4_graph 300 python bench.py --batch-size 4 --graph on --steps 50 --warmup 10
step bench_fp32_b32 400 python bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
step bench_fp32_b32_hand 400 env DTD_GEMM_F32=1 python bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
step bench_fp32_ref_b32 400 python bench.py --dtype fp32 --impl reference --batch-size 32 --steps 5 --warmup 2
step tests_graph_rccl 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_graph_gpu.py -k "rccl or mp_script"
echo done
