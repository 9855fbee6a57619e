#!/usr/bin/env bash
# Round 4 session 2: new kernels' tests (fp32 attention, gemm4), ZeRO world-2 on one GPU,
# per-tensor bf16 gradient bound, force-collectives and graphed-collectives benches, fp32 bench.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_attn_f32 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py -k f32
step tests_model 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "track or matches"
step tests_parallel 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_parallel_gpu.py
step gemm4_probe 400 python scripts/gemm4_probe.py
step bench_force 300 python bench.py --force-collectives
step bench_default 300 python bench.py
step bench_b4_graph_force 300 python bench.py --batch-size 4 --graph on --force-collectives --steps 50 --warmup 10
step bench_b4_graph 300 python bench.py --batch-size 4 --graph on --steps 50 --warmup 10
step bench_f32_gemm 200 python scripts/bench_f32_gemm.py
step bench_fp32_b32 400 python bench.py --dtype fp32 --batch-size 32 --steps 5 --warmup 2
step bench_fp32_ref_b32 400 python bench.py --dtype fp32 --impl reference --batch-size 32 --steps 5 --warmup 2
step prof_force 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_force -o run --output-format csv -- python bench.py --force-collectives --steps 3 --warmup 2
echo done
