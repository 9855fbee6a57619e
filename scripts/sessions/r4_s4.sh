#!/usr/bin/env bash
# Round 4 session 4: fused one-kernel attention backward -- numerics first, then the kernel timing,
# whole-step A/B and a kernel profile.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step tests_attn_fused 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py -k fused
grep -q "passed" gpurun_out/tests_attn_fused.log && ! grep -q "failed" gpurun_out/tests_attn_fused.log || { echo "fused tests did not pass; stopping"; exit 0; }
step bench_attn 200 env B=256 python scripts/bench_attn.py 3,2,3 fused 3,2,3 fused
step bench_fused 300 env DTD_ATTN_BWD=fused python bench.py
step bench_split 300 python bench.py
step prof_fused 400 env DTD_ATTN_BWD=fused rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run --output-format csv -- python bench.py --steps 3 --warmup 2
step tests_attn_all 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py
echo done
