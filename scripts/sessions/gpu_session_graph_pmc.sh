#!/usr/bin/env bash
# Graph-captured bench (b4 / b32, eager vs graph), attention PMC counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
step build 300 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench_b4 300 python bench.py --steps 20 --warmup 5 --batch-size 4
step bench_b4_graph 300 python bench.py --steps 20 --warmup 5 --batch-size 4 --graph on
step bench_b32 300 python bench.py --steps 20 --warmup 5 --batch-size 32
step bench_b32_graph 300 python bench.py --steps 20 --warmup 5 --batch-size 32 --graph on
export TMPDIR=/tmp
step list_counters 120 rocprofv3 --list-avail
step pmc_attn1 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc1 -o run --output-format csv -- python scripts/bench_attn.py 3,2,3
step pmc_attn2 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc2 -o run --output-format csv -- python scripts/bench_attn.py 3,2,3
echo done
