#!/usr/bin/env bash
# Round-3 session-2 verification: full GPU suite (incl. the new zero_dp_training BERT graph test),
# smoke, bench x2, ZeRO-2 bench, the BERT ZeRO-2 script config, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
step bench_default2 300 python bench.py
step bench_zero2 300 python bench.py --zero-stage 2
step cfg_bert_base_zero2 300 python zero_dp_training.py --model-name bert-base-cased --stage 2 --batch-size 32 --training-steps 30 --quiet --no-memstats
step prof_default 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python bench.py --steps 5 --warmup 2
echo done
