cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
bash scripts/gpu_session_configs.sh
step cfg_gpt2m_ddp 300 python bench.py --model gpt2-medium --batch-size 32 --steps 10 --warmup 3
step cfg_gpt2m_zero3_bench 300 python bench.py --model gpt2-medium --zero-stage 3 --batch-size 32 --steps 10 --warmup 3
step cfg_opt125m 300 python bench.py --model opt-125m --batch-size 32 --steps 10 --warmup 3
step cfg_bloom_zero0 300 python zero_dp_training.py --stage 0 --batch-size 1 --training-steps 30 --quiet --no-memstats
echo done2
