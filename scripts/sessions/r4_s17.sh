#!/usr/bin/env bash
# Round 4 session 17: re-tune every hipBLASLt GEMM shape of the b256 step with TunableOp on the
# current build, then A/B the fresh table against the committed one (same box, interleaved)
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
  PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_new%d.csv step tune 1000 python bench.py --steps 2 --warmup 1
ls -la gpurun_out/tunableop_new0.csv
step ab_table 600 python scripts/ab.py base retuned --rounds 3
echo done
