#!/usr/bin/env bash
# Round 6: validation after the stage-3 bucket aliasing and the K-split LM-head input gradient --
# full GPU suite, smoke, driver bench command, the reference's default ZeRO configs (bloom-560m b1,
# stages 0-3) and an after-profile of the stage-3 step.
cd "${GRAFT_REPO_ROOT}"
source scripts/gpu_step.sh
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
R="${GRAFT_REPO_ROOT}"
step gpu_suite 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')"
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
for st in 0 1 2 3; do
  MASTER_PORT=2933$st step bloom_z${st} 300 python zero_dp_training.py --stage $st --quiet --no-memstats
done
MASTER_PORT=29339 DTD_HEAD_SPLITK=0 step bloom_z3_sk0 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
MASTER_PORT=29338 step bloom_z3_b 300 python zero_dp_training.py --stage 3 --quiet --no-memstats
cd /tmp
MASTER_PORT=29337 step bloom_z3_prof_after 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/bloomprof_after" -o bloom -- python3 "$R/zero_dp_training.py" --stage 3 --quiet --no-memstats --training-steps 200
echo done
