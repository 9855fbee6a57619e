#!/usr/bin/env bash
# Prepare every node of a cluster inventory for multi-node runs (reference: scripts/generate-keys.sh,
# scripts/worker-prereqs.sh).
#   1. render hostfile / ssh_config / .dtd_env from the inventory (launch/cluster.py)
#   2. create a cluster key pair (once) and install it on every worker, so workers can ssh each other
#      (the launcher's ssh fan-out runs from any node)
#   3. copy the repo + rendered files to each worker and run worker-prereqs.sh there (builds the
#      gfx950 kernels in-tree and checks ROCm / RCCL / the GPUs)
# Workers are prepared in parallel; the script fails if any worker fails.
#
#   scripts/cluster/bootstrap-workers.sh infra/mi355x_cluster.example.yaml [remote_dir]
set -euo pipefail
INV=${1:?usage: bootstrap-workers.sh INVENTORY [REMOTE_DIR]}
REMOTE_DIR=${2:-dtd}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/cluster"
python -m distributed_training_and_deepspeed_amd.launch.cluster "$INV" --out-dir "$OUT"
KEY=$(python - "$INV" <<'PY'
import os, sys
from distributed_training_and_deepspeed_amd.launch.cluster import Cluster
print(os.path.expanduser(Cluster.load(sys.argv[1]).ssh_key))
PY
)
[ -f "$KEY" ] || ssh-keygen -t ed25519 -N "" -f "$KEY" -C dtd-cluster
HOSTS=$(awk '{print $1}' "$OUT/hostfile")

setup_worker() {
  local h=$1
  ssh -F "$OUT/ssh_config" "$h" "mkdir -p ~/.ssh && chmod 700 ~/.ssh"
  scp -F "$OUT/ssh_config" -q "$KEY" "$KEY.pub" "$h:.ssh/"
  ssh -F "$OUT/ssh_config" "$h" "cat ~/.ssh/$(basename "$KEY").pub >> ~/.ssh/authorized_keys"
  scp -F "$OUT/ssh_config" -q "$OUT/ssh_config" "$h:.ssh/config"
  rsync -a --delete --exclude .git --exclude gpurun_out -e "ssh -F $OUT/ssh_config" "$ROOT/" "$h:$REMOTE_DIR/"
  ssh -F "$OUT/ssh_config" "$h" "cd $REMOTE_DIR && bash scripts/cluster/worker-prereqs.sh"
}

pids=()
for h in $HOSTS; do
  setup_worker "$h" > "$OUT/bootstrap-$h.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
[ $rc -eq 0 ] && echo "all workers ready" || echo "some workers failed: see $OUT/bootstrap-*.log"
exit $rc
