#!/usr/bin/env bash
# Multi-node ZeRO run over every node of the hostfile (reference: scripts/launch-multinode.sh).
# Differences on purpose: --model-name matches the script's flag (the
# reference's --model_name was silently ignored), and the master address is resolved here, on the
# launching node (the reference single-quoted $MASTER_ADDR so it expanded to empty remotely).
#
#   scripts/launch-multinode.sh [hostfile] [stage] [model]
set -euo pipefail
cd "$(dirname "$0")/.."
HOSTFILE=${1:-cluster/hostfile}
STAGE=${2:-2}
MODEL=${3:-facebook/opt-125m}
MASTER_ADDR=${MASTER_ADDR:-$(awk 'NF && $1 !~ /^#/ {print $1; exit}' "$HOSTFILE")}
exec python -m distributed_training_and_deepspeed_amd.launch.multinode --hostfile "$HOSTFILE" \
  --master-addr "$MASTER_ADDR" --master-port "${MASTER_PORT:-29500}" \
  zero_dp_training.py --stage="$STAGE" --model-name "$MODEL"
