#!/usr/bin/env bash
# Per-node prerequisites (reference: scripts/worker-prereqs.sh installed pdsh + ninja for DeepSpeed).
# Here nothing is installed: the launcher needs only ssh + python, and the HIP kernels are built
# in-tree for gfx950 with hipcc.  The script checks the toolchain and the GPUs, then builds.
set -euo pipefail
cd "$(dirname "$0")/../.."
command -v hipcc >/dev/null || { echo "hipcc not found (ROCm missing?)"; exit 1; }
python -c "import torch; assert torch.version.hip, 'torch is not a ROCm build'; print('torch', torch.__version__, 'hip', torch.version.hip)"
python -c "import torch; n = torch.cuda.device_count(); print('visible GPUs:', n); assert n > 0"
python -c "import __graft_entry__ as g; g.build()"
echo "worker ready: $(hostname)"
