#!/usr/bin/env bash
# Run one GPU step under its own time limit, logging to gpurun_out/<name>.log.
# Usage: source scripts/gpu_step.sh; step NAME SECONDS cmd...
# A step that crashes (signal / abort / segfault / timeout) ends the whole session (exit 99):
# nothing more is started on the GPU after a fault.  Ordinary failures (rc 1-2, e.g. failing
# tests) are recorded and the session continues.
_GO="${GRAFT_REPO_ROOT:-$PWD}/gpurun_out"
mkdir -p "$_GO"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name="$1" secs="$2"; shift 2
  echo "=== [$name] $(date +%T) $*" | tee -a "$_GO/session.log"
  timeout -k 10 "$secs" "$@" > "$_GO/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc $(date +%T)" | tee -a "$_GO/session.log"
  tail -n 5 "$_GO/$name.log" | sed 's/^/    /' | tee -a "$_GO/session.log"
  if [ $rc -ge 3 ]; then
    echo "FATAL: step $name rc=$rc; stopping GPU session" | tee -a "$_GO/session.log"
    exit 99
  fi
  return 0
}
