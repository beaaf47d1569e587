#!/bin/bash
# Run named steps on the GPU box, each under its own time limit; stop at the first step that
# crashes, faults or times out (exit codes other than 0/1).  Logs in gpurun_out/<name>.log.
set -u
mkdir -p gpurun_out
: > gpurun_out/status.txt
step() {
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name" | tee -a gpurun_out/status.txt
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/status.txt
  tail -n 5 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "stopping: $name exited with $rc" | tee -a gpurun_out/status.txt
    exit "$rc"
  fi
}
