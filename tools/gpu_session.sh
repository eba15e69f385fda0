#!/bin/bash
# One GPU-box session (gpurun) from a plan file: each line "<seconds> <name> <command...>" runs
# under its own `timeout -k 10`, output to gpurun_out/<name>.log.  A step that fails normally
# (exit 1-5: test failures, usage errors) does not stop the session; a time limit, abort or crash
# (exit >= 124, or a signal) ends it, and nothing further touches the GPU.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_session.sh tools/plans/<plan>.txt'
PLAN=${1:?plan file}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
while read -r secs name cmd; do
  [[ -z "$secs" || "$secs" == \#* ]] && continue
  echo "== $(date +%T) $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $(date +%T) $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  if (( rc >= 124 )); then
    echo "== stopping: $name ended abnormally (rc $rc)"
    exit "$rc"
  fi
done < "$PLAN"
echo "== session done"
