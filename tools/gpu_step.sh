#!/bin/bash
# Run GPU steps in order; stop at the first step that faulted, aborted, segfaulted or
# timed out (exit 124/134/137/139 or negative signal codes).  Ordinary failures (1, 2)
# let later steps run.  Usage: tools/gpu_step.sh "<name>:<seconds>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
overall=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== step $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== step $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    1|2|3|4|5) overall=1 ;;
    *) echo "=== step $name ended abnormally (rc=$rc); stopping"; exit $rc ;;
  esac
done
exit $overall
