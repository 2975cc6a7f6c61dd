#!/bin/bash
# Run GPU steps in order on the box; each step "name|seconds|command" under its own
# timeout.  A step that exits 0 or 1 (tests failed, ran to the end) lets the next one run;
# a timeout (124/137), abort (134), segfault (139) or any other status stops the call.
# Output: gpurun_out/<name>.log per step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
