#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that
# crashes, aborts or times out (rc >= 2 and not a plain test failure), as the pool's
# rules require.  Usage: tools/gpu_steps.sh "name|seconds|command" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/steps
mkdir -p $O
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name (limit ${secs}s): $cmd"
  ( cd $R && timeout -k 10 $secs bash -c "$cmd" ) > $O/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -6 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
