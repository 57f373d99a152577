#!/bin/bash
# Re-submit a gpurun call while the pool has no free box (exit 3: nothing ran,
# nothing charged); any other exit status -- success, a failed command, a
# refusal -- ends the loop at once.  Usage: gpurun_wait.sh <tries> <gpurun args...>
tries=$1; shift
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no box (try $i/$tries); waiting 150 s"
  sleep 150
done
exit 3
