#!/bin/bash
# gpurun_wait.sh LOG TIMEOUT 'COMMAND': run COMMAND through gpurun; while the
# pool has no box free (gpurun exit 3, or a transient infrastructure status
# with nothing run and nothing charged) wait three minutes and ask again.  A
# command that ran -- whatever its outcome -- is never re-run.
log=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None" "$log"; then
    echo "[gpurun_wait] attempt $i: no box ($rc); waiting" >> "$log.wait"
    sleep 180
    continue
  fi
  exit $rc
done
exit 3
