#!/bin/bash
# gpurun with queueing: when the pool has no free box (nothing ran, nothing
# charged) wait and submit again; any other outcome is returned as is.
#   scripts/gpurun_q.sh TIMEOUT 'command'
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > /tmp/gpurun_q.$$ 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_q.$$; then
    sleep 150
    continue
  fi
  cat /tmp/gpurun_q.$$
  rm -f /tmp/gpurun_q.$$
  exit $rc
done
cat /tmp/gpurun_q.$$
exit 3
