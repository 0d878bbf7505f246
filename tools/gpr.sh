#!/bin/bash
# gpurun with retries on infrastructure transients only (refused before anything ran, nothing
# charged): no box / slot free, pool busy, or the client's back-off. A command that ran is never
# retried, whatever its exit status.
#   tools/gpr.sh OUTFILE [gpurun args...]
out=$1; shift
rc=1
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if grep -q "status=ok\|status=fail\|status=timeout\|status=killed" "$out"; then exit $rc; fi
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" "$out"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$out" | tail -1 | grep -o "[0-9]*")
    sleep $(( ${wait_s:-60} + 5 ))
    continue
  fi
  exit $rc
done
exit $rc
