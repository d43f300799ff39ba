#!/bin/bash
# Host-side gpurun wrapper: retries only when no box was obtained or it failed while being prepared
# (nothing ran, nothing charged), up to 40 attempts a minute apart.  Usage: tools/gpr.sh TIMEOUT 'cmd'
t=$1; shift
for attempt in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > /tmp/gpr_last.txt 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" /tmp/gpr_last.txt && ! grep -q "status=ok" /tmp/gpr_last.txt; then
    echo "[gpr] attempt $attempt: no box, retrying in 60 s"
    sleep 60
    continue
  fi
  grep -v "every call sends the whole tree" /tmp/gpr_last.txt | tail -4
  exit $rc
done
echo "[gpr] gave up after 40 attempts"
exit 3
