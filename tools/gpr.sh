#!/bin/bash
# gpurun with waiting for a free slot: retries only on exit code 3 (no box / slot free, nothing ran, nothing
# charged); any other exit (including a failed or timed-out GPU step) is returned as is.
# usage: tools/gpr.sh <timeout_s> '<command>'
T=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 90
done
exit 3
