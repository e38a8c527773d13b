#!/bin/bash
# Retry a gpurun call only while the pool answers 3 (no box / transient
# infrastructure failure: nothing ran, nothing charged).  Any other exit code
# (including a failure of the command itself) is final.
out=$1; shift
for attempt in 1 2 3 4 5 6 7 8; do
  timeout 1500 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > "$out" 2>&1
  rc=$?
  echo "attempt $attempt exit $rc" >> "$out.attempts"
  if [ $rc -ne 3 ]; then echo "exit $rc" >> "$out"; exit $rc; fi
  sleep 60
done
echo "exit 3 (gave up)" >> "$out"
