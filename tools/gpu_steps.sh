#!/bin/bash
# Run GPU steps in order, each already wrapped in its own `timeout -k 10 N`.  A step that passes (0) or whose tests
# fail (1) lets the next one run; anything else (a fault, an abort, a time limit) ends the call there.
for step in "$@"; do
  echo "=== $(date +%T) $step"
  bash -c "$step"
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
