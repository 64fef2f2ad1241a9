#!/bin/bash
# (development helper, runs here, not on the GPU box; usage: scripts/gpurun_retry.sh OUTFILE gpurun-args...)
# local helper: run a gpurun command, retrying (up to 8 times, 150 s apart) only when no GPU slot/box
# was available (nothing ran, nothing charged)
OUT=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  rc=$?
  if grep -q "status=transient" $OUT || [ $rc -eq 3 ]; then sleep 150; continue; fi
  break
done
echo "rc=$rc" >> $OUT
