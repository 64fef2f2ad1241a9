#!/bin/bash
# Build (here) / run (GPU box) the potrfTile micro-benchmark and its phase cuts.
# bash scripts/ubench_ptile.sh build [extra flags]  |  bash scripts/ubench_ptile.sh run
cd "$(dirname "$0")/.."
if [ "$1" = build ]; then
  for n in 0 1; do
    f=""; [ $n -gt 0 ] && f="-DOKG_POTRF_STOP=$n"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include $f $2 -DOKG_TAG="\"stop$n\"" scripts/ubench_ptile.hip -o scripts/ubench_ptile_$n &
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DOKG_SWEEP_TRACE $2 -DOKG_TAG="\"trace\"" scripts/ubench_ptile.hip -o scripts/ubench_ptile_T &
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -DOKG_SWEEP_TRACE -DOKG_SWEEP_SOLO $2 -DOKG_TAG="\"solo\"" scripts/ubench_ptile.hip -o scripts/ubench_ptile_S &
  wait
else
  timeout -k 5 60 scripts/ubench_ptile_T || exit 1
  timeout -k 5 60 scripts/ubench_ptile_S || exit 1
  for n in 0 1; do timeout -k 5 60 scripts/ubench_ptile_$n || exit 1; done
fi
