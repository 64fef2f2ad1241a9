#!/bin/bash
# Local wrapper: rebuild (must succeed), then run scripts/gpu_check.sh TAG on the GPU box.
set -e
cd /root/repo
make -s -C okvis2-x_amd -j8 2>&1 | grep -E "error" && { echo "BUILD FAILED"; exit 1; }
make -s -C okvis2-x_amd 2>&1 | grep -q "error" && { echo "BUILD FAILED"; exit 1; }
timeout 1800 /usr/local/graft/bin/gpurun --timeout 1200 -- "bash scripts/gpu_check.sh $1" 2>&1 | tail -3 | cut -c1-250
python3 scripts/kstats.py gpurun_out/$1/prof/run_kernel_stats.csv ${2:-8}
