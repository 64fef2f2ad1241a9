#!/bin/bash
# A/B of the batch graph's assembly on three streams (libokvisgpu.so) against two (lib_asm2.so):
# the default batched bench line twice each, then 256 windows per GPU.
# (the OKG_ASM_STREAMS switch lived in runtime.cpp for this A/B only; result: profiles/r06_asm_streams_ab.txt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06asm}; mkdir -p $OUT
AB_STEPS=20 AB_WARMUP=5 bash scripts/lib_ab.sh $(basename $OUT)_ab "base asm2 base asm2" | tee $OUT/ab.txt || exit 1
for lib in libokvisgpu.so lib_asm2.so libokvisgpu.so lib_asm2.so; do
  OKVISGPU_LIB=$PWD/okvis2-x_amd/$lib timeout -k 10 300 python bench.py --windows 256 --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib 256', round(d['value']), round(d['ms_per_step'],3))" | tee -a $OUT/w256.txt || exit 1
done
