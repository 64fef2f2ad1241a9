#!/bin/bash
# A/B of the batch graph's gradient test beside the GN prep and the assembly (libokvisgpu.so)
# against after k_fgrad (lib_fgn0.so): the batched bench line twice each, 256 windows, then the
# (the OKG_FORKED_GRADNORM switch lived in runtime.cpp for this A/B only; result: profiles/r06_forked_gradnorm_ab.txt)
# solve-parity GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06fgnb}; mkdir -p $OUT
AB_STEPS=20 AB_WARMUP=5 bash scripts/lib_ab.sh $(basename $OUT)_ab "base fgn0 base fgn0" | tee $OUT/ab.txt || exit 1
for lib in libokvisgpu.so lib_fgn0.so libokvisgpu.so lib_fgn0.so; do
  OKVISGPU_LIB=$PWD/okvis2-x_amd/$lib timeout -k 10 300 python bench.py --windows 256 --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib 256', round(d['value']), round(d['ms_per_step'],3))" | tee -a $OUT/w256.txt || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; exit 1; }
tail -1 $OUT/pytest.txt
