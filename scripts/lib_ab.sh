#!/bin/bash
# A/B of library builds (okvis2-x_amd/lib_NAME.so, scripts/build_variant.sh): single-window rate and
# the default batched bench value. Usage (via gpurun): bash scripts/lib_ab.sh TAG "base NAME1 NAME2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in $2; do
  # NAME or NAME+VAR=VALUE (the library of NAME run with that environment variable)
  n=${v%%+*}; ev=; [ "$n" != "$v" ] && ev=${v#*+}
  if [ "$n" = base ]; then lib=$PWD/okvis2-x_amd/libokvisgpu.so; else lib=$PWD/okvis2-x_amd/lib_$n.so; fi
  env $ev OKVISGPU_LIB=$lib timeout -k 10 120 python scripts/single_window.py 50 0 > $OUT/single_$v.txt 2>&1 || { cat $OUT/single_$v.txt; exit 1; }
  env $ev OKVISGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-latency ${PROFILE_FLAG---no-profile} --steps ${AB_STEPS:-10} --warmup ${AB_WARMUP:-3} > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v rc=$?"; tail -20 $OUT/bench_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1])
ks = ' '.join(f'{k} {v[\"ms\"]:.3f}' for k, v in sorted(d.get('kernels', {}).items()))
print('$v', open('$OUT/single_$v.txt').read().split(',')[0], '| batch', round(d['value']), 'ms/it', round(d['ms_per_step'],3), 'cost sum', repr(d['gather']['final_cost_sum']), '|', ks)
"
done
