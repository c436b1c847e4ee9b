#!/bin/bash
# Forward-only bench A/B on one box: default kernels vs an env variant (VARIANT_ENV, e.g.
# "SNVRAG_ATTN_V2=1"), alternated REPS times; prints ms/step and the kernel-class times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS="--steps ${BSTEPS:-5} --warmup 2 --cpu-baseline 0 --f32-leg 0 --train-steps 0"
for r in $(seq ${REPS:-2}); do
  for v in base alt; do
    if [ $v = base ]; then E=""; else E="$VARIANT_ENV"; fi
    env $E timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$v', d['ms_per_step'], 'attn', k['attention']['ms_per_step'], 'ffn', k['ffn_fused']['ms_per_step'], 'gemm', k['gemm']['ms_per_step'])"
  done
done
