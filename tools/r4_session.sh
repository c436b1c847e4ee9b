#!/bin/bash
# Round-4 GPU session (STEPS selects): new tests, attention / train-attention timing, full GPU
# suite, smoke, bench, rocprofv3 stats of the bench.  Each GPU step has its own time limit; a
# crash / abort / timeout (rc not in {0,1}) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r4}
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n ${TAILN:-12} "$OUT/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v -rf --timeout 300 --timeout-method thread -s"
for s in ${STEPS:-new attn bench}; do
  case $s in
    new)   step pytest_new 900 $PT ${NEW_TESTS:-tests/test_gpu_ddp.py tests/test_gpu_infer.py tests/test_gpu_rccl.py} ;;
    attnt) step pytest_attn 400 $PT tests/test_gpu_kernels.py tests/test_gpu_train.py -k "attention or attn" ;;
    attn)  step attn_only 240 env REPS=8 ROUNDS=3 ATTN_VARIANTS=${ATTN_VARIANTS:-0} python tools/attn_only.py
           step train_attn 200 python tools/train_attn_micro.py ;;
    traffic) step pmc_traffic 900 bash tools/pmc.sh ;;
    pmc)   step attn_pmc 300 env TAG=${TAG}_attn bash tools/pmc_attn.sh ;;
    stacks) step train_stacks 400 python tools/train_dispatch_log.py ;;
    tprof) step train_torchprof 400 python tools/train_torchprof.py
           step train_only 300 python tools/train_only.py ;;
    c2)    step knn_emb_micro 300 python tools/knn_emb_micro.py ;;
    tprof2) step train_rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trainprof_$TAG -o train \
             -- python3 tools/train_only.py
           rm -f $OUT/trainprof_$TAG/*/*.db $OUT/trainprof_$TAG/*.db
           python3 tools/prof_top.py $OUT/trainprof_$TAG 40 > $OUT/${TAG}_train_prof_top.txt 2>&1; head -45 $OUT/${TAG}_train_prof_top.txt ;;
    dx)    step dx_micro 300 python tools/dx_micro.py ;;
    sgt)   step sg_train_micro 300 python tools/sg_train_micro.py ;;
    tblas) step train_only_blas0 300 env BLAS_DX=0 python tools/train_only.py
           step train_only_blas1 300 env BLAS_DX=1 python tools/train_only.py ;;
    ln)    step ln_micro 300 python tools/ln_micro.py ;;
    dw)    step dw_micro 300 env DW_XCD=0,1 python tools/dw_micro.py ;;
    tonly) step train_only_a 300 env SNVRAG_DW_XCD=0 python tools/train_only.py
           step train_only_b 300 env SNVRAG_DW_XCD=1 python tools/train_only.py ;;
    gpu)   step pytest_gpu 1100 $PT tests -m gpu ${PYTEST_ARGS:-} ;;
    sel)   step pytest_sel 800 $PT tests -m gpu -k "${PYTEST_K}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps ${BSTEPS:-10} --warmup 3 ${BENCH_ARGS:-} ;;
    prof)  step prof 700 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench \
             -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0
           rm -f $OUT/prof_$TAG/*/*.db $OUT/prof_$TAG/*.db
           python3 tools/prof_top.py $OUT/prof_$TAG 30 > $OUT/${TAG}_prof_top.txt 2>&1; head -30 $OUT/${TAG}_prof_top.txt ;;
  esac
done
