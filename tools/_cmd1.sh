set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "rag_mean or model or forward" > gpurun_out/t1.log 2>&1; rc=$?; tail -5 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/knn_micro.py > gpurun_out/knn_micro.log 2>&1; rc=$?; cat gpurun_out/knn_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/bench2.log 2>&1; tail -1 gpurun_out/bench2.log
