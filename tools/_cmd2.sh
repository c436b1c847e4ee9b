set -u
mkdir -p gpurun_out
timeout -k 10 300 python tools/knn_micro.py > gpurun_out/knn_micro2.log 2>&1; rc=$?; cat gpurun_out/knn_micro2.log; exit $rc
