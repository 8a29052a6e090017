set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_photo.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6b_photo.log 2>&1; tail -2 gpurun_out/r6b_photo.log
bash tools/k1_traffic_attr.sh r6b "stop8 stop1 stop2 stop4 nozero full cf16 cf2" > gpurun_out/r6b_attr.log 2>&1; cat gpurun_out/r6b_attr.log
bash tools/ab_tree.sh "new cf16 cf2" 2 --steps 20 --warmup 5 > gpurun_out/r6b_ab.log 2>&1; cat gpurun_out/r6b_ab.log
