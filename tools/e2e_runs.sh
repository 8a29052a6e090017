mkdir -p gpurun_out
timeout -k 10 400 python tools/loader_bench.py --n 20000 --epochs 2 > gpurun_out/loader_bench.log 2> gpurun_out/loader_bench.err || { tail -20 gpurun_out/loader_bench.err; exit 1; }
cat gpurun_out/loader_bench.log
FFCV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --dataset-size 65536 > gpurun_out/bench_2r.log 2>&1 || { tail -20 gpurun_out/bench_2r.log; exit 1; }
tail -1 gpurun_out/bench_2r.log | cut -c1-400
timeout -k 10 300 python bench.py --config c5 --steps 30 --warmup 5 --cpu-budget 8 > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log
timeout -k 10 300 python bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-300
