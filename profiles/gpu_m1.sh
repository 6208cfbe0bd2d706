set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/m1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/m1/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/m1/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/m1/pytest_gpu.log
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/m1/bench1.json 2> gpurun_out/m1/bench1.err || { tail gpurun_out/m1/bench1.err; exit 1; }
cat gpurun_out/m1/bench1.json
TSDF_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --no-cpu > gpurun_out/m1/bench2.json 2> gpurun_out/m1/bench2.err || { tail gpurun_out/m1/bench2.err; exit 1; }
cat gpurun_out/m1/bench2.json
