set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03l}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_multigpu.py tests/test_host_replay.py tests/test_gpu_parity.py" "" || exit 1
TSDF_HIP_LIB=noetic-slam_amd/lib/var/libtsdf_hip_xcd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_literal.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_xcd.log 2>&1 || { tail -20 $O/t_xcd.log; exit 1; }
echo "xcd: $(tail -1 $O/t_xcd.log)"
STEPS=32 bash profiles/variants.sh $O/var1 || exit 1
STEPS=32 bash profiles/variants.sh $O/var2 || exit 1
TSDF_HOST_TIMING=1 bash profiles/gpu_live.sh $O/live || exit 1
for n in 2 4 8; do grep -h "over 352" $O/live/h$n.err; done
TSDF_BENCH_SHARED_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 8 --no-cpu > $O/bench_gpus2_shared.json 2> $O/g2.err || { tail -5 $O/g2.err; exit 1; }
cat $O/bench_gpus2_shared.json
