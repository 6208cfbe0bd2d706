# k_compact variants (chunk 1024 real / 2048 / 4096) at 1-scan and 64-scan batches; parity first.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03f}
mkdir -p $O
bash profiles/gpu_iter.sh $O/t1 "tests/test_gpu_parity.py tests/test_growth.py" "" || exit 1
BENCH_ARGS="--batch 1 --steps 256 --warmup 8" STEPS=256 bash profiles/variants.sh $O/var_b1 || exit 1
STEPS=32 bash profiles/variants.sh $O/var_b64 || exit 1
for v in ch2k ch4k; do
  TSDF_HIP_LIB=noetic-slam_amd/lib/var/libtsdf_hip_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "composition or small or pipelined" > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/t_$v.log)"
done
