# Persistent k_place A/B: parity subset on the default build, then the default build, the
# one-item-per-workgroup build and HEAD's build twice each, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03p}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_growth.py tests/test_literal.py tests/test_multigpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for n in real one head; do
    lib=""; [ $n != real ] && lib=noetic-slam_amd/lib/var/libtsdf_hip_$n.so
    TSDF_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 32 --no-cpu > $O/${n}_$i.json 2> $O/${n}_$i.err || { tail -5 $O/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('$n', d['value'], d['kernel_ms_per_launch'])"
  done
done
