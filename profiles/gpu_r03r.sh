# k_place A/B with parity: GPU parity subset on the default build, then the default build against
# every variant build in noetic-slam_amd/lib/var, interleaved, $REPS rounds (profiles/gpu_r03q.sh).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03r}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_growth.py tests/test_literal.py tests/test_multigpu.py tests/test_voxblox.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/gpu_r03q.sh $O
