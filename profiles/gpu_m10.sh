set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/m10
timeout -k 10 600 python3 -u -m pytest tests/test_multigpu.py tests/test_growth.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/m10/pytest.log 2>&1 || { tail -30 gpurun_out/m10/pytest.log; exit 1; }
tail -1 gpurun_out/m10/pytest.log
bash profiles/gpu_scale_rehearsal.sh gpurun_out/m10
