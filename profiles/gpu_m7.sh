set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/m7
timeout -k 10 300 python3 -u -m pytest tests/test_multigpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/m7/pytest.log 2>&1 || { tail -30 gpurun_out/m7/pytest.log; exit 1; }
tail -1 gpurun_out/m7/pytest.log
bash profiles/gpu_scale_rehearsal.sh gpurun_out/m7
