set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/m5
timeout -k 10 300 python3 -u -m pytest tests/test_metrics.py tests/test_ouster.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/m5/pytest.log 2>&1 || { tail -30 gpurun_out/m5/pytest.log; exit 1; }
tail -2 gpurun_out/m5/pytest.log
timeout -k 10 900 python3 -u profiles/c5_e2e.py --scans 64 --out gpurun_out/m5/c5.json > gpurun_out/m5/c5.log 2>&1 || { tail -30 gpurun_out/m5/c5.log; exit 1; }
tail -3 gpurun_out/m5/c5.log
