# GPU parity suite only: bash profiles/gpu_tests.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/t}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -15
exit $rc
