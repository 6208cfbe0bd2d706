# GPU parity suite, then the rank-0 rehearsals of the N-GPU runs (N = 1, 2, 4, 8) on one GPU.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/scale}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash profiles/gpu_scale_rehearsal.sh $OUT
