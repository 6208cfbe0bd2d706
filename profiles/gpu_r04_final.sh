#!/bin/bash
# Round 4 final evidence on HEAD: the whole GPU suite, smoke(), the 2-rank shared-GPU rehearsal of
# `bench.py --gpus 2`, then profiles/run_round.sh perf (PMC traffic, the bench line, rocprofv3
# stats of the pipelined and the serial bench commands).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/${1:-final}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  --durations=15 > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TSDF_BENCH_SHARED_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu > $O/bench_gpus2_shared.json 2> $O/bench_gpus2_shared.err || { tail -20 $O/bench_gpus2_shared.err; exit 1; }
cut -c1-300 $O/bench_gpus2_shared.json
bash profiles/run_round.sh $O perf
