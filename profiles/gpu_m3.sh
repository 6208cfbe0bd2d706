set -o pipefail
bash profiles/gpu_tests.sh gpurun_out/m3 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu --semantics vdbfusion_f64 --steps 16 > gpurun_out/m3/bench_f64.json 2> gpurun_out/m3/bench_f64.err || exit 1
cat gpurun_out/m3/bench_f64.json
