set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/gap}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tr -o run --output-format csv -- python3 bench.py --no-cpu --steps 64 --warmup 8 --batch 1 > $O/b1.json 2> $O/b1.err || { tail -5 $O/b1.err; exit 1; }
python3 profiles/gap_trace.py $O/tr | tee $O/gaps_b1.txt
rm -rf $O/tr
