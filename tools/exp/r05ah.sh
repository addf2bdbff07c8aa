set -e
mkdir -p gpurun_out/r05ah
for i in 1 2 3 4 5; do
  timeout -k 10 240 python3 -u bench.py --steps 50 --warmup 10 --no-secondary --no-cpu-baseline >> gpurun_out/r05ah/bench_spread.jsonl 2>> gpurun_out/r05ah/bench_spread.err
done
