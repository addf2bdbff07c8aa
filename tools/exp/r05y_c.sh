set -e
mkdir -p gpurun_out/r05y
timeout -k 10 700 bash tools/pmc_lattices.sh r05y c4,coronary,ldc64 > gpurun_out/r05y/pmc2.log 2>&1
