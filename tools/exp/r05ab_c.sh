set -e
mkdir -p gpurun_out/r05ab
timeout -k 10 700 bash tools/pmc_lattices.sh r05ab c4,coronary,ldc64 > gpurun_out/r05ab/pmc2.log 2>&1
