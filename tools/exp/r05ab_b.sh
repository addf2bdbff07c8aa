set -e
mkdir -p gpurun_out/r05ab
timeout -k 10 600 bash tools/gpu_profile.sh r05ab > gpurun_out/r05ab/gpu_profile.log 2>&1
timeout -k 10 700 bash tools/pmc_lattices.sh r05ab c3,c4x4,ldc256 > gpurun_out/r05ab/pmc1.log 2>&1
