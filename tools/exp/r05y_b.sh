set -e
mkdir -p gpurun_out/r05y
timeout -k 10 600 bash tools/gpu_profile.sh r05y > gpurun_out/r05y/gpu_profile.log 2>&1
timeout -k 10 700 bash tools/pmc_lattices.sh r05y c3,c4x4,ldc256 > gpurun_out/r05y/pmc1.log 2>&1
