set -e
mkdir -p gpurun_out/r05x
timeout -k 10 900 bash tools/gpu_profile.sh r05x > gpurun_out/r05x/gpu_profile.log 2>&1
timeout -k 10 900 bash tools/pmc_lattices.sh r05x c3,c4,c4x4,coronary,ldc64,ldc256 > gpurun_out/r05x/pmc_lattices.log 2>&1
