set -e
mkdir -p gpurun_out/r05x
timeout -k 10 600 bash tools/gpu_profile.sh r05x > gpurun_out/r05x/gpu_profile.log 2>&1
timeout -k 10 600 bash tools/pmc_lattices.sh r05x c3,c4,c4x4 > gpurun_out/r05x/pmc_lattices1.log 2>&1
