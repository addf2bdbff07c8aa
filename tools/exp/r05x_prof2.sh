set -e
mkdir -p gpurun_out/r05x
timeout -k 10 700 bash tools/pmc_lattices.sh r05x coronary,ldc64,ldc256 > gpurun_out/r05x/pmc_lattices2.log 2>&1
AB_CASES=c4,coronary timeout -k 10 300 python3 -u tools/ab_lattices.py 3 product tools/ab/c1_wg256 tools/ab/c1_wg64 > gpurun_out/r05x/c1_wg_ab.log 2>&1
AB_CASES=c4x4 timeout -k 10 300 python3 -u tools/ab_lattices.py 3 product product@9:1 product@9:4 product@9:16 > gpurun_out/r05x/c4x4_seg_ab.log 2>&1
