set -e
mkdir -p gpurun_out/r05y
timeout -k 10 700 bash tools/pmc_lattices.sh r05y c4,coronary,ldc64 > gpurun_out/r05y/pmc2.log 2>&1
AB_CASES=coronary,c4 timeout -k 10 300 python3 -u tools/ab_lattices.py 3 product product@13:1 product@13:4 > gpurun_out/r05y/c1_xcd_ab.log 2>&1
AB_CASES=c3 timeout -k 10 400 python3 -u tools/ab_lattices.py 3 product product@12:2 tools/ab/rec_dma_only@12:2 tools/ab/no_nee@12:1 > gpurun_out/r05y/rec_dma_ab.log 2>&1
