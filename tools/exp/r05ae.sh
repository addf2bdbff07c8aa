set -e
mkdir -p gpurun_out/r05ae
AB_CASES=c4x4 timeout -k 10 600 python3 -u tools/ab_lattices.py 3 product product@1:1 product@1:1,13:17 > gpurun_out/r05ae/c4x4_cpl_ab.log 2>&1
