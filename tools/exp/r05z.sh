set -e
mkdir -p gpurun_out/r05z
AB_CASES=coronary timeout -k 10 400 python3 -u tools/ab_lattices.py 4 product product@13:3 product@13:4 product@13:5 product@13:6 > gpurun_out/r05z/cor_xcd_ab.log 2>&1
