set -e
mkdir -p gpurun_out/r05ad
AB_CASES=c3 timeout -k 10 600 python3 -u tools/ab_lattices.py 3 product product@13:2 product@13:3 > gpurun_out/r05ad/c3_runs_ab.log 2>&1
AB_CASES=coronary timeout -k 10 300 python3 -u tools/ab_lattices.py 3 product product@13:1 product@13:2 > gpurun_out/r05ad/cor_runs_ab.log 2>&1
