set -e
mkdir -p gpurun_out/r05ag
AB_CASES=ldc256,ldc512 timeout -k 10 900 python3 -u tools/ab_lattices.py 3 product product@13:2 product@13:3 > gpurun_out/r05ag/ldc_runs_ab.log 2>&1
