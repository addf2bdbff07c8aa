set -e
mkdir -p gpurun_out/r05ab
timeout -k 10 700 bash tools/pmc_lattices.sh r05ab c4,coronary,ldc64 > gpurun_out/r05ab/pmc2.log 2>&1
AB_CASES=c4x4 timeout -k 10 300 python3 -u tools/ab_lattices.py 3 product product@13:3 product@13:4 > gpurun_out/r05ab/c4x4_xcd_ab.log 2>&1
timeout -k 10 600 python3 -u tools/probe_order_lab.py 3 > gpurun_out/r05ab/probe_order.log 2>&1
