set -e
mkdir -p gpurun_out/r05ac
AB_SHOW_PLACEMENT=1 AB_CASES=ldc256 timeout -k 10 900 python3 -u tools/ab_lattices.py 6 product product@13:1 > gpurun_out/r05ac/c2_rr_ab.log 2>&1
