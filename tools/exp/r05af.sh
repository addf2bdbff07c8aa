set -e
mkdir -p gpurun_out/r05af
AB_CASES=c3 timeout -k 10 600 python3 -u tools/ab_lattices.py 3 product tools/ab/fix_empty tools/ab/fix_noload tools/ab/nee_nostore > gpurun_out/r05af/fix_parts_ab.log 2>&1
