set -e
mkdir -p gpurun_out/r05g
AB_CASES=c3 timeout -k 10 400 python3 -u tools/ab_lattices.py 3 product tools/ab/nee_nostore tools/ab/no_nee@12:1 tools/ab/no_nee_valu@12:1 > gpurun_out/r05g/nee_cost.log 2>&1
AB_CASES=ldc256,c3 timeout -k 10 500 python3 -u tools/ab_lattices.py 4 tools/ab/xcdrun@13:0 tools/ab/xcdrun@13:1 tools/ab/xcdrun@13:3 > gpurun_out/r05g/xcd_ab.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mask.py -k write_no_wall_slot -x -v --timeout 120 --timeout-method thread > gpurun_out/r05g/tests.txt 2>&1
