set -e
mkdir -p gpurun_out/r05l
AB_CASES=ldc64,c4,coronary,c4x4,c3,ldc256 timeout -k 10 900 python3 -u tools/ab_lattices.py 3 product tools/ab/t1_dense tools/ab/t4g_loads tools/ab/t4g_stores tools/ab/t4g_both tools/ab/t4_stores > gpurun_out/r05l/temporal_ab.log 2>&1
