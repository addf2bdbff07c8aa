set -e
mkdir -p gpurun_out/r05m
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05m/tests.txt 2>&1
AB_CASES=ldc64,c4,coronary,ldc32 timeout -k 10 400 python3 -u tools/ab_lattices.py 3 product tools/ab/t1_ntstores > gpurun_out/r05m/t1_ntstores_ab.log 2>&1
