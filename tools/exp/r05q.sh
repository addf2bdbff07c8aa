set -e
mkdir -p gpurun_out/r05q
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05q/tests.txt 2>&1
AB_CASES=c3,ldc256,c4x4 timeout -k 10 600 python3 -u tools/ab_lattices.py 3 product product@13:17 > gpurun_out/r05q/xcd_auto_ab.log 2>&1
AB_CASES=c3,c4x4 timeout -k 10 400 python3 -u tools/ab_lattices.py 3 product tools/ab/fix64 > gpurun_out/r05q/fix64_ab.log 2>&1
