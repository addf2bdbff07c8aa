set -e
mkdir -p gpurun_out/r05h
AB_CASES=c3 timeout -k 10 400 python3 -u tools/ab_lattices.py 3 product product@12:2 tools/ab/no_nee@12:1 > gpurun_out/r05h/rec_ab.log 2>&1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05h/gpu_tests.txt 2>&1
