set -e
mkdir -p gpurun_out/r05i
AB_CASES=c3 timeout -k 10 500 python3 -u tools/ab_lattices.py 3 product tools/ab/rec_exact product@12:2 tools/ab/no_nee@12:1 > gpurun_out/r05i/rec_ab.log 2>&1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05i/gpu_tests.txt 2>&1
