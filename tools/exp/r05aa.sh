set -e
mkdir -p gpurun_out/r05aa
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_mask.py::test_xcd_run_bitwise" > gpurun_out/r05aa/tests.txt 2>&1
AB_CASES=coronary,c4,c3 timeout -k 10 500 python3 -u tools/ab_lattices.py 3 product product@13:17 > gpurun_out/r05aa/auto_ab.log 2>&1
