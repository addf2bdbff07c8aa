set -e
mkdir -p gpurun_out/r05k
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_checkpoint.py tests/test_gpu_bench.py "tests/test_gpu_parity.py::test_poiseuille_nee_paths_bitwise" > gpurun_out/r05k/tests.txt 2>&1
AB_CASES=c4,coronary,c4x4 timeout -k 10 500 python3 -u tools/ab_lattices.py 3 product tools/ab/c1_mask tools/ab/c1_temporal tools/ab/c1_mask_temporal > gpurun_out/r05k/c1_ab.log 2>&1
AB_CASES=c3 timeout -k 10 400 python3 -u tools/ab_lattices.py 3 product product@12:2 product@12:1 tools/ab/no_nee@12:1 > gpurun_out/r05k/c3_nee_ab.log 2>&1
