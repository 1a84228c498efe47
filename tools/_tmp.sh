set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_file_random.py tests/test_gpu_layout.py tests/test_gpu_host_pageable.py tests/test_gpu_jni_core.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tee_r5zc.log 2>&1 || { tail -30 gpurun_out/pytest_tee_r5zc.log; exit 1; }
tail -1 gpurun_out/pytest_tee_r5zc.log
RSAMD_TEST_LIB=java-reed-solomon-distributed-file-system_amd/lib/bounds/librsamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_file_random.py tests/test_gpu_host_pageable.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tee_bounds_r5zc.log 2>&1 || { tail -30 gpurun_out/pytest_tee_bounds_r5zc.log; exit 1; }
tail -1 gpurun_out/pytest_tee_bounds_r5zc.log
timeout -k 10 600 python3 tools/host_legs.py --var RSAMD_DECODE_TEE=0 RSAMD_DECODE_TEE=1 RSAMD_DECODE_TEE=0 RSAMD_DECODE_TEE=1 RSAMD_DECODE_TEE=0 RSAMD_DECODE_TEE=1 > gpurun_out/host_legs_tee_r5zc.txt
