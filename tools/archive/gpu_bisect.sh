mkdir -p gpurun_out
P="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 200 $P tests/test_ops_gpu.py tests/test_xgmi_gpu.py -k "not linear_ln and not prealloc-True" > gpurun_out/bis3.log 2>&1
timeout -k 10 200 $P tests/test_ops_gpu.py tests/test_xgmi_gpu.py -k "not linear_ln and not prealloc-False" > gpurun_out/bis9.log 2>&1
true
