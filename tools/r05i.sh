export TMPDIR=/tmp; out=gpurun_out/r05_i; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_llm_layers_gpu.py tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py tests/test_llm_gpu.py -x -v --timeout 300 --timeout-method thread > $out/llm_tests.log 2>&1; echo tests_rc=$?
echo done
