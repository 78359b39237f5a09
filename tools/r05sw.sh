export TMPDIR=/tmp; out=gpurun_out/r05_sw; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_llm_batch_gpu.py -k engine_switches > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
echo done
