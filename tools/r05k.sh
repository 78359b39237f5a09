export TMPDIR=/tmp; out=gpurun_out/r05_k; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_llm_batch_gpu.py tests/test_llm_gpu.py -x -q --timeout 300 --timeout-method thread > $out/llm_tests.log 2>&1 || { echo tests_failed; exit 1; }
timeout -k 10 500 python -u bench.py --preset 12 --no-cpu-baseline --no-cpu-c1 > $out/bf16.json 2> $out/bf16.err
echo done
