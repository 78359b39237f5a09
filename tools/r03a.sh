set -e
out=gpurun_out/r03_a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_llm_layers_gpu.py tests/test_llm_batch_gpu.py tests/test_codec_gpu.py -x -v -s --timeout 600 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python -u tools/prefill_time.py > $out/prefill.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --batch 0 > $out/bench.json 2> $out/bench.err
