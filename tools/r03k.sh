set -e
out=gpurun_out/r03_k
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
# prologue quantization straight from registers (no LDS staging row): LLM parity suites
timeout -k 10 900 $T tests/test_llm_gpu.py tests/test_llm_layers_gpu.py tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py > $out/tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
timeout -k 10 200 python3 -u tools/step_timeline.py --pos 400 > $out/tl400.txt 2>&1
