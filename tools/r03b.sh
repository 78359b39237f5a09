set -e
out=gpurun_out/r03_b
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_lfm2_gpu.py > $out/lfm2.log 2>&1
timeout -k 10 600 $T "tests/test_llm_layers_gpu.py::test_layers_match_oracle_on_gpu_inputs[7]" \
  "tests/test_llm_layers_gpu.py::test_layers_match_oracle_on_gpu_inputs[8]" \
  "tests/test_llm_layers_gpu.py::test_layers_match_oracle_on_gpu_inputs[6]" \
  tests/test_codec_gpu.py::test_codec_f16_weights tests/test_llm_gpu.py > $out/tests.log 2>&1
timeout -k 10 200 python -u tools/prefill_time.py > $out/prefill.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --batch 0 > $out/bench.json 2> $out/bench.err
