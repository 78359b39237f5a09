set -e
out=gpurun_out/r04_att1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_llm_gpu.py tests/test_llm_layers_gpu.py tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 60 tools/micro/mfma_i8_probe > $out/mfma_probe.txt 2>&1
bash tools/ab.sh r04_att1/ab 2 "python -u tools/llm_ab.py" c32@miotts-llama.cpp_amd/build c64@miotts-llama.cpp_amd/build_c64 c128@miotts-llama.cpp_amd/build_c128
bash tools/ab.sh r04_att1/bq 1 "python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" q1 q0:MIO_ATT_Q=0
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
cat $out/ab/*.json
python -c "import json;d=json.load(open('$out/bench.json'));print(d['value'],d['llm_ms_per_token'],d['roofline']['per_token_us'],d['batched'])"
