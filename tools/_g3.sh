set -e
out=gpurun_out/r04_att3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lfm2_gpu.py -q --timeout 300 --timeout-method thread -rf > $out/lfm2.log 2>&1 || true
tail -5 $out/lfm2.log
MIO_BUILD_DIR=miotts-llama.cpp_amd/build_c128 timeout -k 10 300 python -u -m pytest tests/test_lfm2_gpu.py -k "generate or prefill" -q --timeout 300 --timeout-method thread -rf > $out/lfm2_c128.log 2>&1 || true
tail -5 $out/lfm2_c128.log
timeout -k 10 60 tools/micro/mfma_i8_probe > $out/mfma_probe.txt 2>&1
cat $out/mfma_probe.txt
bash tools/ab.sh r04_att3/ab 2 "python -u tools/llm_ab.py" c32@miotts-llama.cpp_amd/build c64@miotts-llama.cpp_amd/build_c64 c128@miotts-llama.cpp_amd/build_c128
bash tools/ab.sh r04_att3/bq 1 "python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline" q1 q0:MIO_ATT_Q=0
cat $out/ab/*.json
python3 -c "
import json,glob
for f in sorted(glob.glob('$out/bq/*.json')):
    d=json.load(open(f)); print(f, d['value'], d['llm_ms_per_token'], d['roofline']['per_token_us'], d['batched'])
"
