export TMPDIR=/tmp; out=gpurun_out/r05_g; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py tests/test_llm_layers_gpu.py tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py -x -q --timeout 200 --timeout-method thread > $out/llm_tests.log 2>&1; echo tests_rc=$?
bash tools/ab.sh r05_g/ab 2 "python -u tools/llm_ab.py" mfma r04@miotts-llama.cpp_amd/build_r04; echo ab_rc=$?
for p in 100 400 700; do timeout -k 10 120 python -u tools/trace_kernels.py --pos $p > $out/trace_$p.txt 2>&1 || exit 1; done
echo done
