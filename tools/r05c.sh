export TMPDIR=/tmp; out=gpurun_out/r05_e; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_llm_gpu.py tests/test_llm_layers_gpu.py tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py -x -v --timeout 200 --timeout-method thread > $out/llm_tests.log 2>&1; echo tests_rc=$?
bash tools/ab.sh r05_e/ab 2 "python -u tools/llm_ab.py" mfma att0@miotts-llama.cpp_amd/build_att0 expf@miotts-llama.cpp_amd/build_expf r04@miotts-llama.cpp_amd/build_r04; echo ab_rc=$?
timeout -k 10 120 python -u tools/trace_kernels.py --pos 400 > $out/trace_mfma.txt 2>&1
MIO_BUILD_DIR=miotts-llama.cpp_amd/build_att0 timeout -k 10 120 python -u tools/trace_kernels.py --pos 400 > $out/trace_att0.txt 2>&1

MIO_BUILD_DIR=miotts-llama.cpp_amd/build_expf timeout -k 10 120 python -u tools/trace_kernels.py --pos 400 > $out/trace_expf.txt 2>&1
echo done
