set -e
out=gpurun_out/r03_h
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_llm_gpu.py::test_mmq_equals_single_token_matvec tests/test_llm_batch_gpu.py tests/test_llm_gpu.py::test_batched_prefill_matches_sequential > $out/tests.log 2>&1
for p in 4 3; do
  for b in build build_u8 build build_u8; do
    MIO_BUILD_DIR=miotts-llama.cpp_amd/$b timeout -k 10 200 python3 -u tools/batch_prof.py 8 200 $p >> $out/b8_p${p}_units.txt 2>&1
    echo "  ^ $b" >> $out/b8_p${p}_units.txt
  done
done
timeout -k 10 200 python3 -u tools/prefill_time.py 4 > $out/prefill_p4.txt 2>&1
