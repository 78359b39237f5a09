set -e
out=gpurun_out/r03_g
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_llm_gpu.py::test_mmq_equals_single_token_matvec tests/test_llm_batch_gpu.py tests/test_llm_gpu.py::test_batched_prefill_matches_sequential > $out/tests.log 2>&1
for mask in 5 0 1 3 15; do
  MIO_MMQ_MASK=$mask timeout -k 10 200 python3 -u tools/batch_prof.py 8 200 4 > $out/b8_p4_mask${mask}.txt 2>&1
done
timeout -k 10 200 python3 -u tools/batch_prof.py 8 200 3 > $out/b8_p3_mask5.txt 2>&1
MIO_MMQ=1 timeout -k 10 200 python3 -u tools/batch_prof.py 8 200 4 > $out/b8_p4_mmqall.txt 2>&1
