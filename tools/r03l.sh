set -e
# batched decode at B=8: engine masks on the 2.6B Q8_0 (preset 4) and 1.7B Q4_K_M (preset 3)
# models after the MMQ one-pass prefetch; then the LLM GPU parity suites
out=gpurun_out/r03_l
mkdir -p $out
export TMPDIR=/tmp
for p in 4 3; do
  for m in 1 5 7 15; do
    MIO_MMQ_MASK=$m timeout -k 10 200 python3 tools/batch_prof.py 8 200 $p > $out/b8_p${p}_mask$m.txt 2>&1
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_llm_gpu.py tests/test_llm_batch_gpu.py > $out/tests.log 2>&1
