set -e
# persistent one-pass Q8_0 MMQ (B=8): parity suites first, then engine masks on the 2.6B Q8_0
out=gpurun_out/r03_m
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_llm_gpu.py tests/test_llm_batch_gpu.py > $out/tests.log 2>&1
for m in 1 3 5 7; do
  MIO_MMQ_MASK=$m timeout -k 10 200 python3 tools/batch_prof.py 8 200 4 > $out/b8_p4_mask$m.txt 2>&1
done
MIO_MMQ_PERSIST=0 MIO_MMQ_MASK=7 timeout -k 10 200 python3 tools/batch_prof.py 8 200 4 > $out/b8_p4_mask7_nopersist.txt 2>&1
