set -e
# in-launch quantization from preloaded inputs (MIO_BT_FQ): parity + 8-stream step times
out=gpurun_out/${OUT:-r04_f}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_llm_batch_gpu.py tests/test_llm_gpu.py -k "batch or prefill or mmq" > $out/tests.txt 2>&1
for fqv in 3 0 1 2; do
  for p in 4 3; do
    echo "fq=$fqv p=$p $(MIO_BT_FQ=$fqv timeout -k 10 200 python3 tools/batch_prof.py 8 200 $p 2>&1 | tail -1)" >> $out/times.txt
  done
done
MIO_BT_FQ=0 timeout -k 10 200 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests_fq0.txt 2>&1
cat $out/times.txt; grep -h passed $out/tests*.txt
