set -e
# transposed row totals in the multi-token dot4 engine: parity (batch == single, prefill ==
# sequential) and the 8-stream step time of the 2.6B Q8_0 / 1.7B Q4_K_M
out=gpurun_out/${OUT:-r04_b}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_llm_batch_gpu.py tests/test_llm_gpu.py -k "batch or prefill or mmq" > $out/tests.txt 2>&1
timeout -k 10 200 python3 tools/batch_prof.py 8 200 4 > $out/p4_b8.txt 2>&1
timeout -k 10 200 python3 tools/batch_prof.py 8 200 3 > $out/p3_b8.txt 2>&1
timeout -k 10 200 python3 tools/batch_prof.py 16 200 4 > $out/p4_b16.txt 2>&1
cat $out/*.txt | grep -E "passed|failed|ms/step"
