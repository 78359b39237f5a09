set -e
out=gpurun_out/r03_d
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py "tests/test_llm_gpu.py::test_batched_prefill_matches_sequential" > $out/tests.log 2>&1
timeout -k 10 200 python -u tools/batch_prof.py 8 200 3 > $out/b8.txt 2>&1
MIO_FUSED_QUANT=0 timeout -k 10 200 python -u tools/batch_prof.py 8 200 3 > $out/b8_nofq.txt 2>&1
timeout -k 10 200 python -u tools/batch_prof.py 16 200 3 > $out/b16.txt 2>&1
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
