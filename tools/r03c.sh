set -e
out=gpurun_out/r03_c
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_llm_gpu.py > $out/tests.log 2>&1
timeout -k 10 200 python -u tools/prefill_time.py > $out/prefill.txt 2>&1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
export MIO_NO_GRAPH=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/bprof -o b -- python3 tools/batch_prof.py 8 64 3 > $out/bprof.txt 2>&1
