set -e
# batch/prefill parity on the final engine choice, then the C4 and C5 configuration lines
out=gpurun_out/r04_n
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_llm_batch_gpu.py tests/test_llm_gpu.py -k "batch or prefill or mmq" > $out/tests.txt 2>&1
timeout -k 10 400 python -u bench.py --preset 4 --utts-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/c4_bench.json 2> $out/c4_bench.err
timeout -k 10 300 python -u bench.py --preset 2 --steps 5 --warmup 1 --no-cpu-baseline --batch 0 > $out/c2_bench.json 2> $out/c2_bench.err
AB_K=3 timeout -k 10 300 python -u tools/stream_ab.py > $out/c5_stream.jsonl 2> $out/c5_stream.err
tail -1 $out/tests.txt
