# Q8_0 one-pass tile loop (k_mmq16_loop): parity, then C4 A/B
export TMPDIR=/tmp; out=gpurun_out/r05_x; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py -x -q --timeout 200 --timeout-method thread > $out/batch_tests.log 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/loop_$r.json 2> $out/loop_$r.err || { echo c4_failed; exit 1; }
MIO_MMQ_LOOP=0 timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/noloop_$r.json 2> $out/noloop_$r.err || { echo c40_failed; exit 1; }
done
echo done
