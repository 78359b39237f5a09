# C4: Q8_0 down on the 16x16 matrix cores with in-launch quantization (MIO_MMQ_MASK=15) vs dot4 (default 7)
export TMPDIR=/tmp; out=gpurun_out/r05_t; mkdir -p $out
MIO_MMQ_MASK=15 timeout -k 10 300 python -u -m pytest tests/test_llm_batch_gpu.py -x -q --timeout 200 --timeout-method thread -k "c4 or equal" > $out/tests15.log 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
MIO_MMQ_MASK=15 timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/m15_$r.json 2> $out/m15_$r.err || { echo b15_failed; exit 1; }
timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/m7_$r.json 2> $out/m7_$r.err || { echo b7_failed; exit 1; }
done
echo done
