# C4 down: dot4 with in-launch producers (default) vs 16x16 matrix cores with chunked in-launch
# producers and W's first pass issued before the wait (MIO_MMQ_MASK=15)
export TMPDIR=/tmp; out=gpurun_out/r05_q8d; mkdir -p $out
MIO_MMQ_MASK=15 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py -k "c4 or equals_single" > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/dot4_$r.json 2> $out/dot4_$r.err || { echo b_failed; exit 1; }
MIO_MMQ_MASK=15 timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/mfma_$r.json 2> $out/mfma_$r.err || { echo b1_failed; exit 1; }
done
MIO_MMQ_MASK=15 MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4 -o run -- python3 tools/batch_prof.py 8 64 4 > $out/p4.txt 2>&1 || { echo p4_failed; exit 1; }
echo done
