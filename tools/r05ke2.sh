# K-quant tiles issuing their weight loads early, now also without in-launch quantization (the
# batched O projection): default vs MIO_KQ_EARLY=0; 8-stream 1.7B
export TMPDIR=/tmp; out=gpurun_out/r05_ke2; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 3 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/ke_$r.json 2> $out/ke_$r.err || { echo b_failed; exit 1; }
MIO_KQ_EARLY=0 timeout -k 10 300 python -u bench.py --preset 3 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/noke_$r.json 2> $out/noke_$r.err || { echo b1_failed; exit 1; }
done
MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p3 -o run -- python3 tools/batch_prof.py 8 64 3 > $out/p3.txt 2>&1 || { echo p3_failed; exit 1; }
echo done
