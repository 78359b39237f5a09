# occupancy-bounded in-launch quantization kernels (k_mmq16q, 3 workgroups per CU): parity + A/B
export TMPDIR=/tmp; out=gpurun_out/r05_w; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_llm_batch_gpu.py -x -q --timeout 200 --timeout-method thread > $out/batch_tests.log 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_$r.json 2> $out/c4_$r.err || { echo c4_failed; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-c1 > $out/b8_$r.json 2> $out/b8_$r.err || { echo b8_failed; exit 1; }
done
echo done
