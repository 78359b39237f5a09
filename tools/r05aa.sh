# consumer-side merge in the fused attention launches (MIO_ATT_CM_KB): parity + A/B on C2 / C3
export TMPDIR=/tmp; out=gpurun_out/r05_aa; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_llm_layers_gpu.py tests/test_llm_gpu.py tests/test_lfm2_gpu.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 2 --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c2_cm_$r.json 2> $out/c2_cm_$r.err || { echo b_failed; exit 1; }
MIO_ATT_CM_KB=0 timeout -k 10 300 python -u bench.py --preset 2 --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c2_nocm_$r.json 2> $out/c2_nocm_$r.err || { echo b0_failed; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c3_cm_$r.json 2> $out/c3_cm_$r.err || { echo b3_failed; exit 1; }
MIO_ATT_CM_KB=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c3_nocm_$r.json 2> $out/c3_nocm_$r.err || { echo b30_failed; exit 1; }
done
echo done
