# pipelined wait_count (MIO_POLL_DEPTH 4): C2 and C3 with the whole attention block in one launch
# (default) vs attn_in + k_att_o (MIO_LAYER_ATT=0); the fused-launch bit-identity test first
export TMPDIR=/tmp; out=gpurun_out/r05_pp; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_gpu.py -k "fused_attention or layers" > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
for p in 2 3; do
timeout -k 10 300 python -u bench.py --preset $p --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c${p}_la_$r.json 2> $out/c${p}_la_$r.err || { echo b_failed; exit 1; }
MIO_LAYER_ATT=0 timeout -k 10 300 python -u bench.py --preset $p --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c${p}_ao_$r.json 2> $out/c${p}_ao_$r.err || { echo b0_failed; exit 1; }
done
done
timeout -k 10 200 python -u tools/step_timeline.py --preset 2 > $out/tl_c2_la.txt 2>&1 || { echo tl_failed; exit 1; }
echo done
