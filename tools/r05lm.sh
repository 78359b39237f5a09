# batched lm_head on the int8 matrix cores + k_bt_gumbel (MIO_BT_LM_MMQ=1) vs the dot4 k_bt_lm_head
# (default): batch tests with it, then 8-stream 1.7B and C4
export TMPDIR=/tmp; out=gpurun_out/r05_lm2; mkdir -p $out
MIO_BT_LM_MMQ=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
for p in 3 4; do
timeout -k 10 300 python -u bench.py --preset $p --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/p${p}_def_$r.json 2> $out/p${p}_def_$r.err || { echo b_failed; exit 1; }
MIO_BT_LM_MMQ=1 timeout -k 10 300 python -u bench.py --preset $p --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/p${p}_mmq_$r.json 2> $out/p${p}_mmq_$r.err || { echo b1_failed; exit 1; }
done
done
MIO_BT_LM_MMQ=1 MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p3 -o run -- python3 tools/batch_prof.py 8 64 3 > $out/p3.txt 2>&1 || { echo p3_failed; exit 1; }
echo done
