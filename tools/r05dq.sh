# C4 (2.6B Q8_0, 8 streams): dot4 down quantizing h in the launch (default) vs behind
# k_bt_quant_split (MIO_BT_DQ=0); q|k|v on the matrix cores in both; batch tests first
export TMPDIR=/tmp; out=gpurun_out/r05_dq; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_dq_$r.json 2> $out/c4_dq_$r.err || { echo c4_failed; exit 1; }
MIO_BT_DQ=0 timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_nodq_$r.json 2> $out/c4_nodq_$r.err || { echo c40_failed; exit 1; }
done
MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4 -o run -- python3 tools/batch_prof.py 8 64 4 > $out/p4.txt 2>&1 || { echo p4_failed; exit 1; }
echo done
