# K-quant down (1.7B, K = 6144) with in-launch producers per (token, 2048 chunk) (default) vs
# one per token (MIO_BT_QCHUNK=0); 8-stream 1.7B
export TMPDIR=/tmp; out=gpurun_out/r05_qc; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 3 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/qc_$r.json 2> $out/qc_$r.err || { echo b_failed; exit 1; }
MIO_BT_QCHUNK=0 timeout -k 10 300 python -u bench.py --preset 3 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/noqc_$r.json 2> $out/noqc_$r.err || { echo b1_failed; exit 1; }
done
MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p3 -o run -- python3 tools/batch_prof.py 8 64 3 > $out/p3.txt 2>&1 || { echo p3_failed; exit 1; }
echo done
