# in-launch quantization of the batched matmuls (launch_mmq_q): parity, then A/B of the
# batched line (1.7B, 8 streams) and C4 (2.6B Q8_0, 8 streams)
export TMPDIR=/tmp; out=gpurun_out/r05_r; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py -x -q --timeout 200 --timeout-method thread > $out/batch_tests.log 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-c1 > $out/qf_$r.json 2> $out/qf_$r.err || { echo bench_failed; exit 1; }
MIO_BT_QF=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-cpu-c1 > $out/noqf_$r.json 2> $out/noqf_$r.err || { echo bench0_failed; exit 1; }
done
timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_qf.json 2> $out/c4_qf.err || { echo c4_failed; exit 1; }
MIO_BT_QF=0 timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_noqf.json 2> $out/c4_noqf.err || { echo c40_failed; exit 1; }
echo done
