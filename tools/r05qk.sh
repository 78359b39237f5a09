# C4 (2.6B Q8_0, 8 streams): q|k|v on the dot4 engine quantizing in the launch (default) vs on
# the 16x16 matrix cores with in-launch quantization producers (MIO_BT_FQ=0); batch tests first
export TMPDIR=/tmp; out=gpurun_out/r05_qk; mkdir -p $out
MIO_BT_FQ=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_def_$r.json 2> $out/c4_def_$r.err || { echo c4_failed; exit 1; }
MIO_BT_FQ=0 timeout -k 10 300 python -u bench.py --preset 4 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/c4_fq0_$r.json 2> $out/c4_fq0_$r.err || { echo c40_failed; exit 1; }
done
echo done
