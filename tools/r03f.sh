set -e
out=gpurun_out/r03_f
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
# per-kind engine choice at <= 8 tokens (q|k|v and gate|up on int8 MFMA): bit-exactness
timeout -k 10 600 $T tests/test_llm_batch_gpu.py tests/test_lfm2_gpu.py tests/test_llm_gpu.py::test_batched_prefill_matches_sequential tests/test_llm_gpu.py::test_mmq_equals_single_token_matvec > $out/tests.log 2>&1
for p in 3 4; do
  timeout -k 10 200 python3 -u tools/batch_prof.py 8 200 $p > $out/b8_p${p}_mask5.txt 2>&1
  MIO_MMQ_MASK=0 timeout -k 10 200 python3 -u tools/batch_prof.py 8 200 $p > $out/b8_p${p}_mask0.txt 2>&1
done
# the bench lines: C3 (+ 8 utterances batched), C4 per GPU (2.6B Q8_0, 8 utterances)
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
timeout -k 10 400 python -u bench.py --preset 4 --utts-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_c4.json 2> $out/bench_c4.err
# codec MFMA-busy share with the f32 GEMMs
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/pmcc -o codec -- python3 tools/codec_trace.py > $out/pmcc.txt 2>&1
# last: graph probe with decode-sized graphs (1128 nodes = 8 steps x 141 launches) x 30 replays
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/gprobe -o g -- python3 tools/graph_replay_probe.py 30 1128 > $out/gprobe.txt 2>&1 || echo "probe exit $?" >> $out/gprobe.txt
