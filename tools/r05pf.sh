# K-quant 16x16 matmuls: every pass's loads first (default build) vs pass by pass (build_ab,
# -DMIO_KQ_PF=0): batch tests, then the 8-stream 1.7B step, interleaved
export TMPDIR=/tmp; out=gpurun_out/r05_pf; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 3 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/pf_$r.json 2> $out/pf_$r.err || { echo b_failed; exit 1; }
MIO_BUILD_DIR=$PWD/miotts-llama.cpp_amd/build_ab timeout -k 10 300 python -u bench.py --preset 3 --utts-per-gpu 8 --no-cpu-baseline --batch 0 > $out/nopf_$r.json 2> $out/nopf_$r.err || { echo b1_failed; exit 1; }
done
MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p3 -o run -- python3 tools/batch_prof.py 8 64 3 > $out/p3.txt 2>&1 || { echo p3_failed; exit 1; }
echo done
