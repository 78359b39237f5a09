set -e
# two workgroups per CU for the one-pass batched matvecs (build_b: MIO_BT_UNITS=2, MIO_BT_MINB=2)
out=gpurun_out/r04_j
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
  echo "base $(timeout -k 10 200 python3 tools/batch_prof.py 8 200 4 2>&1 | tail -1)" >> $out/times.txt
  echo "b wgm1 $(MIO_BUILD_DIR=miotts-llama.cpp_amd/build_b timeout -k 10 200 python3 tools/batch_prof.py 8 200 4 2>&1 | tail -1)" >> $out/times.txt
  echo "b wgm2 $(MIO_BT_WGM=2 MIO_BUILD_DIR=miotts-llama.cpp_amd/build_b timeout -k 10 200 python3 tools/batch_prof.py 8 200 4 2>&1 | tail -1)" >> $out/times.txt
done
echo "p3 base $(timeout -k 10 200 python3 tools/batch_prof.py 8 200 3 2>&1 | tail -1)" >> $out/times.txt
echo "p3 b wgm2 $(MIO_BT_WGM=2 MIO_BUILD_DIR=miotts-llama.cpp_amd/build_b timeout -k 10 200 python3 tools/batch_prof.py 8 200 3 2>&1 | tail -1)" >> $out/times.txt
MIO_BT_WGM=2 MIO_BUILD_DIR=miotts-llama.cpp_amd/build_b timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_llm_batch_gpu.py > $out/tests_b.txt 2>&1 || true
cat $out/times.txt; tail -1 $out/tests_b.txt
