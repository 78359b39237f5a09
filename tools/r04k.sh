set -e
# weight units per register group of the batched dot4 engine (MIO_BT_UNITS) and the VGPR budget
out=gpurun_out/r04_k
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
 for b in build build_b build_c build_d; do
  for p in 4 3; do
   echo "$b p$p $(MIO_BUILD_DIR=miotts-llama.cpp_amd/$b timeout -k 10 200 python3 tools/batch_prof.py 8 200 $p 2>&1 | tail -1)" >> $out/times.txt
  done
 done
done
for b in build_b build_c build_d; do
  echo "$b B16 p4 $(MIO_BUILD_DIR=miotts-llama.cpp_amd/$b timeout -k 10 200 python3 tools/batch_prof.py 16 200 4 2>&1 | tail -1)" >> $out/times.txt
done
cat $out/times.txt
