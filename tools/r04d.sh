set -e
# eager kernel stats + VALU/wait PMC of the 8-stream batched decode, 2.6B Q8_0
out=gpurun_out/${OUT:-r04_d}
mkdir -p $out
export TMPDIR=/tmp
export MIO_NO_GRAPH=1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/k -o k -- python3 tools/batch_prof.py 8 48 ${PRESET:-4} > $out/k.out 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $out/a -o a -- python3 tools/batch_prof.py 8 16 ${PRESET:-4} > $out/a.out 2>&1
python3 tools/pmc_kernels.py $(find $out/a -name 'a_counter_collection.csv') k_pf_ k_mmq k_bt_ > $out/pass_a.txt
find $out -name '*.csv' -size +20M -delete
echo done
