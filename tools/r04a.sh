set -e
# PMC passes over the 8-stream batched decode of the 2.6B Q8_0 (eager launches, default
# engine choice): where the batched dot4 kernels' cycles go
out=gpurun_out/r04_a
mkdir -p $out
export TMPDIR=/tmp
export MIO_NO_GRAPH=1
timeout -k 10 200 python3 tools/batch_prof.py 8 48 4 > $out/time.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $out/a -o a -- python3 tools/batch_prof.py 8 16 4 > $out/a.out 2>&1
python3 tools/pmc_kernels.py $(find $out/a -name 'a_counter_collection.csv') k_pf_ k_mmq k_bt_ > $out/pass_a.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/b -o b -- python3 tools/batch_prof.py 8 16 4 > $out/b.out 2>&1
python3 tools/pmc_kernels.py $(find $out/b -name 'b_counter_collection.csv') k_pf_ k_mmq k_bt_ > $out/pass_b.txt
find $out -name '*.csv' -size +20M -delete
echo done
