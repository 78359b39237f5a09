set -e
# round-end pass on one box: every GPU test, the default bench line, the eager kernel stats and
# the PMC traffic passes (tools/gpu_round.sh), the codec MFMA-busy PMC pass, smoke
bash tools/gpu_round.sh r04_final
out=gpurun_out/r04_final
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $out/pmcc -o codec -- python3 tools/codec_trace.py > $out/pmcc.out 2>&1
python3 tools/pmc_codec.py $(find $out/pmcc -name 'codec_counter_collection.csv') > $out/pmc_codec_mfma.json
find $out/pmcc -name '*kernel_trace.csv' -delete
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
echo done
