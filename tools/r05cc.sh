# C2 (0.1B): the whole attention block in one launch (default) vs attn_in + k_att_o (MIO_LAYER_ATT=0)
export TMPDIR=/tmp; out=gpurun_out/r05_cc; mkdir -p $out
for r in 1 2; do
timeout -k 10 300 python -u bench.py --preset 2 --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c2_la_$r.json 2> $out/c2_la_$r.err || { echo b_failed; exit 1; }
MIO_LAYER_ATT=0 timeout -k 10 300 python -u bench.py --preset 2 --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c2_ao_$r.json 2> $out/c2_ao_$r.err || { echo b0_failed; exit 1; }
done
MIO_LAYER_ATT=0 timeout -k 10 200 python -u tools/step_timeline.py --preset 2 > $out/tl_c2_ao.txt 2>&1 || { echo tl_failed; exit 1; }
echo done
