# whole attention block in one launch (default) vs attn_in + k_att_o (MIO_LAYER_ATT=0) on presets 4 and 12
export TMPDIR=/tmp; out=gpurun_out/r05_pq; mkdir -p $out
for r in 1 2; do
for p in 4 12; do
timeout -k 10 300 python -u bench.py --preset $p --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c${p}_la_$r.json 2> $out/c${p}_la_$r.err || { echo b_failed; exit 1; }
MIO_LAYER_ATT=0 timeout -k 10 300 python -u bench.py --preset $p --no-cpu-baseline --no-cpu-c1 --batch 0 > $out/c${p}_ao_$r.json 2> $out/c${p}_ao_$r.err || { echo b0_failed; exit 1; }
done
done
echo done
