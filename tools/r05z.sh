# C4 (2.6B Q8_0, 8 streams) and the 1.7B 8-stream step: eager kernel stats of the batched decode
export TMPDIR=/tmp; out=gpurun_out/r05_z; mkdir -p $out
MIO_BT_QF=0 MIO_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4 -o run -- python3 bench.py --preset 4 --utts-per-gpu 8 --steps 1 --warmup 0 --no-cpu-baseline --batch 0 > $out/c4_prof.json 2> $out/c4_prof.err || { echo prof4_failed; exit 1; }
find $out/p4 -name '*kernel_stats.csv' -exec cp {} $out/c4_kernel_stats.csv \;
rm -rf $out/p4
echo done
