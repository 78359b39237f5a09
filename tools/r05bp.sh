# batched decode kernel stats: 1.7B Q4_K_M at 8 streams and 2.6B Q8_0 at 8 streams (eager launches)
export TMPDIR=/tmp; out=gpurun_out/r05_bp; mkdir -p $out
MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p3 -o run -- python3 tools/batch_prof.py 8 64 3 > $out/p3.txt 2>&1 || { echo p3_failed; exit 1; }
MIO_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4 -o run -- python3 tools/batch_prof.py 8 64 4 > $out/p4.txt 2>&1 || { echo p4_failed; exit 1; }
echo done
