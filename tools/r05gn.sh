# codec GroupNorm: three launches (MIO_GN=3, default) vs one workgroup per group (MIO_GN=1) vs
# the sliced five launches (MIO_GN=5): codec parity tests, codec ms at T=700, kernel stats
export TMPDIR=/tmp; out=gpurun_out/r05_gn2; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_codec_gpu.py > $out/tests.txt 2>&1 || { echo tests_failed; exit 1; }
for g in 3 1 5 3 1 5; do
MIO_GN=$g timeout -k 10 200 python -u tools/codec_time.py >> $out/codec_gn$g.txt 2>&1 || { echo ct_failed; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/codec_time.py > $out/prof.txt 2>&1 || { echo prof_failed; exit 1; }
echo done
