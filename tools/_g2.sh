set -e
out=gpurun_out/r04_mmq16
mkdir -p $out
export TMPDIR=/tmp
MIO_MMQ16=0 timeout -k 10 300 python -u -m pytest tests/test_lfm2_gpu.py -q --timeout 300 --timeout-method thread -rf > $out/lfm2_old.log 2>&1 || true
tail -5 $out/lfm2_old.log
timeout -k 10 600 python -u -m pytest tests/test_llm_gpu.py -k "mmq or prefill" tests/test_llm_batch_gpu.py -q --timeout 300 --timeout-method thread -rf > $out/tests.log 2>&1 || true
tail -8 $out/tests.log
