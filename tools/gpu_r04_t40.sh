# column splitter: single-byte --encoding (latin-1, cp1252, ...) golden cases + the wcs suite
export TMPDIR=/tmp; D=gpurun_out/r04_t40; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q tests/test_gpu_split.py --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
echo __done__
