# round 4: co-rank fix check + PMC passes on the split scan
export TMPDIR=/tmp; D=gpurun_out/r04_t2; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -k "corank or topk or tiny or equals" > $D/dist.log 2>&1 && \
bash tools/pmc.sh $D/pmc > $D/pmc.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $D/dist_split.log 2>&1
