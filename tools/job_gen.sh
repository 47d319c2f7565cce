set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_native.py -v --timeout 200 --timeout-method thread > gpurun_out/gen.log 2>&1; echo "gen rc=$?"
tail -25 gpurun_out/gen.log
