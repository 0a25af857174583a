set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "container or inverted or hll or empty" tests/test_gpu_configs.py -k "container or inverted or hll or empty or config5" > gpurun_out/c5_tests.log 2>&1 || { tail -30 gpurun_out/c5_tests.log; exit 1; }
tail -2 gpurun_out/c5_tests.log
timeout -k 10 400 python3 -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c5.json')); r=d['roofline']; print('config5 ms_per_step', round(d['ms_per_step'],3), 'kernel_ms', round(r['kernel_ms'],3), r.get('kernel'))"
PH_AGG_CONT=0 timeout -k 10 400 python3 -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu --no-parity > gpurun_out/c5b.json 2> gpurun_out/c5b.err || { tail -5 gpurun_out/c5b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c5b.json')); r=d['roofline']; print('config5 bitmaps ms_per_step', round(d['ms_per_step'],3), 'kernel_ms', round(r['kernel_ms'],3))"
