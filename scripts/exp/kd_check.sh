# key dictionary: GPU tests, then the strings workload
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_keys.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/kd_tests.log 2>&1
rc=$?
tail -4 gpurun_out/kd_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; grep -E "Error|assert" gpurun_out/kd_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --workload strings --no-cpu-baseline > gpurun_out/wl_strings2.json 2> gpurun_out/wl_strings2.err && \
python3 -c "
import json; d=json.loads(open('gpurun_out/wl_strings2.json').read().strip().splitlines()[-1]); print('strings', d['value']/1e9, d['ms_per_step'])"
