export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sync.py tests/test_dropin_gpu.py > gpurun_out/adhoc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/adhoc_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/dropin_rx_timing.py --frames 200 --trace > gpurun_out/adhoc_dropin.log 2>&1; rc=$?; tail -c 1500 gpurun_out/adhoc_dropin.log; [ $rc = 0 ] || exit $rc
python3 - <<'PY'
import os, sys, subprocess
sys.path[:0] = ["tools", "tests", "oracle", "c-ofdm_amd/python"]
from dropin_rx_timing import gapped_capture
from test_dropin_gpu import D, O, write_config
g = O.geometry(D)
d = "/tmp/dropin_prof"
os.makedirs(d, exist_ok=True)
write_config(d, D, iterations=140)
pay = g["bytes_per_frame"] - 8
body = bytes((i * 131 + 7) & 0xFF for i in range(100 * pay))
open(os.path.join(d, "FlyMeToTheMoon_mono.wav"), "wb").write(body)
txf = os.path.join(d, "tx.bin")
r = subprocess.run([os.path.abspath("oracle/_ref/tx")], cwd=d, env=dict(os.environ, OFDM_SDR_TX_FILE=txf), capture_output=True, text=True)
assert r.returncode == 0, r.stderr
gapped_capture(txf, g["frame_len"])
PY
cd /tmp/dropin_prof && OFDM_SDR_RX_FILE=/tmp/dropin_prof/tx.bin timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/dprof -o run -- $R/oracle/_ref/rx > $R/gpurun_out/dprof.log 2>&1; echo rc=$?
cd $R && python3 - <<'PY'
import csv, glob
for x in csv.DictReader(open('gpurun_out/dprof/run_kernel_stats.csv')):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1000,1), 'us')
for f in glob.glob('gpurun_out/dprof/*memory_copy_stats.csv'):
    for x in csv.DictReader(open(f)):
        print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1000,1), 'us')
PY
