import os, sys, subprocess, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
from common import G, golden
import test_dropin_gpu as T
d = os.path.abspath('gpurun_out/rxdiag'); os.makedirs(d, exist_ok=True)
T.write_config(d, G, iterations=12)
x = golden()['data']; cap = os.path.join(d, 'cap.bin')
np.stack([x.real, x.imag], 1).astype(np.float64).tofile(cap)
env = dict(os.environ, OFDM_SDR_RX_FILE=cap, OFDM_SDR_RX_FORMAT='f64', OFDM_COMPAT_TRACE='1')
r = subprocess.run([os.path.abspath('oracle/_ref/rx')], cwd=d, env=env, capture_output=True, text=True, timeout=120)
open(os.path.join(d, 'stderr.txt'), 'w').write(r.stderr); open(os.path.join(d, 'stdout.txt'), 'w').write(r.stdout)
os.remove(cap)
print('rc', r.returncode)
