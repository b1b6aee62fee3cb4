"""liblic from several host threads ("safe to call from several host
threads and processes, one device each").  A fresh process starts two threads that hit the
first-launch path of the halo convolution (its dynamic-LDS attribute, csrc/common.hip
ensure_dyn_lds) at the same time (fp16 and fp32 kernels), each on its own stream, and
repeat; every result must equal the single-threaded one bit for bit."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import sys, threading, torch
sys.path.insert(0, ROOT)
from lic_amd.layers import Conv2d
from lic_amd.functional import Act
torch.manual_seed(0)
mods = {dt: Conv2d(192, 192, 3, 1, 1).to("cuda") for dt in (torch.float16, torch.float32)}
xs = {dt: Act((torch.randn(8, 64, 64, 192, device="cuda") * 0.5).to(dt)) for dt in mods}
outs, errs = {}, []
barrier = threading.Barrier(2)

def work(dt):
    try:
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            barrier.wait()
            ys = [mods[dt].run(xs[dt]).t for _ in range(20)]
        s.synchronize()
        outs[dt] = ys
    except Exception as e:  # reported by the parent
        errs.append(repr(e))

ts = [threading.Thread(target=work, args=(dt,)) for dt in mods]
[t.start() for t in ts]
[t.join() for t in ts]
assert not errs, errs
for dt, ys in outs.items():
    ref = mods[dt].run(xs[dt]).t
    torch.cuda.synchronize()
    for y in ys:
        assert torch.equal(y, ref), dt
print("THREADS_OK")
'''


def test_two_host_threads_first_launch():
    r = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + SCRIPT], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "THREADS_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
