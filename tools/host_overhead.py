"""Host-side cost of one C-ABI launch, of torch.empty and of an autograd op."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import _lib, ops  # noqa: E402

x = torch.zeros(1024, device="cuda")
s = torch.ones(1, device="cuda")
lib = _lib.lib()
f = lib.fns["vt_act_fwd"]
st = torch.cuda.current_stream().cuda_stream
torch.cuda.synchronize()
N = 2000


def timeit(name, fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:40s} host {1e6 * (t1 - t0) / N:7.2f} us/call   wall {1e6 * (t2 - t0) / N:7.2f} us/call", flush=True)


timeit("raw ctypes fn (vt_act_fwd, 1024 el)", lambda: f(x.data_ptr(), 1024, 0, x.data_ptr(), st))
timeit("_lib.call", lambda: _lib.call("vt_act_fwd", x.data_ptr(), 1024, 0, x.data_ptr(), _lib.stream()))
timeit("torch.empty(4096)", lambda: torch.empty(4096, device="cuda"))
timeit("torch add (x + x)", lambda: x + x)
timeit("current_stream().cuda_stream", lambda: torch.cuda.current_stream().cuda_stream)
