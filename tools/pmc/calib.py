"""Run the PMC calibration kernels (3 launches each of 1 GiB copies) -- wrap with rocprofv3 --pmc."""
import ctypes, os, sys, torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "_lib", "libcalib.so"))
lib.calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
n = 1 << 30
a = torch.rand(n // 4, device="cuda")
b = torch.empty_like(a)
s = torch.cuda.current_stream().cuda_stream
for kind in (0, 1, 2, 3):
    for _ in range(3):
        assert lib.calib_run(kind, a.data_ptr(), b.data_ptr(), n, 1024, 512, s) == 0
torch.cuda.synchronize()
assert torch.equal(a, b)
print("calib done: bytes read per launch =", n, "written =", n)
