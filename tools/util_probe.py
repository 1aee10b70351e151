"""Lane utilisation of the adjoint march loop (needs tools/libtvam_exp4.so, TVAM_EXPERIMENT=4)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtvam_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.path.abspath(sys.argv[1])
from drtvam_amd.configs import benchy_index_matched, desc_from_config  # noqa: E402
from drtvam_amd.engine import Projection  # noqa: E402

N = int(sys.argv[2]) if len(sys.argv) > 2 else 400
tile = int(sys.argv[3]) if len(sys.argv) > 3 else 0
d = desc_from_config(benchy_index_matched(N=N, angles=N), tile=tile)
p = Projection(d, "cuda:0")
G = torch.rand((N, N, N), device="cuda")
p.adjoint(G, N ** 3, None, 1, 0)
torch.cuda.synchronize()
# read the device counters through a tiny kernel exported by the experiment build
lib = ctypes.CDLL(_abi.LIB_PATH)
out = torch.zeros(2, dtype=torch.int64, device="cuda")
hip = ctypes.CDLL("libamdhip64.so")
fn = ctypes.c_void_p()
mod = None
# hipLaunchKernel on an extern "C" __global__ through the host stub symbol
stub = lib.tvam_exp_read
args = (ctypes.c_void_p * 1)(ctypes.cast(ctypes.pointer(ctypes.c_void_p(out.data_ptr())), ctypes.c_void_p))
rc = hip.hipLaunchKernel(ctypes.cast(stub, ctypes.c_void_p), ctypes.c_uint64(1 | (1 << 32)), ctypes.c_uint32(1),
                         ctypes.c_uint64(1 | (1 << 32)), ctypes.c_uint32(1), args, ctypes.c_size_t(0), None)
torch.cuda.synchronize()
lane, wave = out.tolist()
print(f"rc={rc} lane iterations {lane:.4e}, wave iterations {wave:.4e}, march-loop utilisation {lane / (64 * wave):.3f}")
